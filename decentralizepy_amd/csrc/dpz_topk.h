// Shared declarations of the top-k encoder (exact + sampled paths). See dpz_topk.hip.
#pragma once
#include "dpz_common.h"

namespace dpz {

// ------------------------------------------------------------------------------------------------
// Key source: how a key is formed from the caller's buffers (see DPZ_ACC_* in dpz_codec.h).
// first pass (rekey == 0): change = x - x0 (or x), then ACCUMULATE: acc += change (optionally
// stored), key = |acc|; ADD: key = |change + acc|.  After the first pass has stored acc
// (rekey == 1, ACCUMULATE), key = |acc|.
struct KeySrc {
  const float* x;
  const float* x0;
  float* acc;
  int mode;
  int rekey;
};

template <bool VEC>
__device__ __forceinline__ int load_keys4(const KeySrc& s, int64_t i0, int64_t n, bool store_acc,
                                          uint32_t key[4]) {
  float c[4];
  const int64_t rem = n - i0;
  const int cnt = rem >= 4 ? 4 : (rem > 0 ? (int)rem : 0);
  if (VEC && cnt == 4) {
    if (s.mode == DPZ_ACC_ACCUMULATE && s.rekey) {
      float4 q = *reinterpret_cast<const float4*>(s.acc + i0);
      c[0] = q.x; c[1] = q.y; c[2] = q.z; c[3] = q.w;
    } else {
      float4 a = *reinterpret_cast<const float4*>(s.x + i0);
      c[0] = a.x; c[1] = a.y; c[2] = a.z; c[3] = a.w;
      if (s.x0) {
        float4 b = *reinterpret_cast<const float4*>(s.x0 + i0);
        c[0] = a.x - b.x; c[1] = a.y - b.y; c[2] = a.z - b.z; c[3] = a.w - b.w;
      }
      if (s.mode != DPZ_ACC_NONE) {
        float4 q = *reinterpret_cast<const float4*>(s.acc + i0);
        float4 r;
        r.x = q.x + c[0]; r.y = q.y + c[1]; r.z = q.z + c[2]; r.w = q.w + c[3];
        if (s.mode == DPZ_ACC_ACCUMULATE && store_acc) *reinterpret_cast<float4*>(s.acc + i0) = r;
        c[0] = r.x; c[1] = r.y; c[2] = r.z; c[3] = r.w;
      }
    }
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (e < cnt) {
        const int64_t i = i0 + e;
        float v;
        if (s.mode == DPZ_ACC_ACCUMULATE && s.rekey) {
          v = s.acc[i];
        } else {
          v = s.x0 ? (s.x[i] - s.x0[i]) : s.x[i];
          if (s.mode != DPZ_ACC_NONE) {
            float r = s.acc[i] + v;
            if (s.mode == DPZ_ACC_ACCUMULATE && store_acc) s.acc[i] = r;
            v = r;
          }
        }
        c[e] = v;
      } else {
        c[e] = 0.0f;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) key[e] = key_of(c[e]);
  return cnt;
}

// Control block in the workspace (first 256 bytes).
struct TopkCtrl {
  // exact path
  uint32_t prefix;  // resolved key bits so far / final T
  uint32_t krem;    // elements still to take within the prefix / final #ties to take
  uint32_t status;  // sampled path: 0 ok, 1 miss -> exact fallback
  uint32_t nbound;  // sampled path: boundary entries appended
  uint32_t lo, hi, shift;  // sampled path key window and fine-bin shift
  uint32_t bstar, need;    // threshold bin, entries to take from it
  uint32_t T, icut;        // final threshold key / last selected index among key == T
  uint32_t pad[53];
};
static_assert(sizeof(TopkCtrl) == 256, "ctrl size");

// ---- sizes ---------------------------------------------------------------------------------
constexpr int EX_CHUNK = 8192;     // elements per block in the exact count/write passes
constexpr int EX_HIST_BLOCKS = 1024;
constexpr int SMP_N = 65536;       // samples
constexpr int SMP_CHUNK = 64;      // contiguous elements per sample chunk (one wave)
constexpr int SMP_NCHUNK = SMP_N / SMP_CHUNK;
constexpr int SMP_BLOCKS = 64;     // 16 chunks per block: 4 waves x 4 rounds
constexpr int CB_SHIFT = 20;       // coarse bins: key >> 20 (2048 bins, 8 per octave)
constexpr int CB = 2048;
constexpr int HB = 256;            // fine window bins (+1 "above window" bin)
constexpr int HBR = HB + 1;
#ifndef DPZ_WMAX
#define DPZ_WMAX 8192
#endif
#ifndef DPZ_WMIN_RANGE
#define DPZ_WMIN_RANGE 1024
#endif
#ifndef DPZ_FG
#define DPZ_FG 4
#endif
constexpr int W_MAX = DPZ_WMAX;    // wave segments (one wave streams one contiguous segment)
constexpr int FG = DPZ_FG;         // float4 groups of 256 elements a filter wave loads at once
constexpr int W_MIN_RANGE = DPZ_WMIN_RANGE;
constexpr int GH_COPIES = 16;      // window histogram copies (filter block b adds into copy b % 16)
constexpr int GH_STRIDE = 272;     // >= HBR, 16-aligned
constexpr int SEL_SEGS = 32;       // wave segments per select block (16 waves x 2)
constexpr int SEL_LCAP = 1024;     // boundary entries one select block stages in LDS
constexpr int NSUB = 16;           // boundary sub-lists (one atomic per select block each)
constexpr int SUBCAP = 256;        // entries per sub-list (more -> miss -> exact fallback)
constexpr int BCAP = NSUB * SUBCAP;  // boundary entries compact can hold (more -> miss)
constexpr int RANK_MAX = 1024;     // up to this many boundary entries: rank counting, else radix
constexpr int B_MAX = W_MAX / 4;   // filter blocks (4 wave segments each)
constexpr int STAGE = 128;         // per-wave LDS candidate staging (flushed in coalesced chunks)
constexpr uint32_t DENSE = 0xFFFFFFFFu;

struct FastGeom {
  int64_t W;      // wave segments
  int64_t B;      // filter blocks (4 waves each) = histogram rows
  int64_t R;      // elements per wave segment (multiple of 4)
  int64_t CAP;    // candidate capacity per wave segment
};

static inline FastGeom fast_geom(int64_t n) {
  FastGeom g;
  int64_t W = (n + W_MIN_RANGE - 1) / W_MIN_RANGE;
  if (W > W_MAX) W = W_MAX;
  if (W < 1) W = 1;
  int64_t R = (n + W - 1) / W;
  R = (R + 3) & ~int64_t(3);
  W = (n + R - 1) / R;
  int64_t cap = ((R / 4) + 63) & ~int64_t(63);
  if (cap < 64) cap = 64;
  if (cap > 1024) cap = 1024;
  g.W = W; g.B = (W + 3) / 4; g.R = R; g.CAP = cap;
  return g;
}

static inline size_t align256(size_t v) { return (v + 255) & ~size_t(255); }

struct WsLayout {
  size_t ctrl, chist, ex_hist, ex_gt, ex_eq, ex_off, ex_eqb;
  size_t f_ghist, f_segcnt, f_blkabove, f_blkoff, f_cidx, f_ckey, f_blcnt, f_blkey, f_blidx;
  size_t total;
  int64_t ex_nblk;
  FastGeom fg;
};

static inline WsLayout ws_layout(int64_t n) {
  WsLayout L;
  size_t o = 0;
  L.ex_nblk = (n + EX_CHUNK - 1) / EX_CHUNK;
  if (L.ex_nblk < 1) L.ex_nblk = 1;
  L.fg = fast_geom(n > 0 ? n : 1);
  L.ctrl = o; o += align256(sizeof(TopkCtrl));
  L.chist = o; o += align256(CB * 4);  // must be zero before the first sampled call (self-cleaning)
  L.ex_hist = o; o += align256(4096 * 4);
  L.ex_gt = o; o += align256(L.ex_nblk * 4);
  L.ex_eq = o; o += align256(L.ex_nblk * 4);
  L.ex_off = o; o += align256(L.ex_nblk * 4);
  L.ex_eqb = o; o += align256(L.ex_nblk * 4);
  L.f_ghist = o; o += align256(GH_COPIES * GH_STRIDE * 4);
  L.f_blcnt = o; o += align256(NSUB * 4);
  L.f_segcnt = o; o += align256(L.fg.W * 4);
  L.f_blkabove = o; o += align256(L.fg.B * 4);
  L.f_blkoff = o; o += align256(L.fg.B * 4);
  L.f_cidx = o; o += align256((size_t)L.fg.W * L.fg.CAP * 4);
  L.f_ckey = o; o += align256((size_t)L.fg.W * L.fg.CAP * 4);
  L.f_blkey = o; o += align256((size_t)BCAP * 4);
  L.f_blidx = o; o += align256((size_t)BCAP * 4);
  L.total = o;
  return L;
}

struct EncodeArgs {
  const float* x; const float* x0; float* acc; int acc_mode; const float* vals_src;
  int64_t n, k; int32_t* idx_out; float* val_out; int32_t* counter; char* ws;
  hipStream_t st;
};

// dpz_topk_exact.hip / dpz_topk_sampled.hip
int run_exact(const EncodeArgs& a, const WsLayout& L, int rekey, bool vec);
// phases: bit 0 = streaming pass (sample, filter), bit 1 = selection tail (select .. compact)
int run_sampled(const EncodeArgs& a, const WsLayout& L, bool vec, int phases = 3);
static inline bool use_sampled(int64_t n, int64_t k) {
  return n >= (1 << 18) && k >= 1 && k <= n / 16;
}

}  // namespace dpz
