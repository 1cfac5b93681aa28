// Shared declarations of the top-k encoder (exact + sampled paths). See dpz_topk.hip.
#pragma once
#include <cstdlib>

#include "dpz_common.h"
#include "dpz_replace.h"

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

// The raw loads of 4 consecutive elements (x, x0, acc as the mode needs), split from the key
// computation so a caller can keep them in flight while it does other work.
struct Raw4 {
  float4 a, b, q;
  int cnt;
};

// ACC = false: the caller guarantees s.mode == DPZ_ACC_NONE (no acc registers are held).
template <bool VEC, bool ACC = true>
__device__ __forceinline__ void load_raw4(const KeySrc& s, int64_t i0, int64_t n, Raw4& r) {
  const int64_t rem = n - i0;
  r.cnt = rem >= 4 ? 4 : (rem > 0 ? (int)rem : 0);
  const int mode = ACC ? s.mode : DPZ_ACC_NONE;
  const bool rekey = mode == DPZ_ACC_ACCUMULATE && s.rekey;
  if (VEC && r.cnt == 4) {
    if (rekey) {
      r.q = *reinterpret_cast<const float4*>(s.acc + i0);
    } else {
      r.a = *reinterpret_cast<const float4*>(s.x + i0);
      if (s.x0) r.b = *reinterpret_cast<const float4*>(s.x0 + i0);
      if (mode != DPZ_ACC_NONE) r.q = *reinterpret_cast<const float4*>(s.acc + i0);
    }
  } else {
    float a[4] = {0.f, 0.f, 0.f, 0.f}, b[4] = {0.f, 0.f, 0.f, 0.f}, q[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (e < r.cnt) {
        const int64_t i = i0 + e;
        if (rekey) {
          q[e] = s.acc[i];
        } else {
          a[e] = s.x[i];
          if (s.x0) b[e] = s.x0[i];
          if (mode != DPZ_ACC_NONE) q[e] = s.acc[i];
        }
      }
    }
    r.a = make_float4(a[0], a[1], a[2], a[3]);
    r.b = make_float4(b[0], b[1], b[2], b[3]);
    r.q = make_float4(q[0], q[1], q[2], q[3]);
  }
}

// Keys of the 4 elements of r (elements past the end get key 0); stores acc += change for the
// first pass of DPZ_ACC_ACCUMULATE when store_acc.  Returns the element count.
template <bool VEC, bool ACC = true>
__device__ __forceinline__ int finish_keys4(const KeySrc& s, int64_t i0, bool store_acc,
                                            const Raw4& r, uint32_t key[4]) {
  const int mode = ACC ? s.mode : DPZ_ACC_NONE;
  const float ra[4] = {r.a.x, r.a.y, r.a.z, r.a.w};
  const float rb[4] = {r.b.x, r.b.y, r.b.z, r.b.w};
  const float rq[4] = {r.q.x, r.q.y, r.q.z, r.q.w};
  float c[4];
  const bool rekey = mode == DPZ_ACC_ACCUMULATE && s.rekey;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (rekey) {
      c[e] = rq[e];
    } else {
      float v = s.x0 ? (ra[e] - rb[e]) : ra[e];
      if (mode != DPZ_ACC_NONE) v = rq[e] + v;
      c[e] = v;
    }
  }
  if (!rekey && mode == DPZ_ACC_ACCUMULATE && store_acc) {
    if (VEC && r.cnt == 4) {
      *reinterpret_cast<float4*>(s.acc + i0) = make_float4(c[0], c[1], c[2], c[3]);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (e < r.cnt) s.acc[i0 + e] = c[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) key[e] = e < r.cnt ? key_of(c[e]) : 0u;
  return r.cnt;
}

template <bool VEC>
__device__ __forceinline__ int load_keys4(const KeySrc& s, int64_t i0, int64_t n, bool store_acc,
                                          uint32_t key[4]) {
  Raw4 r;
  load_raw4<VEC>(s, i0, n, r);
  return finish_keys4<VEC>(s, i0, store_acc, r, key);
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
  uint32_t sticky;         // OR of every sampled call's final status since the caller cleared it
                           // (dpz_topk_sticky_status): misses of ASYNC calls never completed
  uint32_t val_h;          // sampled path: the call's value format (1 = fp16), for the exact
                           // re-run dpz_topk_complete makes after a miss
  // prior-round window (DPZ_TOPK_HINT): the exact threshold key of the last sampled call that
  // completed on this workspace and that call's signature (n, k, geometry, key source; never 0);
  // written by compact on success only
  uint32_t hint_T, hint_sig;
  uint32_t hinted;         // this call's filter took its window from hint_T (no sample launch)
  uint32_t pad[48];
};
static_assert(sizeof(TopkCtrl) == 256, "ctrl size");

// ---- sizes ---------------------------------------------------------------------------------
constexpr int EX_CHUNK = 8192;     // elements per block in the exact count/write passes
constexpr int EX_HIST_BLOCKS = 1024;
constexpr int SMP_N = 65536;       // samples
constexpr int SMP_CHUNK = 64;      // contiguous elements per sample chunk (one wave)
constexpr int SMP_NCHUNK = SMP_N / SMP_CHUNK;
constexpr int CB_SHIFT = 20;       // coarse bins: key >> 20 (2048 bins, 8 per octave)
constexpr int CB = 2048;
#ifndef DPZ_HB
#define DPZ_HB 1024
#endif
// fine window bins (+1 "above window" bin): 1024 keep the threshold bin at ~k/1000 entries even
// where the window is wide in count (C3: 25M wavelet coefficients, 256 bins overflowed the
// boundary list)
constexpr int HB = DPZ_HB;
constexpr int HBR = HB + 1;
static_assert(HB % 256 == 0 && HB <= 1024, "fine bins: multiple of 256, at most 1024");
#ifndef DPZ_WMAX
#define DPZ_WMAX 8192
#endif
#ifndef DPZ_WMIN_RANGE
#define DPZ_WMIN_RANGE 1024
#endif
#ifndef DPZ_FG
#define DPZ_FG 2
#endif
constexpr int W_MAX = DPZ_WMAX;    // wave segments (one wave streams one contiguous segment)
// Up to W_SMALL_N elements the filter runs at most W_SMALL segments: measured on MI355X with 3
// node codecs per GPU (bench default), C2 (11 M) 41.4 -> 38.3 us per step and 64 MiB 59.5 ->
// 54.5 us — a filter grid that leaves CU slots free lets the other streams' kernels run beside
// it — with the one-node step unchanged; at 25 M (C3, accumulation) and 67 M (C5) the full
// W_MAX measured faster (tools/diag/ab_bench.sh, workload_ab.sh).
#ifndef DPZ_WSMALL
#define DPZ_WSMALL 3072
#endif
constexpr int W_SMALL = DPZ_WSMALL;
constexpr int64_t W_SMALL_N = (1 << 24) + (1 << 22);
constexpr int FG = DPZ_FG;         // float4 groups of 256 elements a filter wave loads at once
#ifndef DPZ_FOCC
#define DPZ_FOCC 8
#endif
constexpr int FOCC = DPZ_FOCC;     // filter waves per SIMD the register budget is sized for
constexpr int W_MIN_RANGE = DPZ_WMIN_RANGE;
#ifndef DPZ_GH_COPIES
#define DPZ_GH_COPIES 8
#endif
// window histogram copies (filter block b adds into copy b % GH_COPIES): enough to spread the
// filter's end-of-block atomics over the 1024 bins, few enough that every select block can
// sum them (each select block reads GH_COPIES x 4 KiB)
constexpr int GH_COPIES = DPZ_GH_COPIES;
constexpr int GH_STRIDE = HB + 16; // >= HBR, 16-aligned
constexpr int SEL_SEGS = 32;       // wave segments per select block (16 waves x 2)
constexpr int SEL_LCAP = 1024;     // boundary entries one select block stages in LDS
constexpr int NSUB = 16;           // boundary sub-lists (one atomic per select block each)
constexpr int SUBCAP = 256;        // entries per sub-list (more -> miss -> exact fallback)
constexpr int BCAP = NSUB * SUBCAP;  // boundary entries compact can hold (more -> miss)
constexpr int RANK_MAX = 1024;     // up to this many boundary entries: rank counting, else radix
constexpr int B_MAX = W_MAX / 4;   // filter blocks (4 wave segments each)
constexpr int STAGE = 256;         // per-wave LDS candidate staging (flushed in coalesced chunks;
                                   // >= one group's candidates at large alpha)
constexpr uint32_t DENSE = 0xFFFFFFFFu;

struct FastGeom {
  int64_t W;      // wave segments
  int64_t B;      // filter blocks (4 waves each) = histogram rows
  int64_t R;      // elements per wave segment (multiple of 4)
  int64_t CAP;    // candidate capacity per wave segment
};

// k > 0: the candidate capacity per segment grows with alpha = k / n (the key window holds
// about alpha + a few percent of the elements; a segment over capacity turns DENSE, still exact)
// shared: several node codecs share the GPU (a batch enqueue on several streams): up to
// W_SMALL_N elements the filter grid is capped at W_SMALL segments so the other streams' kernels
// find free CU slots; a lone codec (one stream) takes the full W_MAX grid, the faster one alone
// (C2 filter 18.8 vs 20.6 us).
static inline FastGeom fast_geom(int64_t n, int64_t k = 0, bool shared = false) {
  FastGeom g;
  int64_t W = (n + W_MIN_RANGE - 1) / W_MIN_RANGE;
  // DPZ_WLONE=N caps a lone codec's grid at N segments (diagnostic build, A/B)
  const int64_t wlone = DPZ_KNOB_INT(WLONE, 0);
  const int64_t wmax = (shared && n <= W_SMALL_N)
                           ? W_SMALL
                           : ((wlone > 0 && wlone < W_MAX) ? wlone : W_MAX);
  if (W > wmax) W = wmax;
  if (W < 1) W = 1;
  int64_t R = (n + W - 1) / W;
  // a multiple of 32: every 32-element word of a selection mask / sliced counter belongs to one
  // wave segment (dpz_topk_encode_sliced), and of 4 for the float4 streams
  R = (R + 31) & ~int64_t(31);
  W = (n + R - 1) / R;
  int64_t cap = ((R / 4) + 63) & ~int64_t(63);
  if (k > n / 16) {
    const double frac = 1.25 * (double)k / (double)n + 0.05;
    cap = ((int64_t)(frac * (double)R) + 63) & ~int64_t(63);
    if (cap > ((R + 63) & ~int64_t(63))) cap = (R + 63) & ~int64_t(63);
  }
  if (cap < 64) cap = 64;
  if (k <= n / 16 && cap > 1024) cap = 1024;
  g.W = W; g.B = (W + 3) / 4; g.R = R; g.CAP = cap;
  return g;
}

static inline size_t align256(size_t v) { return (v + 255) & ~size_t(255); }

struct WsLayout {
  size_t ctrl, chist, ex_hist, ex_gt, ex_eq, ex_off, ex_eqb;
  size_t f_ghist, f_segcnt, f_blkabove, f_blkoff, f_cidx, f_ckey, f_cval, f_blcnt, f_blkey, f_blidx;
  size_t total;
  int64_t ex_nblk;
  FastGeom fg;
};

static inline WsLayout ws_layout(int64_t n, int64_t k = 0, bool shared = false) {
  WsLayout L;
  size_t o = 0;
  L.ex_nblk = (n + EX_CHUNK - 1) / EX_CHUNK;
  if (L.ex_nblk < 1) L.ex_nblk = 1;
  L.fg = fast_geom(n > 0 ? n : 1, k, shared);
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
  L.f_cval = o; o += align256((size_t)L.fg.W * L.fg.CAP * 4);
  L.f_blkey = o; o += align256((size_t)BCAP * 4);
  L.f_blidx = o; o += align256((size_t)BCAP * 4);
  L.total = o;
  return L;
}

// Workspace bytes a caller must provide: enough for either grid (the flags choose per call).
static inline size_t ws_bytes_needed(int64_t n, int64_t k) {
  const size_t a = ws_layout(n, k, false).total, b = ws_layout(n, k, true).total;
  return a > b ? a : b;
}

struct EncodeArgs {
  const float* x; const float* x0; float* acc; int acc_mode; const float* vals_src;
  int64_t n, k; int32_t* idx_out; float* val_out; int32_t* counter; char* ws;
  hipStream_t st;
  const ReplaceJob* job;  // co-scheduled replace decode (sampled path only), or nullptr
  int32_t* status_out;    // sampled path, ASYNC: compact's block 0 also writes the call's final
                          // status word here (device), or nullptr
  bool shared;            // DPZ_TOPK_SHARED: the filter grid for several codecs per GPU
  int val_h;              // DPZ_TOPK_VAL_FP16: val_out holds fp16 values (RNE)
  const FoldBase* fbase;  // dpz_topk_encode_foldbase: the pipelined filter also writes
  float* base_out;        // base_out[j] = fbase->of(x[j]) (sampled path, fused_foldbase_ok)
  // dpz_topk_encode_sliced: the side effects in coalesced form — selmask (ceil(n/32) words, every
  // word written: bit = selected) instead of the rewind, planes (the counter as 32 bit planes of
  // ceil(n/32) words) += 1 instead of counter[idx] += 1; counter and the rewind are then unused
  uint32_t* selmask;
  uint32_t* planes;
  // DPZ_TOPK_HINT: this call's signature when the filter may take its key window from the
  // previous sampled call's exact threshold (TopkCtrl::hint_T), else 0 (the sample launch runs)
  uint32_t hint_sig;
  bool keep_x;            // DPZ_TOPK_KEEP_X: x streamed with the default cache policy
};
// Signature of a sampled call's geometry and key source: a prior-round window is only taken from
// a call with the same one (the same workspace layout, so its window histogram copies are zero)
static inline uint32_t hint_signature(int64_t n, int64_t k, bool shared, int acc_mode, bool x0) {
  uint64_t h = 1469598103934665603ull;
  const uint64_t v[5] = {(uint64_t)n, (uint64_t)k, shared ? 1ull : 0ull, (uint64_t)acc_mode,
                         x0 ? 1ull : 0ull};
  for (int i = 0; i < 5; ++i) h = (h ^ v[i]) * 1099511628211ull;
  return (uint32_t)(h ^ (h >> 32)) | 1u;
}
// The key window around a prior threshold key T: [T (1 - 1/16), T (1 + 1/16)] — a drift of the
// k-th largest |change| of up to 6.25 % between rounds still brackets it (validated by select's
// counts; a miss re-runs the sampled path with its sample launch).  Measured on MI355X (64 MiB,
// 1 %): +-1/8 put ~19 boundary entries on each of the 16 sub-lists, past the 16 compact loads
// speculatively (a dependent load more: compact 13.5 -> 15.0 us, select 6.8 -> 7.5 us)
#ifndef DPZ_HINT_DELTA
#define DPZ_HINT_DELTA 0.0625f
#endif
constexpr float HINT_LO = 1.0f - DPZ_HINT_DELTA, HINT_HI = 1.0f + DPZ_HINT_DELTA;
// the sampled compact builds a segment's mask words in LDS: segments of at most this many elements
constexpr int64_t SL_RMAX = 8192;
static inline int64_t mask_words(int64_t n) { return (n + 31) >> 5; }
// sliced side effects from idx_out (the exact path, a sampled miss, segments over SL_RMAX):
// selmask zeroed, bits set from idx_out[0..k), planes += selmask (dpz_topk.hip)
// guard (may be NULL): a device status word; the planes are left alone when it is nonzero (a
// sampled call that missed: its output is void and the caller re-runs the encode exactly)
int sliced_from_idx(const EncodeArgs& a, const uint32_t* guard = nullptr);
// the fold base can ride on the pipelined filter: aligned, no accumulation, x0 given
bool fused_foldbase_ok(const EncodeArgs& a, bool vec);
// base_out[j] = fb.of(x[j]) as its own launch (dpz_fold.hip)
int launch_fold_base(const float* x, int64_t n, const FoldBase& fb, float* out, hipStream_t st);

// dpz_topk_exact.hip / dpz_topk_sampled.hip
// keep_ties: select every key >= T (the k-th largest key), no zero keys when T == 0, writing at
// most cap entries; the selected count is left in TopkCtrl.nbound
int run_exact(const EncodeArgs& a, const WsLayout& L, int rekey, bool vec, int keep_ties = 0,
              int64_t cap = 0);
// phases: bit 0 = streaming pass (sample, filter), bit 1 = selection tail (select .. compact)
int run_sampled(const EncodeArgs& a, const WsLayout& L, bool vec, int phases = 3);
// dpz_topk_encode with the final sampled-path status word also written to status_out (device)
// on the stream, as the call's last write: no separate copy (dpz_topk_encode_batch)
int topk_encode_status(const float* x, const float* x0, float* acc, int acc_mode,
                       const float* vals_src, int64_t n, int64_t k, int32_t* idx_out,
                       float* val_out, int32_t* counter, void* ws, size_t ws_bytes,
                       hipStream_t st, int32_t* status_out, bool shared = false,
                       bool val_fp16 = false, bool hint = false);
// dpz_topk_encode_nodes (dpz_topk_sampled.hip): m nodes' encodes, one launch per phase
int topk_encode_nodes(int m, const void* table, int64_t n, int64_t k, size_t ws_bytes, int flags,
                      hipStream_t st);
static inline bool use_sampled(int64_t n, int64_t k) {
  return n >= (1 << 18) && k >= 1 && k <= n / 2;
}

}  // namespace dpz
