// Top-k magnitude encode for the decentralizepy Sharing plugins (PartialModel / Wavelet / JWINS).
//
// Replaces (reference sacs-epfl/decentralizepy, src/decentralizepy/):
//   sharing/PartialModel.py:164-186  extract_top_gradients: |change|, torch.topk, torch.sort(index)
//   sharing/PartialModel.py:205-246  counter[idx] += 1, rewind_accumulation(idx), x[idx]
//   sharing/PartialModel.py:305-331  _pre_step change / accumulation (fused into the first pass)
//   sharing/JWINS/Wavelet.py:142-197 apply_wavelet + the same bookkeeping on coefficients
//
// Selection rule: the k largest uint32 keys (|change| bits, sign cleared, NaN canonical), ties at
// the k-th key broken by lowest index; output in ascending index order (so no sort is needed:
// compaction preserves index order).
//
// Two device paths:
//  * EXACT  — three radix histogram passes (10/11/10 bits) resolve the k-th key T and the number
//             of ties to take, then a count pass, a 1-block scan and an ordered-compaction pass.
//             Works for every n, k (also k = n, heavy ties, NaN).  ~5 reads of the key stream.
//  * SAMPLED (k <= n/16, n >= 2^18) — one read of the inputs:
//      sample  : 1 block estimates a key window [lo, hi) around the k-th key from 16384 samples
//      filter  : one pass over x/x0/acc; keys >= lo are appended, in index order, to a per-block
//                candidate list (idx,key,val); a 256-bin histogram of the window per block
//      selectA : column-sum of the per-block histograms
//      selectB : locate the threshold bin b*; per-segment count above b*; gather bin-b* entries
//      selectC : 1 block sorts the boundary entries -> exact T, tie cut, per-segment offsets
//      compact : ordered write of idx/val + counter / rewind side effects
//    Any miss (window did not bracket the k-th key, boundary overflow) sets ctrl->status; the
//    compact kernel then writes nothing and the host re-runs the EXACT path with keys re-derived
//    from the post-filter state ("rekey").  A block whose candidates overflow its list is marked
//    dense and re-reads its own input range in selectB / compact instead (still exact).
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
constexpr int SMP_N = 16384;       // samples
constexpr int SMP_CHUNK = 64;      // contiguous elements per sample chunk
constexpr int SMP_CB_SHIFT = 18;   // coarse sample bins: key >> 18 (8192 bins, 32 per octave)
constexpr int SMP_CB = 8192;
constexpr int HB = 256;            // fine window bins (+1 "above window" bin)
constexpr int HBR = HB + 1;
constexpr int F_MAX_BLOCKS = 2048;
constexpr int F_MIN_RANGE = 4096;
constexpr int BCAP = 8192;         // boundary entries sortable by selectC
constexpr uint32_t DENSE = 0xFFFFFFFFu;

struct FastGeom {
  int64_t G;      // filter blocks / segments
  int64_t R;      // elements per segment (multiple of 4)
  int64_t CAP;    // candidate capacity per segment
};

static inline FastGeom fast_geom(int64_t n) {
  FastGeom g;
  int64_t G = (n + F_MIN_RANGE - 1) / F_MIN_RANGE;
  if (G > F_MAX_BLOCKS) G = F_MAX_BLOCKS;
  if (G < 1) G = 1;
  int64_t R = (n + G - 1) / G;
  R = (R + 3) & ~int64_t(3);
  G = (n + R - 1) / R;
  int64_t cap = ((R / 4) + 63) & ~int64_t(63);
  if (cap < 256) cap = 256;
  if (cap > 2048) cap = 2048;
  g.G = G; g.R = R; g.CAP = cap;
  return g;
}

static inline size_t align256(size_t v) { return (v + 255) & ~size_t(255); }

struct WsLayout {
  size_t ctrl, ex_hist, ex_gt, ex_eq, ex_off, ex_eqb;
  size_t f_ghist, f_rows, f_segcnt, f_segabove, f_segoff, f_cidx, f_ckey, f_cval, f_bkey, f_bidx;
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
  L.ex_hist = o; o += align256(4096 * 4);
  L.ex_gt = o; o += align256(L.ex_nblk * 4);
  L.ex_eq = o; o += align256(L.ex_nblk * 4);
  L.ex_off = o; o += align256(L.ex_nblk * 4);
  L.ex_eqb = o; o += align256(L.ex_nblk * 4);
  L.f_ghist = o; o += align256(512 * 4);
  L.f_rows = o; o += align256((size_t)L.fg.G * HBR * 4);
  L.f_segcnt = o; o += align256(L.fg.G * 4);
  L.f_segabove = o; o += align256(L.fg.G * 4);
  L.f_segoff = o; o += align256(L.fg.G * 4);
  L.f_cidx = o; o += align256((size_t)L.fg.G * L.fg.CAP * 4);
  L.f_ckey = o; o += align256((size_t)L.fg.G * L.fg.CAP * 4);
  L.f_cval = o; o += align256((size_t)L.fg.G * L.fg.CAP * 4);
  L.f_bkey = o; o += align256(BCAP * 4);
  L.f_bidx = o; o += align256(BCAP * 4);
  L.total = o;
  return L;
}

// ================================================================================================
// EXACT path
// ================================================================================================
template <bool VEC, int P>
__global__ void __launch_bounds__(256) exact_hist_kernel(KeySrc s, int64_t n, const TopkCtrl* ctrl,
                                                         uint32_t* ghist, int store_acc) {
  constexpr int NB = (P == 1) ? 2048 : 1024;
  __shared__ uint32_t h[NB];
  for (int b = threadIdx.x; b < NB; b += 256) h[b] = 0;
  __syncthreads();
  const uint32_t pfx = (P == 0) ? 0u : ctrl->prefix;
  const int64_t ngroups = (n + 3) >> 2;
  for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < ngroups;
       g += (int64_t)gridDim.x * 256) {
    uint32_t key[4];
    const int cnt = load_keys4<VEC>(s, g * 4, n, store_acc != 0, key);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (e < cnt) {
        const uint32_t kk = key[e];
        if (P == 0) {
          atomicAdd(&h[kk >> 21], 1u);
        } else if (P == 1) {
          if ((kk >> 21) == (pfx >> 21)) atomicAdd(&h[(kk >> 10) & 2047u], 1u);
        } else {
          if ((kk >> 10) == (pfx >> 10)) atomicAdd(&h[kk & 1023u], 1u);
        }
      }
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < NB; b += 256) {
    const uint32_t v = h[b];
    if (v) atomicAdd(&ghist[b], v);
  }
}

// One block of 1024 threads: pick the digit holding the krem-th largest key.
template <int P>
__global__ void __launch_bounds__(1024) exact_resolve_kernel(TopkCtrl* ctrl, const uint32_t* ghist,
                                                             uint32_t k) {
  constexpr int NB = (P == 1) ? 2048 : 1024;
  constexpr int SH = (P == 0) ? 21 : (P == 1 ? 10 : 0);
  constexpr int PER = NB / 1024;
  __shared__ uint32_t wsum[16];
  const uint32_t krem = (P == 0) ? k : ctrl->krem;
  const uint32_t pfx = (P == 0) ? 0u : ctrl->prefix;
  // thread t owns descending positions j = t*PER .. t*PER+PER-1, bin = NB-1-j
  uint32_t hv[PER];
  uint32_t local = 0;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    hv[q] = ghist[NB - 1 - (threadIdx.x * PER + q)];
    local += hv[q];
  }
  uint32_t tot;
  uint32_t before = block_excl_scan(local, wsum, &tot);
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    if (before < krem && krem <= before + hv[q]) {
      const uint32_t d = NB - 1 - (threadIdx.x * PER + q);
      ctrl->prefix = pfx | (d << SH);
      ctrl->krem = krem - before;
    }
    before += hv[q];
  }
}

template <bool VEC>
__global__ void __launch_bounds__(256) exact_count_kernel(KeySrc s, int64_t n, const TopkCtrl* ctrl,
                                                          uint32_t* blk_gt, uint32_t* blk_eq) {
  __shared__ uint32_t wsum[16];
  const uint32_t T = ctrl->prefix;
  const int64_t lo = (int64_t)blockIdx.x * EX_CHUNK;
  uint32_t gt = 0, eq = 0;
  for (int r = 0; r < EX_CHUNK / 1024; ++r) {
    const int64_t i0 = lo + r * 1024 + threadIdx.x * 4;
    if (i0 >= n) break;
    uint32_t key[4];
    const int cnt = load_keys4<VEC>(s, i0, n, false, key);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (e < cnt) {
        gt += key[e] > T;
        eq += key[e] == T;
      }
    }
  }
  uint32_t tg, te;
  block_excl_scan(gt, wsum, &tg);
  block_excl_scan(eq, wsum, &te);
  if (threadIdx.x == 0) {
    blk_gt[blockIdx.x] = tg;
    blk_eq[blockIdx.x] = te;
  }
}

// One block of 1024 threads: per-block output offsets and tie allotments (in index order).
__global__ void __launch_bounds__(1024) exact_scan_kernel(const TopkCtrl* ctrl, int64_t nblk,
                                                          const uint32_t* blk_gt,
                                                          const uint32_t* blk_eq, uint32_t* blk_off,
                                                          uint32_t* blk_eqb) {
  __shared__ uint64_t wsum[16];
  const uint64_t ties = ctrl->krem;
  uint64_t carry_eq = 0, carry_off = 0;
  for (int64_t base = 0; base < nblk; base += 1024) {
    const int64_t b = base + threadIdx.x;
    const uint64_t gt = b < nblk ? blk_gt[b] : 0;
    const uint64_t eq = b < nblk ? blk_eq[b] : 0;
    uint64_t te;
    const uint64_t eqb = block_excl_scan64(eq, wsum, &te) + carry_eq;
    uint64_t take = 0;
    if (ties > eqb) take = (ties - eqb) < eq ? (ties - eqb) : eq;
    uint64_t ts;
    const uint64_t off = block_excl_scan64(gt + take, wsum, &ts) + carry_off;
    if (b < nblk) {
      blk_off[b] = (uint32_t)off;
      blk_eqb[b] = (uint32_t)(eqb < ties ? eqb : ties);
    }
    carry_eq += te;
    carry_off += ts;
  }
}

template <bool VEC>
__global__ void __launch_bounds__(256) exact_write_kernel(KeySrc s, int64_t n, const TopkCtrl* ctrl,
                                                          const uint32_t* blk_off,
                                                          const uint32_t* blk_eqb,
                                                          const float* vals_src, int32_t* idx_out,
                                                          float* val_out, int32_t* counter,
                                                          float* rewind, int64_t k) {
  __shared__ uint32_t wsum[16];
  const uint32_t T = ctrl->prefix;
  const uint32_t ties = ctrl->krem;
  const uint32_t off0 = blk_off[blockIdx.x];
  const uint32_t eqb = blk_eqb[blockIdx.x];
  const uint32_t quota = ties > eqb ? ties - eqb : 0u;
  const int64_t lo = (int64_t)blockIdx.x * EX_CHUNK;
  uint32_t gt_run = 0, eq_run = 0;
  for (int r = 0; r < EX_CHUNK / 1024; ++r) {
    const int64_t i0 = lo + r * 1024 + threadIdx.x * 4;
    if (lo + r * 1024 >= n) break;  // uniform
    uint32_t key[4];
    const int cnt = load_keys4<VEC>(s, i0, n, false, key);
    uint32_t ng = 0, ne = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (e < cnt) {
        ng += key[e] > T;
        ne += key[e] == T;
      }
    }
    uint32_t tot;
    const uint32_t ex = block_excl_scan((ne << 16) | ng, wsum, &tot);
    uint32_t g = gt_run + (ex & 0xFFFFu);
    uint32_t q = eq_run + (ex >> 16);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (e < cnt) {
        bool sel = false;
        uint32_t pos = 0;
        if (key[e] > T) {
          sel = true;
          pos = off0 + g + (q < quota ? q : quota);
          ++g;
        } else if (key[e] == T) {
          if (q < quota) {
            sel = true;
            pos = off0 + g + q;
          }
          ++q;
        }
        if (sel && pos < (uint64_t)k) {
          const int64_t i = i0 + e;
          idx_out[pos] = (int32_t)i;
          val_out[pos] = vals_src[i];
          if (counter) counter[i] += 1;
          if (rewind) rewind[i] = 0.0f;
        }
      }
    }
    gt_run += tot & 0xFFFFu;
    eq_run += tot >> 16;
  }
}

// ================================================================================================
// SAMPLED path
// ================================================================================================
__device__ __forceinline__ int64_t sample_chunk_start(int c, int64_t n) {
  return (int64_t)(((__int128)c * (n - SMP_CHUNK)) / (SMP_N / SMP_CHUNK - 1));
}

// One block of 1024 threads.
__global__ void __launch_bounds__(1024) fast_sample_kernel(KeySrc s, int64_t n, int64_t k,
                                                           TopkCtrl* ctrl, uint32_t* ghist) {
  __shared__ uint32_t h[SMP_CB];
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t res[2];
  for (int b = threadIdx.x; b < SMP_CB; b += 1024) h[b] = 0;
  if (threadIdx.x < 512) ghist[threadIdx.x] = 0;
  if (threadIdx.x == 0) { res[0] = 0; res[1] = SMP_CB; }
  __syncthreads();
#pragma unroll 4
  for (int r = 0; r < SMP_N / 1024; ++r) {
    const int j = threadIdx.x + r * 1024;
    const int64_t i = sample_chunk_start(j / SMP_CHUNK, n) + (j % SMP_CHUNK);
    float v;
    if (s.mode == DPZ_ACC_ACCUMULATE && s.rekey) {
      v = s.acc[i];
    } else {
      v = s.x0 ? (s.x[i] - s.x0[i]) : s.x[i];
      if (s.mode != DPZ_ACC_NONE) v = s.acc[i] + v;
    }
    atomicAdd(&h[key_of(v) >> SMP_CB_SHIFT], 1u);
  }
  __syncthreads();
  // ranks (1-based, descending) bracketing the k-th key with a 6-sigma + 16 margin
  const double r_est = (double)k * SMP_N / (double)n;
  const double sd = sqrt(r_est);
  const double rlo_d = ceil(r_est + 6.0 * sd + 16.0);
  const double rhi_d = floor(r_est - 6.0 * sd - 16.0);
  const uint32_t r_lo = rlo_d > SMP_N ? (uint32_t)SMP_N + 1 : (uint32_t)rlo_d;
  const uint32_t r_hi = rhi_d < 1.0 ? 0u : (uint32_t)rhi_d;
  // thread t owns descending bins 8t..8t+7 (bin = SMP_CB-1-j)
  uint32_t hv[8];
  uint32_t local = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    hv[q] = h[SMP_CB - 1 - (threadIdx.x * 8 + q)];
    local += hv[q];
  }
  uint32_t tot;
  uint32_t before = block_excl_scan(local, wsum, &tot);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint32_t bin = SMP_CB - 1 - (threadIdx.x * 8 + q);
    if (r_hi >= 1 && before < r_hi && r_hi <= before + hv[q]) res[1] = bin;  // bin of rank r_hi
    if (r_lo <= (uint32_t)SMP_N && before < r_lo && r_lo <= before + hv[q]) res[0] = bin + 1;
    before += hv[q];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    // lo: lower edge of the bin holding rank r_lo (0 if the sample has fewer than r_lo keys)
    const uint32_t lo = (r_lo <= (uint32_t)SMP_N) ? ((res[0] - 1) << SMP_CB_SHIFT) : 0u;
    // hi: upper edge of the bin holding rank r_hi (2^31: no key reaches it)
    const uint64_t hi64 = (r_hi >= 1) ? ((uint64_t)(res[1] + 1) << SMP_CB_SHIFT) : (1ull << 31);
    const uint32_t hi = (uint32_t)(hi64 > (1ull << 31) ? (1ull << 31) : hi64);
    uint32_t width = hi - lo;
    uint32_t shift = 0;
    while (((uint64_t)width + (1ull << shift) - 1) >> shift > (uint64_t)HB) ++shift;
    ctrl->lo = lo;
    ctrl->hi = hi;
    ctrl->shift = shift;
    ctrl->status = 0;
    ctrl->nbound = 0;
  }
}

__device__ __forceinline__ uint32_t fine_bin(uint32_t key, uint32_t lo, uint32_t hi,
                                             uint32_t shift) {
  return key >= hi ? (uint32_t)HB : ((key - lo) >> shift);
}

// G blocks x 256 threads: block b owns [b*R, min(n, (b+1)*R)).
template <bool VEC>
__global__ void __launch_bounds__(256) fast_filter_kernel(KeySrc s, int64_t n, int64_t R,
                                                          int64_t CAP, const TopkCtrl* ctrl,
                                                          const float* vals_src, int vals_is_x,
                                                          uint32_t* rows, uint32_t* segcnt,
                                                          uint32_t* cidx, uint32_t* ckey,
                                                          float* cval) {
  __shared__ uint32_t h[HBR];
  __shared__ uint32_t wsum[16];
  for (int b = threadIdx.x; b < HBR; b += 256) h[b] = 0;
  const uint32_t lo = ctrl->lo, hi = ctrl->hi, shift = ctrl->shift;
  const int64_t seg = blockIdx.x;
  const int64_t beg = seg * R;
  const int64_t end = (beg + R < n) ? beg + R : n;
  uint32_t* my_idx = cidx + seg * CAP;
  uint32_t* my_key = ckey + seg * CAP;
  float* my_val = cval + seg * CAP;
  uint32_t cnt = 0;
  bool dense = false;
  const bool store_acc = (s.mode == DPZ_ACC_ACCUMULATE) && !s.rekey;
  __syncthreads();
  for (int64_t base = beg; base < end; base += 2048) {
    // two groups of 4 per thread: [base + 4t, +4) and [base + 1024 + 4t, +4)
    uint32_t ka[4], kb[4];
    const int64_t ia = base + threadIdx.x * 4;
    const int64_t ib = ia + 1024;
    const int ca = ia < end ? load_keys4<VEC>(s, ia, end, store_acc, ka) : 0;
    const int cb = ib < end ? load_keys4<VEC>(s, ib, end, store_acc, kb) : 0;
    float va[4], vb[4];
    uint32_t na = 0, nb = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const bool sa = e < ca && ka[e] >= lo;
      const bool sb = e < cb && kb[e] >= lo;
      if (sa) atomicAdd(&h[fine_bin(ka[e], lo, hi, shift)], 1u);
      if (sb) atomicAdd(&h[fine_bin(kb[e], lo, hi, shift)], 1u);
      na += sa;
      nb += sb;
    }
    uint32_t tot;
    const uint32_t ex = block_excl_scan((nb << 16) | na, wsum, &tot);
    const uint32_t tot_a = tot & 0xFFFFu, tot_b = tot >> 16;
    if (!dense && cnt + tot_a + tot_b <= (uint32_t)CAP) {
      uint32_t pa = cnt + (ex & 0xFFFFu);
      uint32_t pb = cnt + tot_a + (ex >> 16);
      if (na | nb) {
        if (vals_is_x && VEC) {
          // values are x itself: reuse the vector load path
          if (ca == 4) { float4 t = *reinterpret_cast<const float4*>(vals_src + ia); va[0]=t.x; va[1]=t.y; va[2]=t.z; va[3]=t.w; }
          if (cb == 4) { float4 t = *reinterpret_cast<const float4*>(vals_src + ib); vb[0]=t.x; vb[1]=t.y; vb[2]=t.z; vb[3]=t.w; }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (e < ca && ka[e] >= lo) {
            my_idx[pa] = (uint32_t)(ia + e);
            my_key[pa] = ka[e];
            my_val[pa] = (vals_is_x && VEC && ca == 4) ? va[e] : vals_src[ia + e];
            ++pa;
          }
          if (e < cb && kb[e] >= lo) {
            my_idx[pb] = (uint32_t)(ib + e);
            my_key[pb] = kb[e];
            my_val[pb] = (vals_is_x && VEC && cb == 4) ? vb[e] : vals_src[ib + e];
            ++pb;
          }
        }
      }
    } else {
      dense = true;
    }
    cnt += tot_a + tot_b;
  }
  __syncthreads();
  uint32_t* row = rows + seg * HBR;
  for (int b = threadIdx.x; b < HBR; b += 256) row[b] = h[b];
  if (threadIdx.x == 0) segcnt[seg] = dense ? DENSE : cnt;
}

// 64 blocks x 256: column sums of the per-segment histograms.
__global__ void __launch_bounds__(256) fast_selectA_kernel(const uint32_t* rows, int64_t G,
                                                           uint32_t* ghist) {
  const int64_t per = (G + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = blockIdx.x * per;
  const int64_t r1 = (r0 + per < G) ? r0 + per : G;
  for (int b = threadIdx.x; b < HBR; b += 256) {
    uint32_t sum = 0;
    for (int64_t r = r0; r < r1; ++r) sum += rows[r * HBR + b];
    if (sum) atomicAdd(&ghist[b], sum);
  }
}

// Threshold bin from the global window histogram (all threads get the same answer).
// Returns false when the window does not bracket the k-th key.
__device__ __forceinline__ bool resolve_bstar(const uint32_t* ghist, uint32_t k, uint32_t* wsum,
                                              uint32_t* sh_res, uint32_t* bstar, uint32_t* need) {
  // 256 threads: thread t owns descending fine bin HB-1-t; "above" bin counted first.
  const uint32_t above = ghist[HB];
  const uint32_t hv = threadIdx.x < HB ? ghist[HB - 1 - threadIdx.x] : 0u;
  uint32_t tot;
  const uint32_t before = block_excl_scan(hv, wsum, &tot) + above;
  if (threadIdx.x == 0) { sh_res[0] = 0xFFFFFFFFu; sh_res[1] = 0; }
  __syncthreads();
  if (threadIdx.x < HB && before < k && k <= before + hv) {
    sh_res[0] = HB - 1 - threadIdx.x;
    sh_res[1] = k - before;
  }
  __syncthreads();
  const bool ok = (above < k) && (above + tot >= k) && sh_res[0] != 0xFFFFFFFFu;
  *bstar = sh_res[0];
  *need = sh_res[1];
  return ok;
}

template <bool VEC>
__global__ void __launch_bounds__(256) fast_selectB_kernel(KeySrc s, int64_t n, int64_t k, int64_t R,
                                                           int64_t CAP, TopkCtrl* ctrl,
                                                           const uint32_t* ghist,
                                                           const uint32_t* segcnt,
                                                           const uint32_t* cidx,
                                                           const uint32_t* ckey,
                                                           uint32_t* segabove, uint32_t* bkey,
                                                           uint32_t* bidx) {
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t sh_res[2];
  uint32_t bstar, need;
  const bool ok = resolve_bstar(ghist, (uint32_t)k, wsum, sh_res, &bstar, &need);
  if (!ok) {
    if (blockIdx.x == 0 && threadIdx.x == 0) ctrl->status = 1;
    return;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    ctrl->bstar = bstar;
    ctrl->need = need;
  }
  const uint32_t lo = ctrl->lo, hi = ctrl->hi, shift = ctrl->shift;
  const int64_t seg = blockIdx.x;
  const uint32_t cnt = segcnt[seg];
  uint32_t above = 0;
  if (cnt != DENSE) {
    for (uint32_t j = threadIdx.x; j < cnt; j += 256) {
      const uint32_t key = ckey[seg * CAP + j];
      const uint32_t b = fine_bin(key, lo, hi, shift);
      if (b > bstar) {
        ++above;
      } else if (b == bstar) {
        const uint32_t p = atomicAdd(&ctrl->nbound, 1u);
        if (p < BCAP) {
          bkey[p] = key;
          bidx[p] = cidx[seg * CAP + j];
        }
      }
    }
  } else {
    const int64_t beg = seg * R;
    const int64_t end = (beg + R < n) ? beg + R : n;
    for (int64_t i0 = beg + threadIdx.x * 4; i0 < end; i0 += 1024) {
      uint32_t key[4];
      const int c = load_keys4<VEC>(s, i0, end, false, key);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (e < c && key[e] >= lo) {
          const uint32_t b = fine_bin(key[e], lo, hi, shift);
          if (b > bstar) {
            ++above;
          } else if (b == bstar) {
            const uint32_t p = atomicAdd(&ctrl->nbound, 1u);
            if (p < BCAP) {
              bkey[p] = key[e];
              bidx[p] = (uint32_t)(i0 + e);
            }
          }
        }
      }
    }
  }
  uint32_t tot;
  block_excl_scan(above, wsum, &tot);
  if (threadIdx.x == 0) segabove[seg] = tot;
}

// One block of 1024 threads: exact order inside the threshold bin + per-segment offsets.
__global__ void __launch_bounds__(1024) fast_selectC_kernel(int64_t k, int64_t G, int64_t R,
                                                            TopkCtrl* ctrl, const uint32_t* bkey,
                                                            const uint32_t* bidx,
                                                            const uint32_t* segabove,
                                                            uint32_t* segoff) {
  __shared__ uint64_t sk[BCAP];
  __shared__ uint32_t segsel[F_MAX_BLOCKS];
  __shared__ uint32_t wsum[16];
  if (ctrl->status) return;
  const uint32_t nb = ctrl->nbound;
  const uint32_t need = ctrl->need;
  if (nb > BCAP || need == 0 || need > nb) {
    if (threadIdx.x == 0) ctrl->status = 1;
    return;
  }
  uint32_t p2 = 1;
  while (p2 < nb) p2 <<= 1;
  for (uint32_t j = threadIdx.x; j < p2; j += 1024)
    sk[j] = j < nb ? (((uint64_t)bkey[j] << 32) | (uint64_t)(0xFFFFFFFFu - bidx[j])) : 0ull;
  for (int64_t j = threadIdx.x; j < G; j += 1024) segsel[j] = 0;
  __syncthreads();
  // bitonic sort, descending
  for (uint32_t size = 2; size <= p2; size <<= 1) {
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      for (uint32_t t = threadIdx.x; t < (p2 >> 1); t += 1024) {
        const uint32_t i = 2 * t - (t & (stride - 1));
        const uint32_t j = i + stride;
        const bool desc = ((i & size) == 0);
        const uint64_t a = sk[i], b = sk[j];
        if ((a < b) == desc) { sk[i] = b; sk[j] = a; }
      }
      __syncthreads();
    }
  }
  for (uint32_t j = threadIdx.x; j < need; j += 1024) {
    const uint32_t idx = 0xFFFFFFFFu - (uint32_t)(sk[j] & 0xFFFFFFFFull);
    atomicAdd(&segsel[idx / (uint32_t)R], 1u);
  }
  if (threadIdx.x == 0) {
    const uint64_t last = sk[need - 1];
    ctrl->T = (uint32_t)(last >> 32);
    ctrl->icut = 0xFFFFFFFFu - (uint32_t)(last & 0xFFFFFFFFull);
  }
  __syncthreads();
  uint32_t carry = 0;
  for (int64_t base = 0; base < G; base += 1024) {
    const int64_t sgi = base + threadIdx.x;
    const uint32_t v = sgi < G ? segabove[sgi] + segsel[sgi] : 0u;
    uint32_t tot;
    const uint32_t ex = block_excl_scan(v, wsum, &tot);
    if (sgi < G) segoff[sgi] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0 && carry != (uint32_t)k) ctrl->status = 2;  // internal inconsistency
}

template <bool VEC>
__global__ void __launch_bounds__(256) fast_compact_kernel(KeySrc s, int64_t n, int64_t R,
                                                           int64_t CAP, const TopkCtrl* ctrl,
                                                           const uint32_t* segcnt,
                                                           const uint32_t* segoff,
                                                           const uint32_t* cidx,
                                                           const uint32_t* ckey, const float* cval,
                                                           const float* vals_src, int32_t* idx_out,
                                                           float* val_out, int32_t* counter,
                                                           float* rewind, int64_t k) {
  __shared__ uint32_t wsum[16];
  if (ctrl->status) return;
  const uint32_t T = ctrl->T, icut = ctrl->icut;
  const int64_t seg = blockIdx.x;
  const uint32_t cnt = segcnt[seg];
  uint32_t run = segoff[seg];
  if (cnt != DENSE) {
    for (uint32_t base = 0; base < cnt; base += 256) {
      const uint32_t j = base + threadIdx.x;
      bool sel = false;
      uint32_t idx = 0, key = 0;
      if (j < cnt) {
        key = ckey[seg * CAP + j];
        idx = cidx[seg * CAP + j];
        sel = key > T || (key == T && idx <= icut);
      }
      uint32_t tot;
      const uint32_t ex = block_excl_scan(sel ? 1u : 0u, wsum, &tot);
      if (sel && run + ex < (uint64_t)k) {
        const uint32_t pos = run + ex;
        idx_out[pos] = (int32_t)idx;
        val_out[pos] = cval[seg * CAP + j];
        if (counter) counter[idx] += 1;
        if (rewind) rewind[idx] = 0.0f;
      }
      run += tot;
    }
  } else {
    const int64_t beg = seg * R;
    const int64_t end = (beg + R < n) ? beg + R : n;
    for (int64_t b0 = beg; b0 < end; b0 += 1024) {
      const int64_t i0 = b0 + threadIdx.x * 4;
      uint32_t key[4];
      const int c = i0 < end ? load_keys4<VEC>(s, i0, end, false, key) : 0;
      uint32_t ns = 0;
      bool sel[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        sel[e] = e < c && (key[e] > T || (key[e] == T && (uint32_t)(i0 + e) <= icut));
        ns += sel[e];
      }
      uint32_t tot;
      uint32_t pos = run + block_excl_scan(ns, wsum, &tot);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (sel[e] && pos < (uint64_t)k) {
          const int64_t i = i0 + e;
          idx_out[pos] = (int32_t)i;
          val_out[pos] = vals_src[i];
          if (counter) counter[i] += 1;
          if (rewind) rewind[i] = 0.0f;
          ++pos;
        }
      }
      run += tot;
    }
  }
}

// acc += x - x0 only (k == 0 with accumulation: the reference still accumulates).
template <bool VEC>
__global__ void __launch_bounds__(256) accumulate_only_kernel(KeySrc s, int64_t n) {
  const int64_t ngroups = (n + 3) >> 2;
  for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < ngroups;
       g += (int64_t)gridDim.x * 256) {
    uint32_t key[4];
    load_keys4<VEC>(s, g * 4, n, true, key);
  }
}

// ================================================================================================
// host side
// ================================================================================================
struct EncodeArgs {
  const float* x; const float* x0; float* acc; int acc_mode; const float* vals_src;
  int64_t n, k; int32_t* idx_out; float* val_out; int32_t* counter; char* ws;
  hipStream_t st;
};

template <bool VEC>
static int run_exact(const EncodeArgs& a, const WsLayout& L, int rekey) {
  KeySrc s{a.x, a.x0, a.acc, a.acc_mode, rekey};
  TopkCtrl* ctrl = reinterpret_cast<TopkCtrl*>(a.ws + L.ctrl);
  uint32_t* hist = reinterpret_cast<uint32_t*>(a.ws + L.ex_hist);
  DPZ_HIP_TRY(hipMemsetAsync(a.ws + L.ctrl, 0, L.ex_gt - L.ctrl, a.st));
  const int64_t groups = (a.n + 3) / 4;
  int hb = (int)((groups + 255) / 256);
  if (hb > EX_HIST_BLOCKS) hb = EX_HIST_BLOCKS;
  if (hb < 1) hb = 1;
  const int store_acc = (a.acc_mode == DPZ_ACC_ACCUMULATE && !rekey) ? 1 : 0;
  exact_hist_kernel<VEC, 0><<<hb, 256, 0, a.st>>>(s, a.n, ctrl, hist, store_acc);
  DPZ_LAUNCH_CHECK();
  s.rekey = 1;
  exact_resolve_kernel<0><<<1, 1024, 0, a.st>>>(ctrl, hist, (uint32_t)a.k);
  DPZ_LAUNCH_CHECK();
  exact_hist_kernel<VEC, 1><<<hb, 256, 0, a.st>>>(s, a.n, ctrl, hist + 1024, 0);
  DPZ_LAUNCH_CHECK();
  exact_resolve_kernel<1><<<1, 1024, 0, a.st>>>(ctrl, hist + 1024, (uint32_t)a.k);
  DPZ_LAUNCH_CHECK();
  exact_hist_kernel<VEC, 2><<<hb, 256, 0, a.st>>>(s, a.n, ctrl, hist + 3072, 0);
  DPZ_LAUNCH_CHECK();
  exact_resolve_kernel<2><<<1, 1024, 0, a.st>>>(ctrl, hist + 3072, (uint32_t)a.k);
  DPZ_LAUNCH_CHECK();
  uint32_t* bgt = reinterpret_cast<uint32_t*>(a.ws + L.ex_gt);
  uint32_t* beq = reinterpret_cast<uint32_t*>(a.ws + L.ex_eq);
  uint32_t* boff = reinterpret_cast<uint32_t*>(a.ws + L.ex_off);
  uint32_t* beqb = reinterpret_cast<uint32_t*>(a.ws + L.ex_eqb);
  exact_count_kernel<VEC><<<(unsigned)L.ex_nblk, 256, 0, a.st>>>(s, a.n, ctrl, bgt, beq);
  DPZ_LAUNCH_CHECK();
  exact_scan_kernel<<<1, 1024, 0, a.st>>>(ctrl, L.ex_nblk, bgt, beq, boff, beqb);
  DPZ_LAUNCH_CHECK();
  float* rewind = (a.acc && a.acc_mode != DPZ_ACC_NONE) ? a.acc : nullptr;
  exact_write_kernel<VEC><<<(unsigned)L.ex_nblk, 256, 0, a.st>>>(
      s, a.n, ctrl, boff, beqb, a.vals_src, a.idx_out, a.val_out, a.counter, rewind, a.k);
  DPZ_LAUNCH_CHECK();
  return DPZ_OK;
}

template <bool VEC>
static int run_fast(const EncodeArgs& a, const WsLayout& L) {
  KeySrc s{a.x, a.x0, a.acc, a.acc_mode, 0};
  TopkCtrl* ctrl = reinterpret_cast<TopkCtrl*>(a.ws + L.ctrl);
  uint32_t* ghist = reinterpret_cast<uint32_t*>(a.ws + L.f_ghist);
  uint32_t* rows = reinterpret_cast<uint32_t*>(a.ws + L.f_rows);
  uint32_t* segcnt = reinterpret_cast<uint32_t*>(a.ws + L.f_segcnt);
  uint32_t* segabove = reinterpret_cast<uint32_t*>(a.ws + L.f_segabove);
  uint32_t* segoff = reinterpret_cast<uint32_t*>(a.ws + L.f_segoff);
  uint32_t* cidx = reinterpret_cast<uint32_t*>(a.ws + L.f_cidx);
  uint32_t* ckey = reinterpret_cast<uint32_t*>(a.ws + L.f_ckey);
  float* cval = reinterpret_cast<float*>(a.ws + L.f_cval);
  uint32_t* bkey = reinterpret_cast<uint32_t*>(a.ws + L.f_bkey);
  uint32_t* bidx = reinterpret_cast<uint32_t*>(a.ws + L.f_bidx);
  const FastGeom& g = L.fg;
  const int vals_is_x = (a.vals_src == a.x) ? 1 : 0;
  fast_sample_kernel<<<1, 1024, 0, a.st>>>(s, a.n, a.k, ctrl, ghist);
  DPZ_LAUNCH_CHECK();
  fast_filter_kernel<VEC><<<(unsigned)g.G, 256, 0, a.st>>>(s, a.n, g.R, g.CAP, ctrl, a.vals_src,
                                                           vals_is_x, rows, segcnt, cidx, ckey,
                                                           cval);
  DPZ_LAUNCH_CHECK();
  s.rekey = 1;
  fast_selectA_kernel<<<64, 256, 0, a.st>>>(rows, g.G, ghist);
  DPZ_LAUNCH_CHECK();
  fast_selectB_kernel<VEC><<<(unsigned)g.G, 256, 0, a.st>>>(s, a.n, a.k, g.R, g.CAP, ctrl, ghist,
                                                            segcnt, cidx, ckey, segabove, bkey,
                                                            bidx);
  DPZ_LAUNCH_CHECK();
  fast_selectC_kernel<<<1, 1024, 0, a.st>>>(a.k, g.G, g.R, ctrl, bkey, bidx, segabove, segoff);
  DPZ_LAUNCH_CHECK();
  float* rewind = (a.acc && a.acc_mode != DPZ_ACC_NONE) ? a.acc : nullptr;
  fast_compact_kernel<VEC><<<(unsigned)g.G, 256, 0, a.st>>>(s, a.n, g.R, g.CAP, ctrl, segcnt,
                                                            segoff, cidx, ckey, cval, a.vals_src,
                                                            a.idx_out, a.val_out, a.counter,
                                                            rewind, a.k);
  DPZ_LAUNCH_CHECK();
  return DPZ_OK;
}

static bool use_fast(int64_t n, int64_t k) { return n >= (1 << 18) && k >= 1 && k <= n / 16; }

template <bool VEC>
static int run_accumulate_only(const EncodeArgs& a) {
  KeySrc s{a.x, a.x0, a.acc, a.acc_mode, 0};
  const int64_t groups = (a.n + 3) / 4;
  int nb = (int)((groups + 255) / 256);
  if (nb > 4096) nb = 4096;
  if (nb < 1) nb = 1;
  accumulate_only_kernel<VEC><<<nb, 256, 0, a.st>>>(s, a.n);
  DPZ_LAUNCH_CHECK();
  return DPZ_OK;
}

static bool all_aligned(const EncodeArgs& a) {
  auto al = [](const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15u) == 0; };
  return al(a.x) && al(a.x0) && al(a.acc) && al(a.vals_src);
}

static int validate(const EncodeArgs& a, size_t ws_bytes) {
  if (a.n < 0 || a.k < 0 || a.k > a.n || a.n >= (int64_t(1) << 31)) return DPZ_ERR_ARG;
  if (a.acc_mode < DPZ_ACC_NONE || a.acc_mode > DPZ_ACC_ADD) return DPZ_ERR_ARG;
  if (a.n > 0 && !a.x) return DPZ_ERR_ARG;
  if (a.acc_mode != DPZ_ACC_NONE && !a.acc) return DPZ_ERR_ARG;
  if (a.k > 0 && (!a.idx_out || !a.val_out || !a.vals_src)) return DPZ_ERR_ARG;
  if (a.n > 0 && (!a.ws || ws_bytes < ws_layout(a.n).total)) return DPZ_ERR_WORKSPACE;
  return DPZ_OK;
}

}  // namespace dpz

using namespace dpz;

extern "C" size_t dpz_topk_workspace_bytes(int64_t n, int64_t k) {
  (void)k;
  return ws_layout(n > 0 ? n : 1).total;
}

static int dpz_topk_dispatch(const EncodeArgs& a, int flags) {
  const WsLayout L = ws_layout(a.n);
  const bool vec = all_aligned(a);
  if (a.k == 0) {
    if (a.acc_mode == DPZ_ACC_ACCUMULATE && a.n > 0)
      return vec ? run_accumulate_only<true>(a) : run_accumulate_only<false>(a);
    return DPZ_OK;
  }
  if (!(flags & DPZ_TOPK_EXACT) && use_fast(a.n, a.k)) {
    int rc = vec ? run_fast<true>(a, L) : run_fast<false>(a, L);
    if (rc != DPZ_OK) return rc;
    if (flags & DPZ_TOPK_ASYNC) return DPZ_OK;
    int fb = 0;
    return dpz_topk_complete(a.x, a.x0, a.acc, a.acc_mode, a.vals_src, a.n, a.k, a.idx_out,
                             a.val_out, a.counter, a.ws, L.total, &fb, a.st);
  }
  int rc = vec ? run_exact<true>(a, L, 0) : run_exact<false>(a, L, 0);
  if (rc != DPZ_OK) return rc;
  if (!(flags & DPZ_TOPK_ASYNC)) DPZ_HIP_TRY(hipStreamSynchronize(a.st));
  return DPZ_OK;
}

extern "C" int dpz_topk_encode(const float* x, const float* x0, float* acc, int acc_mode,
                               const float* vals_src, int64_t n, int64_t k, int32_t* idx_out,
                               float* val_out, int32_t* counter, void* ws, size_t ws_bytes,
                               int flags, dpz_stream_t stream) {
  EncodeArgs a{x, x0, acc, acc_mode, vals_src, n, k, idx_out, val_out, counter,
               static_cast<char*>(ws), static_cast<hipStream_t>(stream)};
  int rc = validate(a, ws_bytes);
  if (rc != DPZ_OK) return rc;
  if (n == 0) return DPZ_OK;
  // the exact path needs the ctrl block with status == 0 for dpz_topk_complete
  return dpz_topk_dispatch(a, flags);
}

extern "C" int dpz_topk_complete(const float* x, const float* x0, float* acc, int acc_mode,
                                 const float* vals_src, int64_t n, int64_t k, int32_t* idx_out,
                                 float* val_out, int32_t* counter, void* ws, size_t ws_bytes,
                                 int* used_fallback, dpz_stream_t stream) {
  EncodeArgs a{x, x0, acc, acc_mode, vals_src, n, k, idx_out, val_out, counter,
               static_cast<char*>(ws), static_cast<hipStream_t>(stream)};
  int rc = validate(a, ws_bytes);
  if (rc != DPZ_OK) return rc;
  if (used_fallback) *used_fallback = 0;
  DPZ_HIP_TRY(hipStreamSynchronize(a.st));
  if (n == 0 || k == 0 || !use_fast(n, k)) return DPZ_OK;
  const WsLayout L = ws_layout(n);
  uint32_t status = 0;
  DPZ_HIP_TRY(hipMemcpy(&status, a.ws + L.ctrl + offsetof(TopkCtrl, status), sizeof(status),
                        hipMemcpyDeviceToHost));
  if (status == 0) return DPZ_OK;
  if (used_fallback) *used_fallback = 1;
  // keys are re-derived from the post-filter state: ACCUMULATE already stored acc += change
  const bool vec = all_aligned(a);
  rc = vec ? run_exact<true>(a, L, 1) : run_exact<false>(a, L, 1);
  if (rc != DPZ_OK) return rc;
  DPZ_HIP_TRY(hipStreamSynchronize(a.st));
  return DPZ_OK;
}
