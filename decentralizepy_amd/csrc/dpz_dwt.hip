// Multilevel sym2 DWT / IDWT (mode "symmetric"), fp32, bit-exact with PyWavelets 1.1.1.
//
// Replaces (reference sacs-epfl/decentralizepy, src/decentralizepy/):
//   sharing/JWINS/Wavelet.py:12-32   change_transformer_wavelet: pywt.wavedec + coeffs_to_array
//   sharing/JWINS/Wavelet.py:311-316 pywt.array_to_coeffs + pywt.waverec
//   sharing/PartialModel.py:317-320  W(x) and W(x - x0) computed in one pass (pre-step)
//   sharing/PartialModel.py:346-349  acc += W(x_new - prev)  (post-step, accumulate mode)
//
// Forward: one block owns TL = 128 level-L outputs and the matching 2^(L-l)*TL outputs of every
// detail level; it stages the input span (16*TL + 30 halo for L = 4) in LDS and walks the levels
// down in LDS (ping-pong buffers), writing each level's owned details straight to the
// concatenated [cA_L, cD_L, ..., cD_1] layout.  Every convolution uses pywt's summation order
// (see oracle/wavelet.py); the whole library is compiled with -ffp-contract=off.
// Inverse: one block owns 4096 final outputs and reconstructs the (halo'd) ranges of each level
// top-down in LDS.
#include "dpz_common.h"

namespace dpz {

constexpr int DWT_MAX_LEVEL = 8;
#ifndef DPZ_DWT_TL
#define DPZ_DWT_TL 128
#endif
constexpr int DWT_TL = DPZ_DWT_TL;
// waves per SIMD the forward kernel is register-bounded for (3 without the bound: 150 VGPRs)
#ifndef DPZ_DWT_WAVES
#define DPZ_DWT_WAVES 4
#endif
#ifndef DPZ_DWT4_WAVES  // the level-4 kernel (interior path)
#define DPZ_DWT4_WAVES 4
#endif
#ifndef DPZ_DWT4_ACC_WAVES  // the level-4 accumulating kernel with the accumulator prefetch
#define DPZ_DWT4_ACC_WAVES 4
#endif
#ifndef DPZ_IDWT_TILE
#define DPZ_IDWT_TILE 4096
#endif
constexpr int IDWT_TILE = DPZ_IDWT_TILE;
// The IDWT's final outputs are stored non-temporally (written once, not re-read by the pass):
// 50.1 -> 44.1 us at N = 25 M standalone, 46.0 -> 45.2 us inside the C3 round (MI355X, same-box
// A/B, tools/diag/idwt_ab.py).  Tried and not kept: non-temporal coefficient loads (no gain), one
// thread per output pair with 8-byte stores (49.5 us), 2048-output tiles (55.1 us).
#ifndef DPZ_IDWT_NT
#define DPZ_IDWT_NT 1
#endif

// sym2 filters (fp32 casts of pywt's double coefficients)
__constant__ float c_dec_lo[4] = {-0.12940952255092145f, 0.22414386804185735f,
                                  0.836516303737469f, 0.48296291314469025f};
__constant__ float c_dec_hi[4] = {-0.48296291314469025f, 0.836516303737469f,
                                  -0.22414386804185735f, -0.12940952255092145f};
__constant__ float c_rec_lo[4] = {0.48296291314469025f, 0.836516303737469f,
                                  0.22414386804185735f, -0.12940952255092145f};
__constant__ float c_rec_hi[4] = {-0.12940952255092145f, -0.22414386804185735f,
                                  0.836516303737469f, -0.48296291314469025f};

struct Levels {
  int64_t len[DWT_MAX_LEVEL + 1];   // len[0] = n, len[l] = floor((len[l-1] + 3) / 2)
  int64_t doff[DWT_MAX_LEVEL + 1];  // offset of cD_l in the coefficient array
  int64_t total;
  int level;
  // accumulate with the deferred rewind (dpz_dwt_sym2_rewind): acc[i] = (bit i ? 0 : acc[i]) + c
  const uint32_t* rmask;
};

// The accumulating pass's read-modify-write of a thread's two adjacent outputs as ONE 8-byte load
// and store (4-byte aligned: the level offsets may be odd; gfx950 global memory takes dword-aligned
// dwordx2): the element-wise form issued 2 loads + 2 stores per pair, each store behind its load
// (PMC: 2.6x the VMEM reads, 2x the writes and 3.4x the wait cycles of the plain pass).
typedef float dwt_f2u __attribute__((ext_vector_type(2), aligned(4)));
__device__ __forceinline__ void acc_pair(const Levels& LV, float* dst, int64_t pos, float a,
                                         float b) {
  const dwt_f2u v = *reinterpret_cast<const dwt_f2u*>(dst);
  float o0 = v.x, o1 = v.y;
  if (LV.rmask) {  // one mask word unless the pair straddles two
    const uint32_t w0 = LV.rmask[pos >> 5];
    const uint32_t w1 = ((pos & 31) == 31) ? LV.rmask[(pos + 1) >> 5] : w0;
    if ((w0 >> (pos & 31)) & 1u) o0 = 0.0f;
    if ((w1 >> ((pos + 1) & 31)) & 1u) o1 = 0.0f;
  }
  dwt_f2u r;
  r.x = o0 + a;
  r.y = o1 + b;
  *reinterpret_cast<dwt_f2u*>(dst) = r;
}

// the accumulator's value before this pass adds to it: 0 where the encode selected the
// coefficient (reference: rewind_accumulation zeroed it during the step, models/Model.py:53-64,
// and the post-step adds 0 + c — kept as a real addition so -0.0 becomes +0.0 as there)
__device__ __forceinline__ float acc_before(const Levels& LV, const float* dst, int64_t pos) {
  const float o = *dst;
  if (LV.rmask && ((LV.rmask[pos >> 5] >> (pos & 31)) & 1u)) return 0.0f;
  return o;
}

// The accumulating pass's interior tiles (dwt4_kernel): every accumulator pair a thread
// rewrites in the tile (level 1: up to 3, level 2: 2, level 3: 1, level 4: cA and cD) and its
// mask words are loaded at the START of the tile, before the next tile's span loads are issued.
// Loaded at the store instead (acc_pair), each pair was a dependent round trip behind a
// vmcnt(0) wait that also drained the next tile's prefetched span: 6-8 exposed HBM latencies per
// tile.  Slots: 0-2 level 1 (group t + 256 q), 3-4 level 2 (pair 1 + t + 256 j), 5 level 3,
// 6 level-4 cA, 7 level-4 cD.  Loads are branch-free (an unused slot re-reads a valid word).
#ifndef DPZ_DWT_ACC_PRE
#define DPZ_DWT_ACC_PRE 1
#endif
constexpr int ACC_SLOTS = 8;
struct AccPre {
  dwt_f2u v[ACC_SLOTS];
  uint32_t m0[ACC_SLOTS], m1[ACC_SLOTS];
};

__device__ __forceinline__ void acc_slot_load(const Levels& LV, const float* cd, int64_t nwords,
                                              bool ok, int64_t pos, AccPre& P, int s) {
  const int64_t q = ok ? pos : 0;
  P.v[s] = *reinterpret_cast<const dwt_f2u*>(cd + q);
  if (LV.rmask) {
    const int64_t w = q >> 5;
    P.m0[s] = LV.rmask[w];
    P.m1[s] = LV.rmask[w + 1 < nwords ? w + 1 : w];
  } else {
    P.m0[s] = 0u;
    P.m1[s] = 0u;
  }
}

// the pair (pos, pos + 1) from its preloaded slot: (bit ? 0 : acc) + c
__device__ __forceinline__ void acc_pair_pre(float* dst, int64_t pos, float a, float b,
                                             const AccPre& P, int s) {
  const uint32_t w0 = P.m0[s];
  const uint32_t w1 = ((pos & 31) == 31) ? P.m1[s] : w0;
  const float o0 = ((w0 >> (pos & 31)) & 1u) ? 0.0f : P.v[s].x;
  const float o1 = ((w1 >> ((pos + 1) & 31)) & 1u) ? 0.0f : P.v[s].y;
  dwt_f2u r;
  r.x = o0 + a;
  r.y = o1 + b;
  *reinterpret_cast<dwt_f2u*>(dst) = r;
}

static inline Levels make_levels(int64_t n, int level) {
  Levels L{};
  L.level = level;
  L.len[0] = n;
  for (int l = 1; l <= level; ++l) L.len[l] = (L.len[l - 1] + 3) / 2;
  int64_t o = L.len[level];
  for (int l = level; l >= 1; --l) {
    L.doff[l] = o;
    o += L.len[l];
  }
  L.total = o;
  return L;
}

// one convolution output o of a level whose input (extended, in LDS) is `in` with origin s_in:
// in[p - s_in] = x~[p].  `last_odd` selects pywt's right-overhang order for the last output of
// an odd-length input.
__device__ __forceinline__ float conv4(const float* in, int64_t s_in, int64_t o, const float* f,
                                       bool last_odd) {
  const int64_t i = 2 * o + 1 - s_in;
  if (!last_odd) {
    float acc = f[0] * in[i];
    acc = acc + f[1] * in[i - 1];
    acc = acc + f[2] * in[i - 2];
    acc = acc + f[3] * in[i - 3];
    return acc;
  }
  float acc = f[2] * in[i - 2];   // x~[n]
  acc = acc + f[1] * in[i - 1];   // x~[n+1]
  acc = acc + f[0] * in[i];       // x~[n+2]
  acc = acc + f[3] * in[i - 3];   // x~[n-1]
  return acc;
}

// conv4 on a 32-bit LDS offset i (= 2 o + 1 - s_in), same summation orders
__device__ __forceinline__ float conv4r(const float* in, int i, const float* f, bool last_odd) {
  if (!last_odd) {
    float acc = f[0] * in[i];
    acc = acc + f[1] * in[i - 1];
    acc = acc + f[2] * in[i - 2];
    acc = acc + f[3] * in[i - 3];
    return acc;
  }
  float acc = f[2] * in[i - 2];   // x~[n]
  acc = acc + f[1] * in[i - 1];   // x~[n+1]
  acc = acc + f[0] * in[i];       // x~[n+2]
  acc = acc + f[3] * in[i - 3];   // x~[n-1]
  return acc;
}

constexpr int DWT_SPAN0 = 16 * DWT_TL + 64;  // level-0 span (covers L <= 4 with slack)
constexpr int DWT_SPAN1 = 8 * DWT_TL + 32;
constexpr int DWT_NG = (DWT_SPAN0 + 4 + 4 * 256 - 1) / (4 * 256);  // float4 groups per thread

// level-0 input span [s0, e0) of a tile (its level-L outputs [a, b) and the halos below)
__device__ __forceinline__ void dwt_span(const Levels& LV, int64_t tile, int64_t* s0,
                                         int64_t* e0) {
  const int L = LV.level;
  const int64_t nL = LV.len[L];
  int64_t sl = tile * DWT_TL;
  int64_t el = (sl + DWT_TL < nL) ? sl + DWT_TL : nL;
  for (int l = L; l >= 1; --l) {
    sl = 2 * sl - 2;
    el = 2 * el;
  }
  *s0 = sl;
  *e0 = el;
}

// Every load of a span is issued before any is used (float4 groups from the 4-aligned start below
// s0; a group not wholly inside [0, n) or an unaligned input takes scalar loads).
template <bool WD>
__device__ __forceinline__ void dwt_span_load(const float* __restrict__ x,
                                              const float* __restrict__ x0, int64_t n, int64_t s0,
                                              int64_t e0, float4 (&va)[DWT_NG],
                                              float4 (&vb)[DWT_NG]) {
  const int64_t g0 = s0 >= 0 ? (s0 & ~int64_t(3)) : -((-s0 + 3) & ~int64_t(3));
  const bool vec = aligned16(x) && (!WD || aligned16(x0));
#pragma unroll
  for (int q = 0; q < DWT_NG; ++q) {
    const int64_t p = g0 + 4 * (threadIdx.x + 256 * q);
    va[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    vb[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (p < e0) {
      if (vec && p >= 0 && p + 4 <= n) {
        va[q] = *reinterpret_cast<const float4*>(x + p);
        if (WD) vb[q] = *reinterpret_cast<const float4*>(x0 + p);
      } else {
        float ta[4] = {0.f, 0.f, 0.f, 0.f}, tb[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (p + e >= 0 && p + e < n) {
            ta[e] = x[p + e];
            if (WD) tb[e] = x0[p + e];
          }
        }
        va[q] = make_float4(ta[0], ta[1], ta[2], ta[3]);
        vb[q] = make_float4(tb[0], tb[1], tb[2], tb[3]);
      }
    }
  }
}

// The span into LDS (x and / or x - x0) plus pywt's symmetric extension at the array ends.
template <bool WX, bool WD>
__device__ __forceinline__ void dwt_span_store(const float4 (&va)[DWT_NG],
                                               const float4 (&vb)[DWT_NG], int64_t n, int64_t s0,
                                               int64_t e0, float* smem) {
  float* bufA[2] = {smem, smem + DWT_SPAN0 + DWT_SPAN1};
  const int64_t g0 = s0 >= 0 ? (s0 & ~int64_t(3)) : -((-s0 + 3) & ~int64_t(3));
#pragma unroll
  for (int q = 0; q < DWT_NG; ++q) {
    const int64_t p = g0 + 4 * (threadIdx.x + 256 * q);
    const float xa[4] = {va[q].x, va[q].y, va[q].z, va[q].w};
    const float xb[4] = {vb[q].x, vb[q].y, vb[q].z, vb[q].w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t pe = p + e;
      if (pe >= s0 && pe < e0 && pe >= 0 && pe < n) {
        if (WX) bufA[0][pe - s0] = xa[e];
        if (WD) bufA[1][pe - s0] = xa[e] - xb[e];
      }
    }
  }
  __syncthreads();
  // extension: only x~[-3..-1] and x~[n..n+2] are ever read
  if (threadIdx.x < 6) {
    const int64_t p = threadIdx.x < 3 ? -1 - (int64_t)threadIdx.x : n + (threadIdx.x - 3);
    const int64_t src = p < 0 ? -1 - p : 2 * n - 1 - p;
    if (p >= s0 && p < e0 && src >= s0 && src < e0) {
      if (WX) bufA[0][p - s0] = bufA[0][src - s0];
      if (WD) bufA[1][p - s0] = bufA[1][src - s0];
    }
  }
  __syncthreads();
}

// The levels of one tile from its level-0 span in LDS.
template <bool WX, bool WD, bool ACCUM>
__device__ __forceinline__ void dwt_levels(const Levels& LV, float* cx, float* cd, int64_t tile,
                                           float* smem) {
  constexpr int SPAN0 = DWT_SPAN0;
  constexpr int SPAN1 = DWT_SPAN1;
  // pipelines: 0 = W(x), 1 = W(x - x0); buffers A (SPAN0) and B (SPAN1) per pipeline
  float* bufA[2] = {smem, smem + SPAN0 + SPAN1};
  float* bufB[2] = {smem + SPAN0, smem + 2 * SPAN0 + SPAN1};
  const int L = LV.level;
  const int64_t nL = LV.len[L];
  const int64_t a = tile * DWT_TL;
  const int64_t b = (a + DWT_TL < nL) ? a + DWT_TL : nL;
  const bool last_block = (b == nL);
  // needed ranges per level (top-down)
  int64_t s[DWT_MAX_LEVEL + 1], e[DWT_MAX_LEVEL + 1];
  s[L] = a;
  e[L] = b;
  for (int l = L; l >= 1; --l) {
    s[l - 1] = 2 * s[l] - 2;
    e[l - 1] = 2 * e[l];
  }
  float* in[2] = {bufA[0], bufA[1]};
  float* outb[2] = {bufB[0], bufB[1]};
  for (int l = 1; l <= L; ++l) {
    const int64_t nin = LV.len[l - 1], nout = LV.len[l];
    const int64_t sl = s[l], el = e[l];
    const bool odd_in = (nin & 1) != 0;
    // owned detail range at this level
    const int64_t own_lo = a << (L - l);
    const int64_t own_hi = last_block ? nout : (b << (L - l));
    const int64_t c_lo = sl > 0 ? sl : 0;
    const int64_t c_hi = el < nout ? el : nout;
    // 32-bit offsets relative to sl (the block-uniform level origin): the input of output
    // sl + r starts at in[2r + 3 - 3] (sin = 2 sl - 2), so conv4's window top is in[2r + 3]
    const int r_lo = (int)(c_lo - sl), r_hi = (int)(c_hi - sl);
    const int64_t own_lo_r = own_lo - sl, own_hi_r = own_hi - sl;
    const int own_a = (int)(own_lo_r < 0 ? 0 : own_lo_r);
    const int own_b = (int)(own_hi_r > r_hi ? r_hi : own_hi_r);
    const int64_t odd_r64 = odd_in ? (nout - 1 - sl) : -1;
    const int odd_r = (odd_r64 >= r_lo && odd_r64 < r_hi) ? (int)odd_r64 : -1;
    float* const cxd = WX ? cx + LV.doff[l] + sl : nullptr;
    float* const cdd = WD ? cd + LV.doff[l] + sl : nullptr;
    float* const cxa = WX ? cx + sl : nullptr;
    float* const cda = WD ? cd + sl : nullptr;
    for (int r = r_lo + (int)threadIdx.x; r < r_hi; r += 256) {
      const bool lo_odd = (r == odd_r);
      const bool own = (r >= own_a && r < own_b);
      const int i = 2 * r + 3;
      if (WX) {
        if (l < L) outb[0][r] = conv4r(in[0], i, c_dec_lo, lo_odd);
        if (own) cxd[r] = conv4r(in[0], i, c_dec_hi, lo_odd);
        if (l == L && own) cxa[r] = conv4r(in[0], i, c_dec_lo, lo_odd);
      }
      if (WD) {
        if (l < L) outb[1][r] = conv4r(in[1], i, c_dec_lo, lo_odd);
        if (own) {
          const float dv = conv4r(in[1], i, c_dec_hi, lo_odd);
          if (ACCUM) cdd[r] = acc_before(LV, cdd + r, LV.doff[l] + sl + r) + dv; else cdd[r] = dv;
        }
        if (l == L && own) {
          const float av = conv4r(in[1], i, c_dec_lo, lo_odd);
          if (ACCUM) cda[r] = acc_before(LV, cda + r, sl + r) + av; else cda[r] = av;
        }
      }
    }
    if (l == L) break;
    __syncthreads();
    if (threadIdx.x < 6) {
      const int64_t p = threadIdx.x < 3 ? -1 - (int64_t)threadIdx.x : nout + (threadIdx.x - 3);
      const int64_t src = p < 0 ? -1 - p : 2 * nout - 1 - p;
      if (p >= sl && p < el && src >= sl && src < el) {
        if (WX) outb[0][p - sl] = outb[0][src - sl];
        if (WD) outb[1][p - sl] = outb[1][src - sl];
      }
    }
    __syncthreads();
    float* t0 = in[0]; in[0] = outb[0]; outb[0] = t0;
    float* t1 = in[1]; in[1] = outb[1]; outb[1] = t1;
  }
}

// ---- interior tiles at level 4 (no array edge within reach, not the first tile of a sharded
// range): level 1 is computed straight from the span registers — group G (inputs g0 + 4G .. +3)
// gives the level-1 outputs 2G, 2G + 1 from its 4 inputs and the 2 before it (the left lane's
// z, w by a shuffle; lane 0 of each wave loads them) — its details go to global memory and its
// approximations to LDS as one 8-byte store.  Levels 2-4 read LDS as 8 + 16-byte vectors: a
// thread computes two adjacent outputs from 6 consecutive inputs (no bank conflicts; the span
// path reads with a stride of 2).  Same pywt summation order as conv4r (no odd-length tail
// inside an interior tile).
constexpr int DWT_IN1 = 8 * DWT_TL + 16;       // level-1 values per pipeline (from 8 TL t - 16)
constexpr int DWT_IN2 = 4 * DWT_TL + 8;        // level-2 values (from 4 TL t - 8)
constexpr int DWT_IN3 = 2 * DWT_TL + 4;        // level-3 values (from 2 TL t - 4)
constexpr int DWT_NGRP = (16 * DWT_TL + 32) / 4;  // float4 groups of an interior span

// interior tiles of a level-4 launch over [tile0, tile_hi): [a, b) with a = max(tile0 + 1, 1)
// (the first tile of a sharded range has only a 32-input halo) and (t + 2) * 16 TL <= n (no
// symmetric extension within reach at any level)
static inline void dwt_interior_range(int64_t n, int64_t tile0, int64_t tile_hi, int64_t* a,
                                      int64_t* b) {
  int64_t lo = tile0 + 1 > 1 ? tile0 + 1 : 1;
  int64_t hi = n / (16 * DWT_TL) - 1;
  if (hi > tile_hi) hi = tile_hi;
  if (lo > tile_hi) lo = tile_hi;
  if (hi < lo) hi = lo;
  *a = lo;
  *b = hi;
}

// the 2 inputs before each wave's first group (lane 0) of an interior span
template <bool WD>
__device__ __forceinline__ void dwt_halo_load(const float* __restrict__ x,
                                              const float* __restrict__ x0, int64_t g0,
                                              float2 (&hx)[DWT_NG], float2 (&hb)[DWT_NG]) {
#pragma unroll
  for (int q = 0; q < DWT_NG; ++q) {
    const int G = threadIdx.x + 256 * q;
    hx[q] = make_float2(0.f, 0.f);
    hb[q] = hx[q];
    if ((threadIdx.x & 63) == 0 && G < DWT_NGRP) {
      const int64_t p = g0 + 4 * (int64_t)G - 2;
      hx[q] = make_float2(x[p], x[p + 1]);
      if (WD) hb[q] = make_float2(x0[p], x0[p + 1]);
    }
  }
}

__device__ __forceinline__ float conv4v(float i0, float i1, float i2, float i3, const float* f) {
  // f0 * x~[top] + f1 * x~[top-1] + f2 * x~[top-2] + f3 * x~[top-3]; i3 = top
  float acc = f[0] * i3;
  acc = acc + f[1] * i2;
  acc = acc + f[2] * i1;
  acc = acc + f[3] * i0;
  return acc;
}

// the tile's accumulator pairs and mask words, issued at the tile's start (AccPre above)
__device__ __forceinline__ void acc_prefetch(const Levels& LV, const float* cd, int64_t tile,
                                             AccPre& P) {
  static_assert(DWT_NG <= 3 && DWT_IN2 / 2 <= 1 + 2 * 256 && DWT_IN3 / 2 <= 257 &&
                (DWT_TL + 2) / 2 <= 257, "the slots cover every owned pair of a thread");
  const int t = (int)threadIdx.x;
  const int64_t nwords = (LV.total + 31) >> 5;
  const int64_t s1 = tile * (8 * DWT_TL) - 16;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int G = t + 256 * q;
    acc_slot_load(LV, cd, nwords, q < DWT_NG && G >= 8 && G < DWT_NGRP, LV.doff[1] + s1 + 2 * G,
                  P, q);
  }
  const int64_t b2 = tile * (4 * DWT_TL) - 8;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int pp = 1 + t + 256 * j;
    acc_slot_load(LV, cd, nwords, pp < DWT_IN2 / 2 && 2 * pp >= 8, LV.doff[2] + b2 + 2 * pp, P,
                  3 + j);
  }
  const int64_t b3 = tile * (2 * DWT_TL) - 4;
  acc_slot_load(LV, cd, nwords, 1 + t < DWT_IN3 / 2 && 2 * (1 + t) >= 4,
                LV.doff[3] + b3 + 2 * (1 + t), P, 5);
  const int64_t b4 = tile * DWT_TL - 2;
  const bool ok4 = 1 + t < (DWT_TL + 2) / 2;
  acc_slot_load(LV, cd, nwords, ok4, b4 + 2 * (1 + t), P, 6);
  acc_slot_load(LV, cd, nwords, ok4, LV.doff[4] + b4 + 2 * (1 + t), P, 7);
}

template <bool WX, bool WD, bool ACCUM, bool PRE = false>
__device__ __forceinline__ void dwt_int_level1(const Levels& LV, float* cx, float* cd, int64_t tile,
                                               const float4 (&va)[DWT_NG],
                                               const float4 (&vb)[DWT_NG],
                                               const float2 (&hx)[DWT_NG],
                                               const float2 (&hb)[DWT_NG], float* smem,
                                               const AccPre* P = nullptr) {
  float* L1[2] = {smem, smem + DWT_IN1};
  const int64_t s1 = tile * (8 * DWT_TL) - 16;  // level-1 position of LDS index 0
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int q = 0; q < DWT_NG; ++q) {
    const int G = threadIdx.x + 256 * q;
    float in[2][6];  // h0, h1, a0..a3 per pipeline
    in[0][2] = va[q].x; in[0][3] = va[q].y; in[0][4] = va[q].z; in[0][5] = va[q].w;
    if (WD) {
      in[1][2] = va[q].x - vb[q].x; in[1][3] = va[q].y - vb[q].y;
      in[1][4] = va[q].z - vb[q].z; in[1][5] = va[q].w - vb[q].w;
    }
    {
      const float zx = __shfl_up(va[q].z, 1, 64), wx = __shfl_up(va[q].w, 1, 64);
      in[0][0] = lane == 0 ? hx[q].x : zx;
      in[0][1] = lane == 0 ? hx[q].y : wx;
      if (WD) {
        const float zd = __shfl_up(in[1][4], 1, 64), wd = __shfl_up(in[1][5], 1, 64);
        in[1][0] = lane == 0 ? hx[q].x - hb[q].x : zd;
        in[1][1] = lane == 0 ? hx[q].y - hb[q].y : wd;
      }
    }
    if (G >= DWT_NGRP) continue;
    const int64_t o = s1 + 2 * G;  // level-1 outputs o, o + 1
    const bool own = G >= 8;        // [8 TL t, 8 TL (t + 1)) is owned
#pragma unroll
    for (int sp = 0; sp < 2; ++sp) {
      if (sp == 0 && !WX) continue;
      if (sp == 1 && !WD) continue;
      const float* v = in[sp];
      const float lo0 = conv4v(v[0], v[1], v[2], v[3], c_dec_lo);
      const float lo1 = conv4v(v[2], v[3], v[4], v[5], c_dec_lo);
      *reinterpret_cast<float2*>(L1[sp] + 2 * G) = make_float2(lo0, lo1);
      if (own) {
        const float hi0 = conv4v(v[0], v[1], v[2], v[3], c_dec_hi);
        const float hi1 = conv4v(v[2], v[3], v[4], v[5], c_dec_hi);
        float* dst = (sp == 0 ? cx : cd) + LV.doff[1] + o;
        if (ACCUM && sp == 1) {
          if constexpr (PRE) acc_pair_pre(dst, LV.doff[1] + o, hi0, hi1, *P, q);
          else acc_pair(LV, dst, LV.doff[1] + o, hi0, hi1);
        } else {
          dst[0] = hi0;
          dst[1] = hi1;
        }
      }
    }
  }
}

// one level from LDS `in` (index 0 = position base_in) into LDS `out` (or cA at the top level):
// outputs u in [2, nu), u = position - base_out, reading in[2u - 2 .. 2u + 1]; owned details for
// u >= u_own.
template <bool WX, bool WD, bool ACCUM, bool TOP, bool PRE = false>
__device__ __forceinline__ void dwt_int_level(const Levels& LV, float* cx, float* cd, int l,
                                              int64_t base_out, int nu, int u_own, float* const* in,
                                              float* const* out, const AccPre* P = nullptr,
                                              int slot0 = 0) {
  const int npairs = nu / 2;  // pairs p = 1 .. npairs - 1 (u = 2p, 2p + 1): <= 2 per thread
  // iteration j: the preloaded slot slot0 + j (TOP: cA slot0, cD slot0 + 1), compile-time
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int p = 1 + (int)threadIdx.x + 256 * j;
    if (p >= npairs) break;
    const int u = 2 * p;
    const int64_t pos = base_out + u;
#pragma unroll
    for (int sp = 0; sp < 2; ++sp) {
      if (sp == 0 && !WX) continue;
      if (sp == 1 && !WD) continue;
      const float2 A = *reinterpret_cast<const float2*>(in[sp] + 2 * u - 2);
      const float4 B = *reinterpret_cast<const float4*>(in[sp] + 2 * u);
      const float lo0 = conv4v(A.x, A.y, B.x, B.y, c_dec_lo);
      const float lo1 = conv4v(B.x, B.y, B.z, B.w, c_dec_lo);
      float* g = sp == 0 ? cx : cd;
      const bool acc = ACCUM && sp == 1;
      if (TOP) {
        if (u >= u_own) {
          float* dst = g + pos;
          if (acc) {
            if constexpr (PRE) acc_pair_pre(dst, pos, lo0, lo1, *P, slot0);
            else acc_pair(LV, dst, pos, lo0, lo1);
          } else {
            dst[0] = lo0;
            dst[1] = lo1;
          }
        }
      } else {
        *reinterpret_cast<float2*>(out[sp] + u) = make_float2(lo0, lo1);
      }
      if (u >= u_own) {
        const float hi0 = conv4v(A.x, A.y, B.x, B.y, c_dec_hi);
        const float hi1 = conv4v(B.x, B.y, B.z, B.w, c_dec_hi);
        float* dst = g + LV.doff[l] + pos;
        if (acc) {
          if constexpr (PRE) acc_pair_pre(dst, LV.doff[l] + pos, hi0, hi1, *P, TOP ? slot0 + 1 : slot0 + j);
          else acc_pair(LV, dst, LV.doff[l] + pos, hi0, hi1);
        } else {
          dst[0] = hi0;
          dst[1] = hi1;
        }
      }
    }
  }
}

template <bool WX, bool WD, bool ACCUM, bool PRE = false>
__device__ __forceinline__ void dwt_int_levels234(const Levels& LV, float* cx, float* cd,
                                                  int64_t tile, float* smem,
                                                  const AccPre* P = nullptr) {
  float* L1[2] = {smem, smem + DWT_IN1};
  float* L2[2] = {smem + 2 * DWT_IN1, smem + 2 * DWT_IN1 + DWT_IN2};
  float* L3[2] = {smem + 2 * DWT_IN1 + 2 * DWT_IN2, smem + 2 * DWT_IN1 + 2 * DWT_IN2 + DWT_IN3};
  // level 2: positions 4 TL t - 8 + u, owned from u = 8
  dwt_int_level<WX, WD, ACCUM, false, PRE>(LV, cx, cd, 2, tile * (4 * DWT_TL) - 8, DWT_IN2, 8, L1,
                                           L2, P, 3);
  __syncthreads();
  dwt_int_level<WX, WD, ACCUM, false, PRE>(LV, cx, cd, 3, tile * (2 * DWT_TL) - 4, DWT_IN3, 4, L2,
                                           L3, P, 5);
  __syncthreads();
  dwt_int_level<WX, WD, ACCUM, true, PRE>(LV, cx, cd, 4, tile * DWT_TL - 2, DWT_TL + 2, 2, L3,
                                          nullptr, P, 6);
}

// Persistent grid (about as many blocks as the CUs hold at once, each walking tiles with a
// grid stride): the per-tile blocks were short enough (~2.6 us) that the workgroup dispatcher,
// not HBM, bounded the launch (SQ_WAVE_CYCLES showed ~21 % of the wave slots in use).  Used for
// levels other than 4; level 4 runs dwt4_kernel below.
template <bool WX, bool WD, bool ACCUM>
__global__ void __launch_bounds__(256, DPZ_DWT_WAVES) dwt_kernel(const float* __restrict__ x,
                                                  const float* __restrict__ x0, Levels LV,
                                                  float* cx, float* cd, int64_t tile0,
                                                  int64_t ntiles) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int64_t n = LV.len[0];
  int64_t tile = tile0 + blockIdx.x;  // tiles [tile0, ntiles): a rank's share when sharded
  if (tile >= ntiles) return;
  float4 va[DWT_NG], vb[DWT_NG];
  int64_t s0, e0;
  dwt_span(LV, tile, &s0, &e0);
  dwt_span_load<WD>(x, x0, n, s0, e0, va, vb);
  for (;;) {
    dwt_span_store<WX, WD>(va, vb, n, s0, e0, smem);
    // the next tile's span loads are in flight while this tile's levels are computed
    const int64_t next = tile + gridDim.x;
    if (next < ntiles) {
      dwt_span(LV, next, &s0, &e0);
      dwt_span_load<WD>(x, x0, n, s0, e0, va, vb);
    }
    dwt_levels<WX, WD, ACCUM>(LV, cx, cd, tile, smem);
    __syncthreads();  // the next tile reuses the LDS buffers
    if (next >= ntiles) break;
    tile = next;
  }
}

// Level 4 (every shipped JWINS config): blocks [0, n_edge) first take one EDGE tile each — the
// tiles that touch an array end or start a sharded range ([tile0, a) and [b, tile_hi)) — on the
// span path above, without prefetch; then every block walks the INTERIOR tiles [a, b) on the
// register / vector-LDS path with the next tile's loads in flight.  Nothing is live across the
// two phases, so the span path's registers do not add to the interior loop's (94 VGPRs alone,
// 194 with both paths in one loop).
template <bool WX, bool WD, bool ACCUM>
__global__ void __launch_bounds__(256, (ACCUM && WD && DPZ_DWT_ACC_PRE) ? DPZ_DWT4_ACC_WAVES : DPZ_DWT4_WAVES) dwt4_kernel(const float* __restrict__ x,
                                                   const float* __restrict__ x0, Levels LV,
                                                   float* cx, float* cd, int64_t tile0,
                                                   int64_t a, int64_t b, int64_t tile_hi) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int64_t n = LV.len[0];
  const int64_t n_lo = a - tile0;
  if ((int64_t)blockIdx.x < n_lo + (tile_hi - b)) {
    const int64_t tile = (int64_t)blockIdx.x < n_lo ? tile0 + blockIdx.x : b + (blockIdx.x - n_lo);
    float4 va[DWT_NG], vb[DWT_NG];
    int64_t s0, e0;
    dwt_span(LV, tile, &s0, &e0);
    dwt_span_load<WD>(x, x0, n, s0, e0, va, vb);
    dwt_span_store<WX, WD>(va, vb, n, s0, e0, smem);
    dwt_levels<WX, WD, ACCUM>(LV, cx, cd, tile, smem);
    __syncthreads();
  }
  int64_t tile = a + blockIdx.x;
  if (tile >= b) return;
  float4 va[DWT_NG], vb[DWT_NG];
  float2 hx[DWT_NG], hb[DWT_NG];
  int64_t s0, e0;
  dwt_span(LV, tile, &s0, &e0);
  dwt_span_load<WD>(x, x0, n, s0, e0, va, vb);
  dwt_halo_load<WD>(x, x0, s0 & ~int64_t(3), hx, hb);
  constexpr bool PRE = ACCUM && WD && DPZ_DWT_ACC_PRE != 0;
  AccPre P;
  for (;;) {
    if constexpr (PRE) acc_prefetch(LV, cd, tile, P);  // before the next tile's span loads
    dwt_int_level1<WX, WD, ACCUM, PRE>(LV, cx, cd, tile, va, vb, hx, hb, smem, &P);
    // the next tile's loads are in flight while this tile's levels 2-4 are computed
    const int64_t next = tile + gridDim.x;
    if (next < b) {
      dwt_span(LV, next, &s0, &e0);
      dwt_span_load<WD>(x, x0, n, s0, e0, va, vb);
      dwt_halo_load<WD>(x, x0, s0 & ~int64_t(3), hx, hb);
    }
    __syncthreads();  // level-1 approximations in LDS
    dwt_int_levels234<WX, WD, ACCUM, PRE>(LV, cx, cd, tile, smem, &P);
    __syncthreads();  // the next tile reuses the LDS buffers
    if (next >= b) break;
    tile = next;
  }
}

// Inverse: a block owns final outputs [c, d) (a multiple of IDWT_TILE) and needs, per level l,
// the coefficients [cl[l], dl[l]) of cD_l (and of cA_L at the top).  Persistent blocks stage
// a tile's whole coefficient footprint (<= 4.2 K floats) into LDS, issue the NEXT tile's loads
// into registers, then rebuild the levels top-down from LDS (32-bit LDS-relative offsets).
__host__ __device__ constexpr int idwt_seg_max(int l) { return (IDWT_TILE >> l) + 4; }
__host__ __device__ constexpr int idwt_iters(int l) { return (idwt_seg_max(l) + 255) / 256; }
__host__ __device__ constexpr int idwt_doff(int l) {  // LDS offset of cD_l's segment
  int o = 0;
  for (int j = 1; j < l; ++j) o += idwt_seg_max(j);
  return o;
}
template <int LEV>
__host__ __device__ constexpr int idwt_npv() {
  int s = idwt_iters(LEV);
  for (int l = 1; l <= LEV; ++l) s += idwt_iters(l);
  return s;
}
constexpr int IDWT_SPAN = IDWT_TILE / 2 + 16;

struct IdwtRanges {
  int64_t cl[DWT_MAX_LEVEL + 1], dl[DWT_MAX_LEVEL + 1];
};

template <int LEV>
__device__ __forceinline__ IdwtRanges idwt_ranges(const Levels& LV, int64_t tile) {
  IdwtRanges R;
  const int64_t n = LV.len[0];
  R.cl[0] = tile * IDWT_TILE;
  R.dl[0] = (R.cl[0] + IDWT_TILE < n) ? R.cl[0] + IDWT_TILE : n;
#pragma unroll
  for (int l = 1; l <= LEV; ++l) {
    R.cl[l] = R.cl[l - 1] >> 1;
    R.dl[l] = ((R.dl[l - 1] - 1) >> 1) + 2;
    if (R.dl[l] > LV.len[l]) R.dl[l] = LV.len[l];
  }
  return R;
}

// the tile's coefficients into registers (cA_L first, then cD_1 .. cD_LEV); all loads issued
// before any is used
template <int LEV>
__device__ __forceinline__ void idwt_load(const float* __restrict__ coeffs, const Levels& LV,
                                          const IdwtRanges& R, float (&pv)[idwt_npv<LEV>()]) {
  // branch-free (a position past the range re-reads the range's first coefficient; idwt_stage
  // never stores it): one wait for the tile instead of one per guarded load in the ISA — the
  // same time on MI355X (41.1-41.9 vs 41.5-41.7 us at 25 M, profiles/r05_haar_idwt_ab.txt)
  const int t = threadIdx.x;
  int k = 0;
#pragma unroll
  for (int u = 0; u < idwt_iters(LEV); ++u, ++k) {
    const int64_t p = R.cl[LEV] + t + 256 * u;
    pv[k] = coeffs[p < R.dl[LEV] ? p : R.cl[LEV]];
  }
#pragma unroll
  for (int l = 1; l <= LEV; ++l) {
#pragma unroll
    for (int u = 0; u < idwt_iters(l); ++u, ++k) {
      const int64_t p = R.cl[l] + t + 256 * u;
      pv[k] = coeffs[LV.doff[l] + (p < R.dl[l] ? p : R.cl[l])];
    }
  }
}

template <int LEV>
__device__ __forceinline__ void idwt_stage(const IdwtRanges& R, const float (&pv)[idwt_npv<LEV>()],
                                           float* A, float* D) {
  const int t = threadIdx.x;
  int k = 0;
  const int na = (int)(R.dl[LEV] - R.cl[LEV]);
#pragma unroll
  for (int u = 0; u < idwt_iters(LEV); ++u, ++k) {
    const int r = t + 256 * u;
    if (r < na) A[r] = pv[k];
  }
#pragma unroll
  for (int l = 1; l <= LEV; ++l) {
    const int nd = (int)(R.dl[l] - R.cl[l]);
#pragma unroll
    for (int u = 0; u < idwt_iters(l); ++u, ++k) {
      const int r = t + 256 * u;
      if (r < nd) D[idwt_doff(l) + r] = pv[k];
    }
  }
}

template <int LEV>
__device__ __forceinline__ void idwt_levels(const Levels& LV, const IdwtRanges& R,
                                            float* __restrict__ out, float* A, float* B,
                                            const float* D) {
  float* a = A;
  float* bnext = B;
  const float r0 = c_rec_lo[0], r1 = c_rec_lo[1], r2 = c_rec_lo[2], r3 = c_rec_lo[3];
  const float h0 = c_rec_hi[0], h1 = c_rec_hi[1], h2 = c_rec_hi[2], h3 = c_rec_hi[3];
#pragma unroll
  for (int l = LEV; l >= 1; --l) {
    const float* dd = D + idwt_doff(l);
    int64_t q_hi = R.dl[l - 1];
    if (q_hi > LV.len[l - 1]) q_hi = LV.len[l - 1];
    const int nq = (int)(q_hi - R.cl[l - 1]);  // cl[l - 1] is even: m - cl[l] = qr >> 1
    float* const o1 = out + R.cl[0];
    for (int qr = threadIdx.x; qr < nq; qr += 256) {
      const int mr = qr >> 1;
      const float am = a[mr], am1 = a[mr + 1];
      const float dm = dd[mr], dm1 = dd[mr + 1];
      float ya, yd;
      if ((qr & 1) == 0) {
        ya = r0 * am1; ya = ya + r2 * am;
        yd = h0 * dm1; yd = yd + h2 * dm;
      } else {
        ya = r1 * am1; ya = ya + r3 * am;
        yd = h1 * dm1; yd = yd + h3 * dm;
      }
      const float y = ya + yd;
      if (l == 1) {
        if (DPZ_IDWT_NT) __builtin_nontemporal_store(y, o1 + qr);
        else o1[qr] = y;
      } else {
        bnext[qr] = y;
      }
    }
    if (l == 1) break;
    __syncthreads();
    float* tsw = a; a = bnext; bnext = tsw;
  }
}

template <int LEV>
__global__ void __launch_bounds__(256) idwt_kernel(const float* __restrict__ coeffs, Levels LV,
                                                   float* __restrict__ out, int64_t tile0,
                                                   int64_t ntiles) {
  __shared__ __attribute__((aligned(16))) float A[IDWT_SPAN];
  __shared__ __attribute__((aligned(16))) float B[IDWT_SPAN];
  // the detail segments of levels 1..LEV only: at LEV = 4 the block's LDS drops under 32 KB,
  // five blocks per CU instead of four
  __shared__ __attribute__((aligned(16))) float D[idwt_doff(LEV + 1)];
  int64_t tile = tile0 + blockIdx.x;
  if (tile >= ntiles) return;
  float pv[idwt_npv<LEV>()];
  IdwtRanges R = idwt_ranges<LEV>(LV, tile);
  idwt_load<LEV>(coeffs, LV, R, pv);
  for (;;) {
    idwt_stage<LEV>(R, pv, A, D);
    __syncthreads();
    const IdwtRanges Rc = R;
    const int64_t next = tile + gridDim.x;
    if (next < ntiles) {  // the next tile's loads are in flight while this one is rebuilt
      R = idwt_ranges<LEV>(LV, next);
      idwt_load<LEV>(coeffs, LV, R, pv);
    }
    idwt_levels<LEV>(LV, Rc, out, A, B, D);
    __syncthreads();  // the next tile reuses A / B / D
    if (next >= ntiles) break;
    tile = next;
  }
}

// blocks of the persistent grids: what the CUs hold at once for the kernel (occupancy API)
template <class K>
static unsigned persistent_grid(K kernel, size_t shm, int64_t ntiles) {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  int per = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, 256, shm) != hipSuccess || per < 1)
    per = 1;
  const int64_t g = (int64_t)cus * per;
  return (unsigned)(ntiles < g ? (ntiles > 0 ? ntiles : 1) : g);
}

static int dwt_levels_ok(int64_t n, int level) {
  if (level < 1 || level > DWT_MAX_LEVEL || n <= 0) return 0;
  int64_t len = n;
  for (int l = 1; l <= level; ++l) {
    if (len < 4) return 0;
    len = (len + 3) / 2;
  }
  return 1;
}

}  // namespace dpz

using namespace dpz;

extern "C" int64_t dpz_wavedec_len(int64_t n, int level) {
  if (!dwt_levels_ok(n, level)) return -1;
  return make_levels(n, level).total;
}

extern "C" int64_t dpz_dwt_tile_width(void) { return DWT_TL; }
extern "C" int64_t dpz_idwt_tile_width(void) { return IDWT_TILE; }

static int dwt_sym2_run(const float* x, const float* x0, int64_t n, int level, int64_t tile_lo,
                        int64_t tile_hi, float* coeffs_x, float* coeffs_diff, int accumulate,
                        const uint32_t* rmask, dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!x || n <= 0) return DPZ_ERR_ARG;
  if (!dwt_levels_ok(n, level) || level > 4) return DPZ_ERR_UNSUPPORTED;
  if (coeffs_diff && !x0) return DPZ_ERR_ARG;
  Levels LV = make_levels(n, level);
  LV.rmask = accumulate ? rmask : nullptr;
  const int64_t ntiles = (LV.len[level] + DWT_TL - 1) / DWT_TL;
  if (tile_lo < 0 || tile_hi > ntiles || tile_lo > tile_hi) return DPZ_ERR_ARG;
  if ((!coeffs_x && !coeffs_diff) || tile_lo == tile_hi) return DPZ_OK;
  constexpr int SPAN0 = 16 * DWT_TL + 64, SPAN1 = 8 * DWT_TL + 32;
  const size_t shm = 2 * (SPAN0 + SPAN1) * sizeof(float);
  const bool wx = coeffs_x != nullptr, wd = coeffs_diff != nullptr;
  const int64_t nt = tile_hi - tile_lo;
  const int tslot = timing_begin(DPZ_KT_DWT, st);
  if (level == 4) {
    int64_t a, b;
    dwt_interior_range(n, tile_lo, tile_hi, &a, &b);
    const int64_t nedge = (a - tile_lo) + (tile_hi - b);
#define DPZ_DWT4_LAUNCH(WXV, WDV, ACV)                                                           \
  {                                                                                              \
    int64_t g = persistent_grid(dwt4_kernel<WXV, WDV, ACV>, shm, b - a);                          \
    if (g < nedge) g = nedge;                                                                    \
    dwt4_kernel<WXV, WDV, ACV><<<(unsigned)g, 256, shm, st>>>(x, x0, LV, coeffs_x, coeffs_diff,  \
                                                             tile_lo, a, b, tile_hi);            \
  }
    if (wx && wd) {
      if (accumulate) DPZ_DWT4_LAUNCH(true, true, true) else DPZ_DWT4_LAUNCH(true, true, false)
    } else if (wx) {
      DPZ_DWT4_LAUNCH(true, false, false)
    } else {
      if (accumulate) DPZ_DWT4_LAUNCH(false, true, true) else DPZ_DWT4_LAUNCH(false, true, false)
    }
#undef DPZ_DWT4_LAUNCH
  } else if (wx && wd) {
    if (accumulate) dwt_kernel<true, true, true><<<persistent_grid(dwt_kernel<true, true, true>, shm, nt), 256, shm, st>>>(x, x0, LV, coeffs_x, coeffs_diff, tile_lo, tile_hi);
    else dwt_kernel<true, true, false><<<persistent_grid(dwt_kernel<true, true, false>, shm, nt), 256, shm, st>>>(x, x0, LV, coeffs_x, coeffs_diff, tile_lo, tile_hi);
  } else if (wx) {
    dwt_kernel<true, false, false><<<persistent_grid(dwt_kernel<true, false, false>, shm, nt), 256, shm, st>>>(x, x0, LV, coeffs_x, nullptr, tile_lo, tile_hi);
  } else {
    if (accumulate) dwt_kernel<false, true, true><<<persistent_grid(dwt_kernel<false, true, true>, shm, nt), 256, shm, st>>>(x, x0, LV, nullptr, coeffs_diff, tile_lo, tile_hi);
    else dwt_kernel<false, true, false><<<persistent_grid(dwt_kernel<false, true, false>, shm, nt), 256, shm, st>>>(x, x0, LV, nullptr, coeffs_diff, tile_lo, tile_hi);
  }
  DPZ_LAUNCH_CHECK();
  timing_end(tslot, st);
  return DPZ_OK;
}

extern "C" int dpz_dwt_sym2_tiles(const float* x, const float* x0, int64_t n, int level,
                                  int64_t tile_lo, int64_t tile_hi, float* coeffs_x,
                                  float* coeffs_diff, int accumulate, dpz_stream_t stream) {
  return dwt_sym2_run(x, x0, n, level, tile_lo, tile_hi, coeffs_x, coeffs_diff, accumulate,
                      nullptr, stream);
}

extern "C" int dpz_dwt_sym2(const float* x, const float* x0, int64_t n, int level,
                            float* coeffs_x, float* coeffs_diff, int accumulate,
                            dpz_stream_t stream) {
  if (!x || n <= 0) return DPZ_ERR_ARG;
  if (!dwt_levels_ok(n, level) || level > 4) return DPZ_ERR_UNSUPPORTED;
  const Levels LV = make_levels(n, level);
  const int64_t ntiles = (LV.len[level] + DWT_TL - 1) / DWT_TL;
  return dwt_sym2_run(x, x0, n, level, 0, ntiles, coeffs_x, coeffs_diff, accumulate, nullptr,
                      stream);
}

extern "C" int dpz_dwt_sym2_rewind(const float* x, const float* x0, int64_t n, int level,
                                   float* acc, const uint32_t* sel_mask, dpz_stream_t stream) {
  if (!x || !x0 || !acc || !sel_mask || n <= 0) return DPZ_ERR_ARG;
  if (!dwt_levels_ok(n, level) || level > 4) return DPZ_ERR_UNSUPPORTED;
  const Levels LV = make_levels(n, level);
  const int64_t ntiles = (LV.len[level] + DWT_TL - 1) / DWT_TL;
  return dwt_sym2_run(x, x0, n, level, 0, ntiles, nullptr, acc, 1, sel_mask, stream);
}

extern "C" int dpz_idwt_sym2_tiles(const float* coeffs, int64_t n, int level, int64_t tile_lo,
                                   int64_t tile_hi, float* out, dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!coeffs || !out || n <= 0) return DPZ_ERR_ARG;
  if (!dwt_levels_ok(n, level)) return DPZ_ERR_UNSUPPORTED;
  const Levels LV = make_levels(n, level);
  const int64_t ntiles = (n + IDWT_TILE - 1) / IDWT_TILE;
  if (tile_lo < 0 || tile_hi > ntiles || tile_lo > tile_hi) return DPZ_ERR_ARG;
  if (tile_lo == tile_hi) return DPZ_OK;
  const int64_t nt = tile_hi - tile_lo;
  switch (level) {
#define DPZ_IDWT_CASE(LEVN)                                                                    \
  case LEVN:                                                                                   \
    DPZ_TIMED(DPZ_KT_IDWT, st, idwt_kernel<LEVN><<<persistent_grid(idwt_kernel<LEVN>, 0, nt), \
                                                  256, 0, st>>>(coeffs, LV, out, tile_lo,      \
                                                                tile_hi));                     \
    break;
    DPZ_IDWT_CASE(1) DPZ_IDWT_CASE(2) DPZ_IDWT_CASE(3) DPZ_IDWT_CASE(4)
    DPZ_IDWT_CASE(5) DPZ_IDWT_CASE(6) DPZ_IDWT_CASE(7) DPZ_IDWT_CASE(8)
#undef DPZ_IDWT_CASE
    default:
      return DPZ_ERR_UNSUPPORTED;
  }
  return DPZ_OK;
}

extern "C" int dpz_idwt_sym2(const float* coeffs, int64_t n, int level, float* out,
                             dpz_stream_t stream) {
  if (n <= 0) return DPZ_ERR_ARG;
  return dpz_idwt_sym2_tiles(coeffs, n, level, 0, (n + IDWT_TILE - 1) / IDWT_TILE, out, stream);
}
