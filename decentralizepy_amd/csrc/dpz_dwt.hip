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
#endif  // level-L outputs per block (forward)
constexpr int IDWT_TILE = 4096;

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
};

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
          if (ACCUM) cdd[r] = cdd[r] + dv; else cdd[r] = dv;
        }
        if (l == L && own) {
          const float av = conv4r(in[1], i, c_dec_lo, lo_odd);
          if (ACCUM) cda[r] = cda[r] + av; else cda[r] = av;
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

// Persistent grid (about as many blocks as the CUs hold at once, each walking tiles with a
// grid stride): the per-tile blocks were short enough (~2.6 us) that the workgroup dispatcher,
// not HBM, bounded the launch (SQ_WAVE_CYCLES showed ~21 % of the wave slots in use).
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
constexpr int IDWT_DALL = idwt_doff(DWT_MAX_LEVEL + 1);

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
  const int t = threadIdx.x;
  int k = 0;
#pragma unroll
  for (int u = 0; u < idwt_iters(LEV); ++u, ++k) {
    const int64_t p = R.cl[LEV] + t + 256 * u;
    pv[k] = p < R.dl[LEV] ? coeffs[p] : 0.0f;
  }
#pragma unroll
  for (int l = 1; l <= LEV; ++l) {
#pragma unroll
    for (int u = 0; u < idwt_iters(l); ++u, ++k) {
      const int64_t p = R.cl[l] + t + 256 * u;
      pv[k] = p < R.dl[l] ? coeffs[LV.doff[l] + p] : 0.0f;
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
      if (l == 1) o1[qr] = y; else bnext[qr] = y;
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
  __shared__ __attribute__((aligned(16))) float D[IDWT_DALL];
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

extern "C" int dpz_dwt_sym2_tiles(const float* x, const float* x0, int64_t n, int level,
                                  int64_t tile_lo, int64_t tile_hi, float* coeffs_x,
                                  float* coeffs_diff, int accumulate, dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!x || n <= 0) return DPZ_ERR_ARG;
  if (!dwt_levels_ok(n, level) || level > 4) return DPZ_ERR_UNSUPPORTED;
  if (coeffs_diff && !x0) return DPZ_ERR_ARG;
  const Levels LV = make_levels(n, level);
  const int64_t ntiles = (LV.len[level] + DWT_TL - 1) / DWT_TL;
  if (tile_lo < 0 || tile_hi > ntiles || tile_lo > tile_hi) return DPZ_ERR_ARG;
  if ((!coeffs_x && !coeffs_diff) || tile_lo == tile_hi) return DPZ_OK;
  constexpr int SPAN0 = 16 * DWT_TL + 64, SPAN1 = 8 * DWT_TL + 32;
  const size_t shm = 2 * (SPAN0 + SPAN1) * sizeof(float);
  const bool wx = coeffs_x != nullptr, wd = coeffs_diff != nullptr;
  const int64_t nt = tile_hi - tile_lo;
  const int tslot = timing_begin(DPZ_KT_DWT, st);
  if (wx && wd) {
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

extern "C" int dpz_dwt_sym2(const float* x, const float* x0, int64_t n, int level,
                            float* coeffs_x, float* coeffs_diff, int accumulate,
                            dpz_stream_t stream) {
  if (!x || n <= 0) return DPZ_ERR_ARG;
  if (!dwt_levels_ok(n, level) || level > 4) return DPZ_ERR_UNSUPPORTED;
  const Levels LV = make_levels(n, level);
  const int64_t ntiles = (LV.len[level] + DWT_TL - 1) / DWT_TL;
  return dpz_dwt_sym2_tiles(x, x0, n, level, 0, ntiles, coeffs_x, coeffs_diff, accumulate,
                            stream);
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
