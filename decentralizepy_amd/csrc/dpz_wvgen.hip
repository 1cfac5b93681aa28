// Generic-filter multilevel DWT / IDWT (mode "symmetric"), fp32, bit-exact with PyWavelets 1.1.1
// for every pywt discrete wavelet with an even filter length F <= 64 (db1-32, sym2-20, coif1-10,
// bior / rbio, dmey) — the wavelets other than sym2 (dpz_dwt.hip) and haar (dpz_haar.hip).
//
// Replaces (reference sacs-epfl/decentralizepy, src/decentralizepy/):
//   sharing/JWINS/Wavelet.py:12-32   change_transformer_wavelet: pywt.wavedec + coeffs_to_array
//   sharing/JWINS/Wavelet.py:311-316 pywt.array_to_coeffs + pywt.waverec
//   sharing/PartialModel.py:346-349  acc += W(x_new - prev) (accumulate mode, optional rewind)
//
// The filter bank is a DEVICE array of 4F floats (dec_lo, dec_hi, rec_lo, rec_hi: the fp32 taps
// pywt applies to float32 data, decentralizepy_amd/wavelet_filters.json); every tap index in the
// loops below is wave-uniform, so the taps are scalar loads.
//
// Forward, one launch per level and stream (x, or x - x0 formed on the fly at level 1; deeper
// levels read the previous approximation from the workspace), one thread per output pair
// (approximation, detail) sharing the F input reads.  pywt's downsampling_convolution order, every
// sum started from 0 (its `TYPE sum = 0`), x~ the half-sample symmetric extension:
//   i = 2o + 1 < n : sum_{j = 0 .. F-1} f[j] x~[i - j]            (j ascending)
//   i >= n         : e = i - n + 1; j = e-1 .. 0 (the extension terms), then j = e .. F-1
// Every level's input must hold >= F values (one reflection per side; pywt's multi-reflection
// branch for shorter inputs is not needed by model-sized vectors and is refused).
// Inverse, one launch per level: pywt's upsampling_convolution_valid_sf, a into a zeroed output
// then d added:  y[2m + p] = (0 + sum_{j < F/2} r[2j+p] a[m+F/2-1-j]) + sum_{j < F/2} h[2j+p] d[..]
// writing exactly the next level's length (pywt's one-longer trim) and, at level 1, n outputs.
// Layout [cA_L, cD_L, ..., cD_1] (pywt.coeffs_to_array), len_l = floor((len_{l-1} + F - 1) / 2).
// Performance is a non-goal beyond coalescing: the shipped configs run the fused sym2 kernels.
#include "dpz_common.h"

namespace dpz {

constexpr int WG_FMAX = 64;
constexpr int WG_LMAX = 8;

struct WgLevels {
  int64_t len[WG_LMAX + 1];
  int64_t doff[WG_LMAX + 1];  // offset of cD_l in the coefficient array
  int64_t total;
};

static bool wg_levels(int64_t n, int level, int F, WgLevels* L) {
  if (n <= 0 || level < 1 || level > WG_LMAX || F < 2 || F > WG_FMAX || (F & 1)) return false;
  L->len[0] = n;
  for (int l = 1; l <= level; ++l) {
    if (L->len[l - 1] < F) return false;
    L->len[l] = (L->len[l - 1] + F - 1) / 2;
  }
  int64_t o = L->len[level];
  for (int l = level; l >= 1; --l) {
    L->doff[l] = o;
    o += L->len[l];
  }
  L->total = o;
  return true;
}

static size_t wg_ws_floats(const WgLevels& L, int level) {
  // two streams x two ping-pong approximation buffers of the longest intermediate level
  return level >= 2 ? (size_t)4 * (size_t)L.len[1] : 0;
}

__device__ __forceinline__ int64_t wg_ext(int64_t p, int64_t n) {
  return p < 0 ? -1 - p : (p >= n ? 2 * n - 1 - p : p);
}

// the accumulator's value before this pass adds to it: +0 where the encode selected it (the
// deferred rewind of dpz_topk_encode_sliced, as in dpz_dwt.hip)
__device__ __forceinline__ float wg_acc_before(const float* dst, const uint32_t* rmask,
                                               int64_t pos) {
  if (rmask && ((rmask[pos >> 5] >> (pos & 31)) & 1u)) return 0.0f;
  return *dst;
}

// DIFF: the input is in - in0 (level 1 of W(x - x0)).  aout / dout: approximation / detail of
// this level (aout may be the workspace); ACC: adds into the coefficient array instead (the
// approximation only at the top level, atop = true), apos / dpos their coefficient positions.
template <bool DIFF, bool ACC>
__global__ void __launch_bounds__(256) wg_dwt_kernel(const float* __restrict__ in,
                                                     const float* __restrict__ in0, int64_t n,
                                                     int64_t nout, const float* __restrict__ bank,
                                                     int F, float* aout, bool atop, int64_t apos,
                                                     float* dout, int64_t dpos,
                                                     const uint32_t* __restrict__ rmask) {
  const int64_t o = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (o >= nout) return;
  const float* __restrict__ lo = bank;
  const float* __restrict__ hi = bank + F;
  auto X = [&](int64_t p) {
    const int64_t q = wg_ext(p, n);
    return DIFF ? in[q] - in0[q] : in[q];
  };
  const int64_t i = 2 * o + 1;
  float sa = 0.0f, sd = 0.0f;
  if (i < n) {
    for (int j = 0; j < F; ++j) {
      const float v = X(i - j);
      sa = sa + lo[j] * v;
      sd = sd + hi[j] * v;
    }
  } else {
    const int e = (int)(i - n + 1);
    for (int j = e - 1; j >= 0; --j) {
      const float v = X(i - j);
      sa = sa + lo[j] * v;
      sd = sd + hi[j] * v;
    }
    for (int j = e; j < F; ++j) {
      const float v = X(i - j);
      sa = sa + lo[j] * v;
      sd = sd + hi[j] * v;
    }
  }
  if (ACC && atop) aout[o] = wg_acc_before(aout + o, rmask, apos + o) + sa;
  else aout[o] = sa;
  if (ACC) dout[o] = wg_acc_before(dout + o, rmask, dpos + o) + sd;
  else dout[o] = sd;
}

__global__ void __launch_bounds__(256) wg_idwt_kernel(const float* __restrict__ a,
                                                      const float* __restrict__ d, int64_t nout,
                                                      const float* __restrict__ bank, int F,
                                                      float* __restrict__ out) {
  const int64_t o = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (o >= nout) return;
  const float* __restrict__ rl = bank + 2 * F;
  const float* __restrict__ rh = bank + 3 * F;
  const int F2 = F >> 1;
  const int64_t m = o >> 1;
  const int p = (int)(o & 1);
  float sa = 0.0f, sd = 0.0f;
  for (int j = 0; j < F2; ++j) {
    sa = sa + rl[2 * j + p] * a[m + F2 - 1 - j];
    sd = sd + rh[2 * j + p] * d[m + F2 - 1 - j];
  }
  float y = 0.0f + sa;
  y = y + sd;
  out[o] = y;
}

static unsigned wg_grid(int64_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace dpz

using namespace dpz;

extern "C" int64_t dpz_wavedec_len_generic(int64_t n, int level, int flen) {
  WgLevels L;
  return wg_levels(n, level, flen, &L) ? L.total : -1;
}

extern "C" size_t dpz_wavelet_generic_workspace_bytes(int64_t n, int level, int flen) {
  WgLevels L;
  if (!wg_levels(n, level, flen, &L)) return 0;
  return wg_ws_floats(L, level) * sizeof(float);
}

extern "C" int dpz_dwt_generic(const float* x, const float* x0, int64_t n, int level,
                               const float* bank, int flen, float* coeffs_x, float* coeffs_diff,
                               int accumulate, const uint32_t* sel_mask, void* ws,
                               size_t ws_bytes, dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!x || !bank || n <= 0) return DPZ_ERR_ARG;
  WgLevels L;
  if (!wg_levels(n, level, flen, &L)) return DPZ_ERR_UNSUPPORTED;
  if (coeffs_diff && !x0) return DPZ_ERR_ARG;
  if (accumulate && !coeffs_diff) return DPZ_ERR_ARG;
  if (sel_mask && !accumulate) return DPZ_ERR_ARG;
  if (!coeffs_x && !coeffs_diff) return DPZ_OK;
  if (level >= 2 && (!ws || ws_bytes < wg_ws_floats(L, level) * sizeof(float)))
    return DPZ_ERR_WORKSPACE;
  float* const wsf = static_cast<float*>(ws);
  const int tslot = timing_begin(DPZ_KT_DWT, st);
  for (int s = 0; s < 2; ++s) {  // stream 0: W(x), stream 1: W(x - x0)
    float* const coeffs = s == 0 ? coeffs_x : coeffs_diff;
    if (!coeffs) continue;
    const bool acc = s == 1 && accumulate;
    const float* in = x;
    for (int l = 1; l <= level; ++l) {
      const bool top = l == level;
      // intermediate approximations ping-pong in the workspace: stream s, buffer (l & 1)
      float* const aout = top ? coeffs : wsf + ((size_t)(2 * s + (l & 1)) * (size_t)L.len[1]);
      const int64_t nout = L.len[l];
      const bool diff = s == 1 && l == 1;
      float* const dout = coeffs + L.doff[l];
#define DPZ_WG_DWT(DF, AC)                                                                     \
  wg_dwt_kernel<DF, AC><<<wg_grid(nout), 256, 0, st>>>(in, x0, L.len[l - 1], nout, bank, flen, \
                                                       aout, top, 0, dout, L.doff[l], sel_mask)
      if (diff) {
        if (acc) DPZ_WG_DWT(true, true);
        else DPZ_WG_DWT(true, false);
      } else {
        if (acc) DPZ_WG_DWT(false, true);
        else DPZ_WG_DWT(false, false);
      }
#undef DPZ_WG_DWT
      DPZ_LAUNCH_CHECK();
      in = aout;
    }
  }
  timing_end(tslot, st);
  return DPZ_OK;
}

extern "C" int dpz_idwt_generic(const float* coeffs, int64_t n, int level, const float* bank,
                                int flen, float* out, void* ws, size_t ws_bytes,
                                dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!coeffs || !out || !bank || n <= 0) return DPZ_ERR_ARG;
  WgLevels L;
  if (!wg_levels(n, level, flen, &L)) return DPZ_ERR_UNSUPPORTED;
  if (level >= 2 && (!ws || ws_bytes < wg_ws_floats(L, level) * sizeof(float)))
    return DPZ_ERR_WORKSPACE;
  float* const wsf = static_cast<float*>(ws);
  const int tslot = timing_begin(DPZ_KT_IDWT, st);
  const float* a = coeffs;  // cA_L
  for (int l = level; l >= 1; --l) {
    // y has 2 (len_l - F/2 + 1) values = len_{l-1} or len_{l-1} + 1: pywt trims the one extra
    // before the next level, and the caller keeps n of the last
    const int64_t nout = L.len[l - 1];
    float* const y = l == 1 ? out : wsf + (size_t)(l & 1) * (size_t)L.len[1];
    wg_idwt_kernel<<<wg_grid(nout), 256, 0, st>>>(a, coeffs + L.doff[l], nout, bank, flen, y);
    DPZ_LAUNCH_CHECK();
    a = y;
  }
  timing_end(tslot, st);
  return DPZ_OK;
}
