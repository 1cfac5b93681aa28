// Multilevel Haar DWT / IDWT (mode "symmetric"), fp32, bit-exact with PyWavelets 1.1.1 — the
// reference Wavelet plugin's DEFAULT wavelet (sharing/JWINS/Wavelet.py:56, wavelet="haar").
//
// Replaces (reference sacs-epfl/decentralizepy, src/decentralizepy/):
//   sharing/JWINS/Wavelet.py:12-32   pywt.wavedec(x, "haar", level) + coeffs_to_array
//   sharing/JWINS/Wavelet.py:311-316 pywt.array_to_coeffs + pywt.waverec(.., "haar")
//   sharing/PartialModel.py:317-320  W(x) and W(x - x0) in one pass; :346-349 acc += W(x - prev)
//
// pywt's order for the 2-tap filters (verified against PyWavelets 1.1.1, oracle/wavelet.py):
//   forward  out[o] = f0 * x~[2o + 1] + f1 * x~[2o]       x~[len] = x[len - 1] (odd len only)
//   inverse  y[2m + p] = rec_lo[p] * a[m] + rec_hi[p] * d[m]
// Level lengths len_l = ceil(len_{l-1} / 2); an approximation one longer than its detail array is
// trimmed (waverec), which only drops a tail value.
//
// Haar supports do not overlap, so no halo exists: a wave owns a chunk of 256 inputs (one float4
// per lane and input stream) and every output of every level that depends on it.  Levels 1-2 stay
// in the lane's registers (4 inputs -> 2 -> 1), levels 3..8 pair values across lanes with
// shuffles.  The inverse rebuilds each lane's 4 outputs top-down from the coefficients that cover
// them (the few coarse-level loads are shared by neighbouring lanes through the L1).
#include "dpz_common.h"

namespace dpz {

constexpr int HAAR_MAX_LEVEL = 8;
constexpr int HAAR_CHUNK = 256;  // level-0 values per wave chunk
constexpr int HAAR_UNROLL = 4;   // chunks whose loads a wave issues before computing

__constant__ float c_haar[2] = {0.7071067811865476f, 0.7071067811865476f};  // |dec_lo| = rec_lo

struct HaarLevels {
  int64_t len[HAAR_MAX_LEVEL + 1];
  int64_t doff[HAAR_MAX_LEVEL + 1];
  int64_t total;
  int level;
  const uint32_t* rmask;  // dpz_dwt_haar_rewind: acc = (selected ? 0 : acc) + c
};

// the accumulator before this pass adds to it: 0 at a coefficient the encode selected (the
// deferred rewind; 0 + c as the reference computes it)
__device__ __forceinline__ float hacc_before(const HaarLevels& LV, const float* base,
                                             const float* p) {
  const float o = *p;
  const int64_t pos = p - base;
  if (LV.rmask && ((LV.rmask[pos >> 5] >> (pos & 31)) & 1u)) return 0.0f;
  return o;
}

static inline HaarLevels haar_levels(int64_t n, int level) {
  HaarLevels L{};
  L.level = level;
  L.len[0] = n;
  for (int l = 1; l <= level; ++l) L.len[l] = (L.len[l - 1] + 1) / 2;
  int64_t o = L.len[level];
  for (int l = level; l >= 1; --l) {
    L.doff[l] = o;
    o += L.len[l];
  }
  L.total = o;
  return L;
}

// The accumulating pipeline's outputs of a chunk (acc += W(x - prev) with the deferred rewind)
// are collected in compile-time slots and their accumulator words (and mask words) loaded
// together, one round trip per chunk: read at each store instead, every output waited on its own
// load with vmcnt(0) (seen in the ISA), which also waited for the chunk's earlier stores.
// Slots: 0-1 level-1 detail, 2-3 level-1 approximation (L = 1), 4 level-2 detail, 5 level-2
// approximation (L = 2), 6 + (l - 3) level-l detail (l = 3..8), 12 the level-L approximation
// (L >= 3).
#ifndef DPZ_HAAR_ACC_BATCH
#define DPZ_HAAR_ACC_BATCH 1
#endif
constexpr int HAAR_SLOTS = 13;
struct HaarAcc {
  float v[HAAR_SLOTS];
  int64_t pos[HAAR_SLOTS];
  bool on[HAAR_SLOTS];
};

template <bool WX, bool WD, bool ACCUM>
__global__ void __launch_bounds__(256) haar_dwt_kernel(const float* __restrict__ x,
                                                       const float* __restrict__ x0, HaarLevels LV,
                                                       float* cx, float* cd, int64_t nchunks,
                                                       int vec) {
  constexpr bool BATCH = ACCUM && WD && DPZ_HAAR_ACC_BATCH != 0;
  const int lane = threadIdx.x & 63;
  const int64_t n = LV.len[0];
  const int L = LV.level;
  const float h = c_haar[0];
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  for (int64_t c0 = wave * HAAR_UNROLL; c0 < nchunks; c0 += nwaves * HAAR_UNROLL) {
    float4 va[HAAR_UNROLL], vb[HAAR_UNROLL];
#pragma unroll
    for (int u = 0; u < HAAR_UNROLL; ++u) {
      const int64_t p = (c0 + u) * HAAR_CHUNK + 4 * lane;
      va[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      vb[u] = va[u];
      if (c0 + u < nchunks) {
        if (vec && p + 4 <= n) {
          va[u] = *reinterpret_cast<const float4*>(x + p);
          if (WD) vb[u] = *reinterpret_cast<const float4*>(x0 + p);
        } else {
          float ta[4] = {0.f, 0.f, 0.f, 0.f}, tb[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (p + e < n) {
              ta[e] = x[p + e];
              if (WD) tb[e] = x0[p + e];
            }
          va[u] = make_float4(ta[0], ta[1], ta[2], ta[3]);
          vb[u] = make_float4(tb[0], tb[1], tb[2], tb[3]);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < HAAR_UNROLL; ++u) {
      const int64_t c = c0 + u;
      if (c >= nchunks) break;  // wave-uniform
      const int64_t p = c * HAAR_CHUNK + 4 * lane;
      HaarAcc A;
      if constexpr (BATCH) {
#pragma unroll
        for (int q = 0; q < HAAR_SLOTS; ++q) {
          A.on[q] = false;
          A.pos[q] = 0;
          A.v[q] = 0.0f;
        }
      }
      // an output of pipeline s at coefficient position ps: stored now, or (the accumulating
      // pipeline) kept in slot q for the chunk's batched read-modify-write
      auto emit = [&](int s, int q, int64_t ps, float val) {
        float* out = s == 0 ? cx : cd;
        if (ACCUM && s == 1) {
          if constexpr (BATCH) {
            A.on[q] = true;
            A.pos[q] = ps;
            A.v[q] = val;
          } else {
            out[ps] = hacc_before(LV, out, out + ps) + val;
          }
        } else {
          out[ps] = val;
        }
      };
      // pipelines: 0 = x, 1 = x - x0
      float v[2][4];
      v[0][0] = va[u].x; v[0][1] = va[u].y; v[0][2] = va[u].z; v[0][3] = va[u].w;
      if (WD) {
        v[1][0] = va[u].x - vb[u].x; v[1][1] = va[u].y - vb[u].y;
        v[1][2] = va[u].z - vb[u].z; v[1][3] = va[u].w - vb[u].w;
      }
      // symmetric extension of an odd level-0 length: x~[n] = x[n - 1] (same lane)
      if (p + 1 == n) { v[0][1] = v[0][0]; v[1][1] = v[1][0]; }
      if (p + 3 == n) { v[0][3] = v[0][2]; v[1][3] = v[1][2]; }
      // level 1: positions q, q + 1 (q = p / 2)
      const int64_t q = p >> 1;
      float lo1[2][2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        if (s == 0 && !WX) continue;
        if (s == 1 && !WD) continue;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float a = v[s][2 * j], b = v[s][2 * j + 1];
          float lo = h * b;
          lo = lo + h * a;
          float hi = (-h) * b;
          hi = hi + h * a;
          lo1[s][j] = lo;
          if (q + j < LV.len[1]) {
            if (L == 1) emit(s, 2 + j, q + j, lo);
            emit(s, j, LV.doff[1] + q + j, hi);
          }
        }
      }
      if (L > 1) {
        // level 2: position r = p / 4 from the lane's two level-1 values
        const int64_t r = p >> 2;
        float cur[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          if (s == 0 && !WX) continue;
          if (s == 1 && !WD) continue;
          const float a = lo1[s][0];
          const float b = (q + 1 == LV.len[1]) ? a : lo1[s][1];
          float lo = h * b;
          lo = lo + h * a;
          float hi = (-h) * b;
          hi = hi + h * a;
          cur[s] = lo;
          if (r < LV.len[2]) {
            if (L == 2) emit(s, 5, r, lo);
            emit(s, 4, LV.doff[2] + r, hi);
          }
        }
        // levels 3..L: lane pairs (stride s2) across the wave; the lane holds the level-(l-1)
        // value at position r >> (l - 3) when lane % s2 == 0
#pragma unroll
        for (int l = 3; l <= HAAR_MAX_LEVEL; ++l) {
          if (l > L) break;  // uniform
          const int s2 = 1 << (l - 3);
          const int64_t pos = r >> (l - 3);        // this lane's level-(l-1) position (if active)
          const int64_t o = pos >> 1;              // level-l output position
          const bool active = (lane & (2 * s2 - 1)) == 0;
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            if (s == 0 && !WX) continue;
            if (s == 1 && !WD) continue;
            const float other = __shfl_down(cur[s], s2, 64);
            if (active) {
              const float a = cur[s];
              const float b = (pos + 1 == LV.len[l - 1]) ? a : other;
              float lo = h * b;
              lo = lo + h * a;
              float hi = (-h) * b;
              hi = hi + h * a;
              cur[s] = lo;
              if (o < LV.len[l]) {
                if (l == L) emit(s, 12, o, lo);
                emit(s, 6 + (l - 3), LV.doff[l] + o, hi);
              }
            }
          }
        }
      }
      if constexpr (BATCH) {
        // the chunk's accumulator and mask words, all loads issued before any is used
        // (branch-free: an unused slot re-reads word 0), then the stores
        float o[HAAR_SLOTS];
        uint32_t m[HAAR_SLOTS];
#pragma unroll
        for (int k = 0; k < HAAR_SLOTS; ++k) {
          const int64_t ps = A.on[k] ? A.pos[k] : 0;
          o[k] = cd[ps];
          m[k] = LV.rmask ? LV.rmask[ps >> 5] : 0u;
        }
#pragma unroll
        for (int k = 0; k < HAAR_SLOTS; ++k) {
          if (A.on[k]) {
            const int64_t ps = A.pos[k];
            const float before = ((m[k] >> (ps & 31)) & 1u) ? 0.0f : o[k];
            cd[ps] = before + A.v[k];
          }
        }
      }
    }
  }
}

// inverse: lane t of chunk c writes outputs Q0 .. Q0 + 3 (Q0 = 256 c + 4 t)
template <int LEV>
__global__ void __launch_bounds__(256) haar_idwt_kernel(const float* __restrict__ coeffs,
                                                        HaarLevels LV, float* __restrict__ out,
                                                        int64_t nchunks, int vec) {
  const int lane = threadIdx.x & 63;
  const int64_t n = LV.len[0];
  const float h = c_haar[0];
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  for (int64_t c = wave; c < nchunks; c += nwaves) {
    const int64_t Q0 = c * HAAR_CHUNK + 4 * lane;
    if (Q0 >= n) continue;
    // level-1 approximations at positions Q0/2 and Q0/2 + 1
    float a10, a11;
    const int64_t m1 = Q0 >> 1;
    if (LEV == 1) {
      a10 = coeffs[m1];
      a11 = (m1 + 1 < LV.len[1]) ? coeffs[m1 + 1] : 0.f;
    } else {
      float a = coeffs[Q0 >> LEV];  // cA_LEV
#pragma unroll
      for (int l = LEV; l >= 3; --l) {
        const int64_t P = Q0 >> (l - 1);
        const float d = coeffs[LV.doff[l] + (P >> 1)];
        float ya, yd;
        if (P & 1) { ya = h * a; yd = (-h) * d; } else { ya = h * a; yd = h * d; }
        a = ya + yd;
      }
      const int64_t m2 = Q0 >> 2;
      const float d2 = coeffs[LV.doff[2] + m2];
      a10 = h * a;
      a10 = a10 + h * d2;
      a11 = h * a;
      a11 = a11 + (-h) * d2;
    }
    const float d10 = coeffs[LV.doff[1] + m1];
    const float d11 = (m1 + 1 < LV.len[1]) ? coeffs[LV.doff[1] + m1 + 1] : 0.f;
    float y[4];
    y[0] = h * a10; y[0] = y[0] + h * d10;
    y[1] = h * a10; y[1] = y[1] + (-h) * d10;
    y[2] = h * a11; y[2] = y[2] + h * d11;
    y[3] = h * a11; y[3] = y[3] + (-h) * d11;
    if (vec && Q0 + 4 <= n) {
      typedef float v4f __attribute__((ext_vector_type(4)));
      const v4f v = {y[0], y[1], y[2], y[3]};  // written once: non-temporal, as the sym2 IDWT
      __builtin_nontemporal_store(v, reinterpret_cast<v4f*>(out + Q0));
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (Q0 + e < n) out[Q0 + e] = y[e];
    }
  }
}

static unsigned haar_grid(int64_t waves_needed) {
  int64_t g = (waves_needed + 3) / 4;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (unsigned)g;
}

}  // namespace dpz

using namespace dpz;

extern "C" int64_t dpz_haar_wavedec_len(int64_t n, int level) {
  if (n <= 0 || level < 1 || level > HAAR_MAX_LEVEL) return -1;
  return haar_levels(n, level).total;
}

static int dwt_haar_run(const float* x, const float* x0, int64_t n, int level, float* coeffs_x,
                        float* coeffs_diff, int accumulate, const uint32_t* rmask,
                        dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!x || n <= 0) return DPZ_ERR_ARG;
  if (level < 1 || level > HAAR_MAX_LEVEL) return DPZ_ERR_UNSUPPORTED;
  if (coeffs_diff && !x0) return DPZ_ERR_ARG;
  if (!coeffs_x && !coeffs_diff) return DPZ_OK;
  HaarLevels LV = haar_levels(n, level);
  LV.rmask = accumulate ? rmask : nullptr;
  const int64_t nchunks = (n + HAAR_CHUNK - 1) / HAAR_CHUNK;
  const int vec = aligned16(x) && (!coeffs_diff || aligned16(x0));
  const unsigned g = haar_grid((nchunks + HAAR_UNROLL - 1) / HAAR_UNROLL);
  const bool wx = coeffs_x != nullptr, wd = coeffs_diff != nullptr;
  const int tslot = timing_begin(DPZ_KT_HAAR, st);
  if (wx && wd) {
    if (accumulate) haar_dwt_kernel<true, true, true><<<g, 256, 0, st>>>(x, x0, LV, coeffs_x, coeffs_diff, nchunks, vec);
    else haar_dwt_kernel<true, true, false><<<g, 256, 0, st>>>(x, x0, LV, coeffs_x, coeffs_diff, nchunks, vec);
  } else if (wx) {
    haar_dwt_kernel<true, false, false><<<g, 256, 0, st>>>(x, x0, LV, coeffs_x, nullptr, nchunks, vec);
  } else {
    if (accumulate) haar_dwt_kernel<false, true, true><<<g, 256, 0, st>>>(x, x0, LV, nullptr, coeffs_diff, nchunks, vec);
    else haar_dwt_kernel<false, true, false><<<g, 256, 0, st>>>(x, x0, LV, nullptr, coeffs_diff, nchunks, vec);
  }
  DPZ_LAUNCH_CHECK();
  timing_end(tslot, st);
  return DPZ_OK;
}

extern "C" int dpz_dwt_haar(const float* x, const float* x0, int64_t n, int level,
                            float* coeffs_x, float* coeffs_diff, int accumulate,
                            dpz_stream_t stream) {
  return dwt_haar_run(x, x0, n, level, coeffs_x, coeffs_diff, accumulate, nullptr, stream);
}

extern "C" int dpz_dwt_haar_rewind(const float* x, const float* x0, int64_t n, int level,
                                   float* acc, const uint32_t* sel_mask, dpz_stream_t stream) {
  if (!x0 || !acc || !sel_mask) return DPZ_ERR_ARG;
  return dwt_haar_run(x, x0, n, level, nullptr, acc, 1, sel_mask, stream);
}

extern "C" int dpz_idwt_haar(const float* coeffs, int64_t n, int level, float* out,
                             dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!coeffs || !out || n <= 0) return DPZ_ERR_ARG;
  if (level < 1 || level > HAAR_MAX_LEVEL) return DPZ_ERR_UNSUPPORTED;
  const HaarLevels LV = haar_levels(n, level);
  const int64_t nchunks = (n + HAAR_CHUNK - 1) / HAAR_CHUNK;
  const int vec = aligned16(out);
  const unsigned g = haar_grid(nchunks);
  switch (level) {
#define DPZ_HAAR_CASE(LEVN)                                                                   \
  case LEVN:                                                                                  \
    DPZ_TIMED(DPZ_KT_HAAR, st,                                                                \
              haar_idwt_kernel<LEVN><<<g, 256, 0, st>>>(coeffs, LV, out, nchunks, vec));      \
    break;
    DPZ_HAAR_CASE(1) DPZ_HAAR_CASE(2) DPZ_HAAR_CASE(3) DPZ_HAAR_CASE(4)
    DPZ_HAAR_CASE(5) DPZ_HAAR_CASE(6) DPZ_HAAR_CASE(7) DPZ_HAAR_CASE(8)
#undef DPZ_HAAR_CASE
    default:
      return DPZ_ERR_UNSUPPORTED;
  }
  return DPZ_OK;
}
