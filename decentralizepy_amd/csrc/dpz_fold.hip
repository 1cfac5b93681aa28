// Batched decode (replace) + Metro-Hastings weighted fold over a gossip round's payloads.
//
// Replaces (reference sacs-epfl/decentralizepy, src/decentralizepy/):
//   sharing/PartialModel.py:257-303  deserialized_model: T = cat(local); T[idx] = params
//   sharing/Sharing.py:156-190       _averaging: total = T_0*w_0; total += T_i*w_i; += (1-sum)*local
//   sharing/Sharing.py:200-229       _averaging_server: w = 1/n, no self term
//   sharing/JWINS/Wavelet.py:269-309 the same fold on wavelet coefficients
//
// One block owns a 4096-element tile of the output.  For each payload (in payload order) the
// block locates its index range by binary search (idx is strictly ascending), scatters the hits
// into an LDS value tile tagged with the payload number, and every thread folds its 16 elements:
//   t = (tag == p) ? hit : local;  total = (p == 0) ? t*w : total + t*w
// in exactly the reference's fp32 order (compiled with -ffp-contract=off: no FMA contraction).
// Bytes per element: read local (4) + write out (4) + 8 per payload hit -> HBM-bound.
#include "dpz_common.h"

namespace dpz {

constexpr int FOLD_TILE = 4096;
constexpr int FOLD_MAXP = 16;  // payloads per launch (longer lists are chained)

struct FoldPayload {
  const int32_t* idx;  // nullptr: dense payload (vals has n entries)
  const float* val;
  int64_t k;
  float w;
};

struct FoldArgs {
  const float* local;
  float* out;
  int64_t n;
  int np;
  int first;        // total starts from payload 0 (else continue from out)
  int add_self;     // add local * w_self at the end
  int replace_only; // out = t_0
  float w_self;
  FoldPayload p[FOLD_MAXP];
};

__device__ __forceinline__ int64_t lower_bound_i32(const int32_t* a, int64_t len, int64_t v) {
  int64_t lo = 0, hi = len;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((int64_t)a[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

template <bool VEC>
__global__ void __launch_bounds__(256) fold_kernel(FoldArgs a) {
  __shared__ __attribute__((aligned(16))) float hv[FOLD_TILE];
  __shared__ __attribute__((aligned(16))) uint8_t htag[FOLD_TILE];
  __shared__ int64_t rng[FOLD_MAXP][2];
  const int64_t tlo = (int64_t)blockIdx.x * FOLD_TILE;
  const int64_t thi = (tlo + FOLD_TILE < a.n) ? tlo + FOLD_TILE : a.n;
  const int t = threadIdx.x;
  if (t < a.np) {
    const FoldPayload& P = a.p[t];
    if (P.idx) {
      rng[t][0] = lower_bound_i32(P.idx, P.k, tlo);
      rng[t][1] = lower_bound_i32(P.idx, P.k, thi);
    } else {
      rng[t][0] = rng[t][1] = 0;
    }
  }
  for (int j = t * 4; j < FOLD_TILE; j += 1024) *reinterpret_cast<uint32_t*>(&htag[j]) = 0xFFFFFFFFu;

  // this thread's elements: q-th group = tlo + q*1024 + 4t .. +3
  float L[16], acc[16];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t i0 = tlo + q * 1024 + t * 4;
    if (VEC && i0 + 3 < thi) {
      float4 v = *reinterpret_cast<const float4*>(a.local + i0);
      L[q * 4 + 0] = v.x; L[q * 4 + 1] = v.y; L[q * 4 + 2] = v.z; L[q * 4 + 3] = v.w;
      if (!a.first) {
        float4 o = *reinterpret_cast<const float4*>(a.out + i0);
        acc[q * 4 + 0] = o.x; acc[q * 4 + 1] = o.y; acc[q * 4 + 2] = o.z; acc[q * 4 + 3] = o.w;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t i = i0 + e;
        L[q * 4 + e] = i < thi ? a.local[i] : 0.0f;
        if (!a.first) acc[q * 4 + e] = i < thi ? a.out[i] : 0.0f;
      }
    }
  }

  for (int p = 0; p < a.np; ++p) {
    const FoldPayload& P = a.p[p];
    __syncthreads();  // previous payload's reads of hv/htag done; rng visible
    if (P.idx) {
      const int64_t b = rng[p][0], e = rng[p][1];
      for (int64_t j = b + t; j < e; j += 256) {
        const int64_t pos = (int64_t)P.idx[j] - tlo;
        if (pos >= 0 && pos < FOLD_TILE) {  // guards against an unsorted caller array
          hv[pos] = P.val[j];
          htag[pos] = (uint8_t)p;
        }
      }
    }
    __syncthreads();
    const float w = P.w;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j0 = q * 1024 + t * 4;
      const int64_t i0 = tlo + j0;
      float tv[4];
      if (P.idx) {
        const float4 h4 = *reinterpret_cast<const float4*>(&hv[j0]);
        const uint32_t g4 = *reinterpret_cast<const uint32_t*>(&htag[j0]);
        const float hh[4] = {h4.x, h4.y, h4.z, h4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e)
          tv[e] = (((g4 >> (8 * e)) & 0xFFu) == (uint32_t)p) ? hh[e] : L[q * 4 + e];
      } else {
        if (VEC && i0 + 3 < thi) {
          float4 v = *reinterpret_cast<const float4*>(P.val + i0);
          tv[0] = v.x; tv[1] = v.y; tv[2] = v.z; tv[3] = v.w;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) tv[e] = (i0 + e < thi) ? P.val[i0 + e] : 0.0f;
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (a.replace_only) {
          acc[q * 4 + e] = tv[e];
        } else {
          const float term = tv[e] * w;
          acc[q * 4 + e] = (a.first && p == 0) ? term : acc[q * 4 + e] + term;
        }
      }
    }
  }
  if (a.add_self) {
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = acc[e] + L[e] * a.w_self;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t i0 = tlo + q * 1024 + t * 4;
    if (VEC && i0 + 3 < thi) {
      *reinterpret_cast<float4*>(a.out + i0) =
          make_float4(acc[q * 4 + 0], acc[q * 4 + 1], acc[q * 4 + 2], acc[q * 4 + 3]);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (i0 + e < thi) a.out[i0 + e] = acc[q * 4 + e];
    }
  }
}

}  // namespace dpz

using namespace dpz;

extern "C" int dpz_decode_average(const float* local, int64_t n, int n_payloads,
                                  const int32_t* const* idx, const float* const* vals,
                                  const int64_t* k, const float* w, float w_self, int flags,
                                  float* out, dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (n < 0 || n_payloads < 0) return DPZ_ERR_ARG;
  if (n == 0) return DPZ_OK;
  if (!local || !out || local == out) return DPZ_ERR_ARG;
  const bool replace_only = (flags & DPZ_FOLD_REPLACE_ONLY) != 0;
  if (replace_only && n_payloads != 1) return DPZ_ERR_ARG;
  if (n_payloads > 0 && (!vals || !k || (!replace_only && !w))) return DPZ_ERR_ARG;
  for (int i = 0; i < n_payloads; ++i) {
    if (!vals[i]) return DPZ_ERR_ARG;
    const bool dense = !idx || !idx[i];
    if (dense && k[i] != n) return DPZ_ERR_ARG;
    if (!dense && (k[i] < 0 || k[i] > n)) return DPZ_ERR_ARG;
  }
  bool vec = ((reinterpret_cast<uintptr_t>(local) | reinterpret_cast<uintptr_t>(out)) & 15u) == 0;
  for (int i = 0; i < n_payloads; ++i)
    if ((!idx || !idx[i]) && (reinterpret_cast<uintptr_t>(vals[i]) & 15u)) vec = false;
  const unsigned grid = (unsigned)((n + FOLD_TILE - 1) / FOLD_TILE);
  if (n_payloads == 0) {
    // no payloads: out = w_self * local (self term only) or zeros
    FoldArgs fa{};
    fa.local = local; fa.out = out; fa.n = n; fa.np = 0; fa.first = 0;
    fa.add_self = (flags & DPZ_FOLD_SELF) ? 1 : 0; fa.w_self = w_self;
    DPZ_HIP_TRY(hipMemsetAsync(out, 0, n * sizeof(float), st));
    if (vec) fold_kernel<true><<<grid, 256, 0, st>>>(fa); else fold_kernel<false><<<grid, 256, 0, st>>>(fa);
    DPZ_LAUNCH_CHECK();
    return DPZ_OK;
  }
  for (int base = 0; base < n_payloads; base += FOLD_MAXP) {
    FoldArgs fa{};
    fa.local = local; fa.out = out; fa.n = n;
    fa.np = (n_payloads - base) < FOLD_MAXP ? (n_payloads - base) : FOLD_MAXP;
    fa.first = base == 0 ? 1 : 0;
    fa.add_self = (base + fa.np == n_payloads && (flags & DPZ_FOLD_SELF)) ? 1 : 0;
    fa.replace_only = replace_only ? 1 : 0;
    fa.w_self = w_self;
    for (int i = 0; i < fa.np; ++i) {
      fa.p[i].idx = idx ? idx[base + i] : nullptr;
      fa.p[i].val = vals[base + i];
      fa.p[i].k = k[base + i];
      fa.p[i].w = replace_only ? 1.0f : w[base + i];
    }
    if (vec) fold_kernel<true><<<grid, 256, 0, st>>>(fa); else fold_kernel<false><<<grid, 256, 0, st>>>(fa);
    DPZ_LAUNCH_CHECK();
  }
  return DPZ_OK;
}
