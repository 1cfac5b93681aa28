// Elementwise fp32 helpers of the Choco sharing update and its threshold mask.
//
// Replaces (reference sacs-epfl/decentralizepy, src/decentralizepy/sharing/Choco.py):
//   :48-70    subtract_state_dicts            d = x - x_hat
//   :73-97    self_add_state_dict             x_hat += 1.0 * q
//   :117-140  topk_sparsification_tensor      q[|q| < T] = 0   (T from dpz_topk_threshold)
//   :441-447  x = x + step_size * (s - x_hat)
// and the owner-side combine of the over-HBM gossip round (decentralizepy_amd/gossip.py,
// reduce-scatter exchange): x_new = x * (c - B) + A.
// One fp32 rounding per operation (-ffp-contract=off), grid-stride, float4 where aligned.
#include "dpz_common.h"
#include "dpz_topk.h"

namespace dpz {

template <int OP>
__device__ __forceinline__ float ew(float a, float b, float d, float c) {
  if (OP == DPZ_EW_SUB) return a - b;
  if (OP == DPZ_EW_ADD) return a + b;
  if (OP == DPZ_EW_MHCOMBINE) {  // x * (c - hit weight) + weighted hit sum
    const float keep = c - b;
    const float base = a * keep;
    return base + d;
  }
  const float diff = b - d;  // s - x_hat
  const float step = c * diff;
  return a + step;
}

template <int OP>
__global__ void __launch_bounds__(256) ew_kernel(const float* a, const float* b, const float* d,
                                                 float c, int64_t n, float* out, int vec) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  if (vec) {
    const int64_t n4 = n >> 2;
    for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < n4; g += stride) {
      const float4 av = reinterpret_cast<const float4*>(a)[g];
      const float4 bv = reinterpret_cast<const float4*>(b)[g];
      float4 dv = make_float4(0.f, 0.f, 0.f, 0.f);
      if (OP == DPZ_EW_CHOCO || OP == DPZ_EW_MHCOMBINE) dv = reinterpret_cast<const float4*>(d)[g];
      reinterpret_cast<float4*>(out)[g] =
          make_float4(ew<OP>(av.x, bv.x, dv.x, c), ew<OP>(av.y, bv.y, dv.y, c),
                      ew<OP>(av.z, bv.z, dv.z, c), ew<OP>(av.w, bv.w, dv.w, c));
    }
    for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
      out[i] = ew<OP>(a[i], b[i], (OP == DPZ_EW_CHOCO || OP == DPZ_EW_MHCOMBINE) ? d[i] : 0.f, c);
  } else {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
      out[i] = ew<OP>(a[i], b[i], (OP == DPZ_EW_CHOCO || OP == DPZ_EW_MHCOMBINE) ? d[i] : 0.f, c);
  }
}

__global__ void __launch_bounds__(256) mask_kernel(const float* x, int64_t n,
                                                   const TopkCtrl* ctrl, float* out) {
  const uint32_t T = ctrl->prefix;  // threshold key of the last dpz_topk_threshold
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float v = x[i];
    out[i] = key_of(v) < T ? 0.0f : v;
  }
}

static unsigned ew_grid(int64_t n) {
  int64_t g = (n / 4 + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (unsigned)g;
}

}  // namespace dpz

using namespace dpz;

extern "C" int dpz_elementwise(int op, const float* a, const float* b, const float* d, float c,
                               int64_t n, float* out, dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (n < 0) return DPZ_ERR_ARG;
  if (n == 0) return DPZ_OK;
  const bool use_d = op == DPZ_EW_CHOCO || op == DPZ_EW_MHCOMBINE;
  if (!a || !b || !out || (use_d && !d)) return DPZ_ERR_ARG;
  const int vec = aligned16(a) && aligned16(b) && aligned16(out) && (!use_d || aligned16(d));
  const unsigned g = ew_grid(n);
  switch (op) {
    case DPZ_EW_SUB: ew_kernel<DPZ_EW_SUB><<<g, 256, 0, st>>>(a, b, d, c, n, out, vec); break;
    case DPZ_EW_ADD: ew_kernel<DPZ_EW_ADD><<<g, 256, 0, st>>>(a, b, d, c, n, out, vec); break;
    case DPZ_EW_CHOCO: ew_kernel<DPZ_EW_CHOCO><<<g, 256, 0, st>>>(a, b, d, c, n, out, vec); break;
    case DPZ_EW_MHCOMBINE: ew_kernel<DPZ_EW_MHCOMBINE><<<g, 256, 0, st>>>(a, b, d, c, n, out, vec); break;
    default: return DPZ_ERR_ARG;
  }
  DPZ_LAUNCH_CHECK();
  return DPZ_OK;
}

extern "C" int dpz_mask_below_threshold(const float* x, int64_t n, const void* ws, float* out,
                                        dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (n < 0 || (n > 0 && (!x || !ws || !out))) return DPZ_ERR_ARG;
  if (n == 0) return DPZ_OK;
  const WsLayout L = ws_layout(n);
  mask_kernel<<<ew_grid(n), 256, 0, st>>>(
      x, n, reinterpret_cast<const TopkCtrl*>(static_cast<const char*>(ws) + L.ctrl), out);
  DPZ_LAUNCH_CHECK();
  return DPZ_OK;
}

// ---- sharded top-k helpers (decentralizepy_amd/shard.py) --------------------------------------
namespace dpz {

// out[j] = x[idx[j]] - x0[idx[j]]  (the change at a candidate; x0 may be null: out = x[idx])
__global__ void __launch_bounds__(256) gather_change_kernel(const float* x, const float* x0,
                                                            const int32_t* idx, int64_t k,
                                                            int64_t n, float* out) {
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < k; j += (int64_t)gridDim.x * 256) {
    const int64_t i = idx[j];
    float v = 0.0f;
    if (i >= 0 && i < n) v = x0 ? x[i] - x0[i] : x[i];
    out[j] = v;
  }
}

// out[j] = src[pos[j]] for 32-bit words (bit copy)
__global__ void __launch_bounds__(256) gather_u32_kernel(const uint32_t* src, int64_t m,
                                                         const int32_t* pos, int64_t k,
                                                         uint32_t* out) {
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < k; j += (int64_t)gridDim.x * 256) {
    const int64_t p = pos[j];
    out[j] = (p >= 0 && p < m) ? src[p] : 0u;
  }
}

// out[j] = src[pos[j]] for 16-bit words (bit copy)
__global__ void __launch_bounds__(256) gather_u16_kernel(const uint16_t* src, int64_t m,
                                                         const int32_t* pos, int64_t k,
                                                         uint16_t* out) {
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < k; j += (int64_t)gridDim.x * 256) {
    const int64_t p = pos[j];
    out[j] = (p >= 0 && p < m) ? src[p] : (uint16_t)0;
  }
}

// dst[idx[j] - offset] += value for idx[j] in [offset, offset + n)
__global__ void __launch_bounds__(256) scatter_add_i32_kernel(int32_t* dst, int64_t n,
                                                              const int32_t* idx, int64_t k,
                                                              int64_t offset, int32_t value) {
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < k; j += (int64_t)gridDim.x * 256) {
    const int64_t i = (int64_t)idx[j] - offset;
    if (i >= 0 && i < n) atomicAdd(&dst[i], value);
  }
}

static unsigned small_grid(int64_t k) {
  int64_t g = (k + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (unsigned)g;
}

}  // namespace dpz

extern "C" int dpz_gather_change(const float* x, const float* x0, int64_t n, const int32_t* idx,
                                 int64_t k, float* out, dpz_stream_t stream) {
  if (n < 0 || k < 0 || (k > 0 && (!x || !idx || !out))) return DPZ_ERR_ARG;
  if (k == 0) return DPZ_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  gather_change_kernel<<<small_grid(k), 256, 0, st>>>(x, x0, idx, k, n, out);
  DPZ_LAUNCH_CHECK();
  return DPZ_OK;
}

extern "C" int dpz_gather_u32(const void* src, int64_t m, const int32_t* pos, int64_t k,
                              void* out, dpz_stream_t stream) {
  if (m < 0 || k < 0 || (k > 0 && (!src || !pos || !out))) return DPZ_ERR_ARG;
  if (k == 0) return DPZ_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  gather_u32_kernel<<<small_grid(k), 256, 0, st>>>(static_cast<const uint32_t*>(src), m, pos, k,
                                                   static_cast<uint32_t*>(out));
  DPZ_LAUNCH_CHECK();
  return DPZ_OK;
}

extern "C" int dpz_gather_u16(const void* src, int64_t m, const int32_t* pos, int64_t k,
                              void* out, dpz_stream_t stream) {
  if (m < 0 || k < 0 || (k > 0 && (!src || !pos || !out))) return DPZ_ERR_ARG;
  if (k == 0) return DPZ_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  gather_u16_kernel<<<small_grid(k), 256, 0, st>>>(static_cast<const uint16_t*>(src), m, pos, k,
                                                   static_cast<uint16_t*>(out));
  DPZ_LAUNCH_CHECK();
  return DPZ_OK;
}

extern "C" int dpz_scatter_add_i32(int32_t* dst, int64_t n, const int32_t* idx, int64_t k,
                                   int64_t offset, int32_t value, dpz_stream_t stream) {
  if (n < 0 || k < 0 || (k > 0 && (!dst || !idx))) return DPZ_ERR_ARG;
  if (k == 0 || n == 0) return DPZ_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  scatter_add_i32_kernel<<<small_grid(k), 256, 0, st>>>(dst, n, idx, k, offset, value);
  DPZ_LAUNCH_CHECK();
  return DPZ_OK;
}
