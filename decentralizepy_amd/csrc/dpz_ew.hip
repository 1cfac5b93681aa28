// Elementwise fp32 helpers of the Choco sharing update and its threshold mask.
//
// Replaces (reference sacs-epfl/decentralizepy, src/decentralizepy/sharing/Choco.py):
//   :48-70    subtract_state_dicts            d = x - x_hat
//   :73-97    self_add_state_dict             x_hat += 1.0 * q
//   :117-140  topk_sparsification_tensor      q[|q| < T] = 0   (T from dpz_topk_threshold)
//   :441-447  x = x + step_size * (s - x_hat)
// One fp32 rounding per operation (-ffp-contract=off), grid-stride, float4 where aligned.
#include "dpz_common.h"
#include "dpz_topk.h"

namespace dpz {

template <int OP>
__device__ __forceinline__ float ew(float a, float b, float d, float c) {
  if (OP == DPZ_EW_SUB) return a - b;
  if (OP == DPZ_EW_ADD) return a + b;
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
      if (OP == DPZ_EW_CHOCO) dv = reinterpret_cast<const float4*>(d)[g];
      reinterpret_cast<float4*>(out)[g] =
          make_float4(ew<OP>(av.x, bv.x, dv.x, c), ew<OP>(av.y, bv.y, dv.y, c),
                      ew<OP>(av.z, bv.z, dv.z, c), ew<OP>(av.w, bv.w, dv.w, c));
    }
    for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
      out[i] = ew<OP>(a[i], b[i], OP == DPZ_EW_CHOCO ? d[i] : 0.f, c);
  } else {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
      out[i] = ew<OP>(a[i], b[i], OP == DPZ_EW_CHOCO ? d[i] : 0.f, c);
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
  if (!a || !b || !out || (op == DPZ_EW_CHOCO && !d)) return DPZ_ERR_ARG;
  const int vec = aligned16(a) && aligned16(b) && aligned16(out) && (op != DPZ_EW_CHOCO || aligned16(d));
  const unsigned g = ew_grid(n);
  switch (op) {
    case DPZ_EW_SUB: ew_kernel<DPZ_EW_SUB><<<g, 256, 0, st>>>(a, b, d, c, n, out, vec); break;
    case DPZ_EW_ADD: ew_kernel<DPZ_EW_ADD><<<g, 256, 0, st>>>(a, b, d, c, n, out, vec); break;
    case DPZ_EW_CHOCO: ew_kernel<DPZ_EW_CHOCO><<<g, 256, 0, st>>>(a, b, d, c, n, out, vec); break;
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
