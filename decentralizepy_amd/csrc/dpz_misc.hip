// fp16 value packing and library-level entry points.
#include "dpz_common.h"

namespace dpz {

__device__ __forceinline__ uint32_t f2h(float v) {
  const _Float16 h = (_Float16)v;  // round-to-nearest-even
  return __builtin_bit_cast(uint16_t, h);
}
__device__ __forceinline__ float h2f(uint32_t b) {
  return (float)__builtin_bit_cast(_Float16, (uint16_t)b);
}

__global__ void __launch_bounds__(256) pack_fp16_kernel(const float* __restrict__ in, int64_t n,
                                                        uint16_t* __restrict__ out) {
  const int64_t n8 = n >> 3;
  for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < n8; g += (int64_t)gridDim.x * 256) {
    const float4 a = reinterpret_cast<const float4*>(in)[2 * g];
    const float4 b = reinterpret_cast<const float4*>(in)[2 * g + 1];
    const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    uint32_t w[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t lo = f2h(v[2 * e]);
      const uint32_t hi = f2h(v[2 * e + 1]);
      w[e] = lo | (hi << 16);
    }
    reinterpret_cast<uint4*>(out)[g] = make_uint4(w[0], w[1], w[2], w[3]);
  }
  const int64_t tail = n8 << 3;
  const int64_t i = tail + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (blockIdx.x == 0 && i < n) out[i] = (uint16_t)f2h(in[i]);
}

__global__ void __launch_bounds__(256) unpack_fp16_kernel(const uint16_t* __restrict__ in,
                                                          int64_t n, float* __restrict__ out) {
  const int64_t n8 = n >> 3;
  for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < n8; g += (int64_t)gridDim.x * 256) {
    const uint4 w = reinterpret_cast<const uint4*>(in)[g];
    const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
    float v[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[2 * e] = h2f(ww[e] & 0xFFFFu);
      v[2 * e + 1] = h2f(ww[e] >> 16);
    }
    reinterpret_cast<float4*>(out)[2 * g] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(out)[2 * g + 1] = make_float4(v[4], v[5], v[6], v[7]);
  }
  const int64_t tail = n8 << 3;
  const int64_t i = tail + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (blockIdx.x == 0 && i < n) out[i] = h2f(in[i]);
}

static unsigned grid_for(int64_t n8) {
  int64_t g = (n8 + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (unsigned)g;
}

}  // namespace dpz

using namespace dpz;

extern "C" int dpz_abi_version(void) { return 2; }

// Hash of the sources this library was built from (Makefile: sha256 of csrc/*.{cpp,h,hip}, the
// Makefile and include/dpz_codec.h, first 16 hex digits); decentralizepy_amd/_lib.py recomputes
// it from the checked-out tree so a stale binary fails loudly instead of being tested.
#ifndef DPZ_BUILD_ID
#define DPZ_BUILD_ID "unknown"
#endif
extern "C" const char* dpz_build_id(void) { return DPZ_BUILD_ID; }

extern "C" const char* dpz_error_string(int code) {
  switch (code) {
    case DPZ_OK: return "ok";
    case DPZ_ERR_ARG: return "invalid argument";
    case DPZ_ERR_WORKSPACE: return "workspace too small";
    case DPZ_ERR_UNSUPPORTED: return "unsupported size or configuration";
    case DPZ_ERR_INTERNAL: return "internal consistency check failed";
    default: return hipGetErrorString(static_cast<hipError_t>(code));
  }
}

extern "C" int dpz_pack_fp16(const float* in, int64_t n, uint16_t* out, dpz_stream_t stream) {
  if (n < 0 || (n > 0 && (!in || !out))) return DPZ_ERR_ARG;
  if (n == 0) return DPZ_OK;
  if ((reinterpret_cast<uintptr_t>(in) & 15u) || (reinterpret_cast<uintptr_t>(out) & 15u))
    return DPZ_ERR_ARG;
  hipStream_t st = static_cast<hipStream_t>(stream);
  DPZ_TIMED(DPZ_KT_FP16, st, pack_fp16_kernel<<<grid_for(n >> 3), 256, 0, st>>>(in, n, out));
  return DPZ_OK;
}

extern "C" int dpz_unpack_fp16(const uint16_t* in, int64_t n, float* out, dpz_stream_t stream) {
  if (n < 0 || (n > 0 && (!in || !out))) return DPZ_ERR_ARG;
  if (n == 0) return DPZ_OK;
  if ((reinterpret_cast<uintptr_t>(in) & 15u) || (reinterpret_cast<uintptr_t>(out) & 15u))
    return DPZ_ERR_ARG;
  hipStream_t st = static_cast<hipStream_t>(stream);
  DPZ_TIMED(DPZ_KT_FP16, st, unpack_fp16_kernel<<<grid_for(n >> 3), 256, 0, st>>>(in, n, out));
  return DPZ_OK;
}

namespace dpz {
__global__ void __launch_bounds__(256) scatter_fill_kernel(float* __restrict__ dst,
                                                           const int32_t* __restrict__ idx,
                                                           int64_t k, int64_t n, float v) {
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < k; j += (int64_t)gridDim.x * 256) {
    const int64_t i = idx[j];
    if (i >= 0 && i < n) dst[i] = v;
  }
}
}  // namespace dpz

extern "C" int dpz_scatter_fill(float* dst, int64_t n, const int32_t* idx, int64_t k, float value,
                                dpz_stream_t stream) {
  if (n < 0 || k < 0 || (k > 0 && (!dst || !idx))) return DPZ_ERR_ARG;
  if (k == 0) return DPZ_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  DPZ_TIMED(DPZ_KT_SCATTER, st,
            scatter_fill_kernel<<<grid_for((k + 255) / 256 * 32), 256, 0, st>>>(dst, idx, k, n, value));
  return DPZ_OK;
}
