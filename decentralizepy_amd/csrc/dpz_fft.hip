// Frequency-domain codec of the FFT sharing plugin: real FFTs through hipFFT (rocFFT), and the
// complex-coefficient kernels around the shared top-k / fold kernels.
//
// Replaces (reference sacs-epfl/decentralizepy, src/decentralizepy/):
//   sharing/JWINS/FFT.py:12-25     change_transformer_fft: torch.fft.rfft(x)
//   sharing/JWINS/FFT.py:301       fft.irfft(total)  (normalisation "backward": 1/n on the inverse)
//   sharing/JWINS/FFT.py:143-156   topk(|change|) over complex64 coefficients, flat_fft[index]
//   sharing/PartialModel.py:315-329  acc += change / change += acc on the complex change
//   models/Model.py:53-64          accumulated_changes[indices] = 0 (complex)
//   sharing/JWINS/FFT.py:282-299   topkf = flat_fft.clone(); topkf[indices] = params  (fold input:
//                                  complex entries become float pairs for dpz_decode_average)
//
// The transforms are library calls (like hipBLASLt for a plain GEMM): a mixed-radix FFT for an
// arbitrary model size is rocFFT's job.  Plans are cached per (device, n, direction) with
// auto-allocation off; the caller passes the work area (dpz_fft_workspace_bytes), so the only
// device memory the library owns is rocFFT's per-plan twiddle tables.  Complex data is
// interleaved fp32 (re, im) = torch.complex64's layout.
#include <hipfft/hipfft.h>

#include <mutex>
#include <map>
#include <tuple>

#include "dpz_common.h"
#include "dpz_topk.h"

namespace dpz {

// key[i] = |c[i]| after the accumulation step of DPZ_ACC_* (fp32, sqrt(re*re + im*im): the
// vectorised ATen-CPU complex abs; the FFT itself differs from pocketfft by rounding, so parity
// of this path is a tolerance parity).
template <int MODE>
__global__ void __launch_bounds__(256) cplx_key_kernel(const float2* __restrict__ change,
                                                       float2* acc, int64_t m,
                                                       float* __restrict__ key) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (int64_t)gridDim.x * 256) {
    float2 c = change[i];
    if (MODE == DPZ_ACC_ACCUMULATE) {
      float2 a = acc[i];
      a.x = a.x + c.x;
      a.y = a.y + c.y;
      acc[i] = a;
      c = a;
    } else if (MODE == DPZ_ACC_ADD) {
      const float2 a = acc[i];
      c.x = c.x + a.x;
      c.y = c.y + a.y;
    }
    const float re2 = c.x * c.x;
    const float im2 = c.y * c.y;
    key[i] = sqrtf(re2 + im2);  // correctly rounded (llvm.sqrt without afn)
  }
}

// out[j] = src[idx[j]]; acc[idx[j]] = 0 when acc is given (Model.rewind_accumulation)
__global__ void __launch_bounds__(256) cplx_gather_kernel(const float2* __restrict__ src, int64_t m,
                                                          const int32_t* __restrict__ idx,
                                                          int64_t k, float2* __restrict__ out,
                                                          float2* acc) {
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < k; j += (int64_t)gridDim.x * 256) {
    const int64_t i = idx[j];
    float2 v = make_float2(0.f, 0.f);
    if (i >= 0 && i < m) {
      v = src[i];
      if (acc) acc[i] = make_float2(0.f, 0.f);
    }
    out[j] = v;
  }
}

// pair[2j] = 2 idx[j], pair[2j + 1] = 2 idx[j] + 1: complex entries as float-pair entries
__global__ void __launch_bounds__(256) cplx_pair_idx_kernel(const int32_t* __restrict__ idx,
                                                            int64_t k, int32_t* __restrict__ pair) {
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < k; j += (int64_t)gridDim.x * 256) {
    const int32_t i = idx[j];
    reinterpret_cast<int2*>(pair)[j] = make_int2(2 * i, 2 * i + 1);
  }
}

__global__ void __launch_bounds__(256) scale_kernel(float* x, int64_t n, float s) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    x[i] = x[i] * s;
}

static unsigned grid_for(int64_t n) {
  int64_t g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (unsigned)g;
}

// ---- plan cache -------------------------------------------------------------------------------
struct FftPlan {
  hipfftHandle h;
  size_t work;
};

static std::mutex g_fft_mu;
static std::map<std::tuple<int, int64_t, int>, FftPlan> g_fft_plans;

// direction 0 = R2C (n reals -> n/2 + 1 complex), 1 = C2R (n/2 + 1 complex -> n reals)
static int fft_plan(int64_t n, int dir, FftPlan* out) {
  int dev = 0;
  DPZ_HIP_TRY(hipGetDevice(&dev));
  const auto key = std::make_tuple(dev, n, dir);
  auto it = g_fft_plans.find(key);
  if (it != g_fft_plans.end()) {
    *out = it->second;
    return DPZ_OK;
  }
  FftPlan p{};
  if (hipfftCreate(&p.h) != HIPFFT_SUCCESS) return DPZ_ERR_INTERNAL;
  if (hipfftSetAutoAllocation(p.h, 0) != HIPFFT_SUCCESS ||
      hipfftMakePlan1d(p.h, (int)n, dir == 0 ? HIPFFT_R2C : HIPFFT_C2R, 1, &p.work) !=
          HIPFFT_SUCCESS) {
    hipfftDestroy(p.h);
    return DPZ_ERR_INTERNAL;
  }
  g_fft_plans.emplace(key, p);
  *out = p;
  return DPZ_OK;
}

static int fft_exec(int64_t n, int dir, void* in, void* out, void* ws, size_t ws_bytes,
                    hipStream_t st) {
  if (n < 2 || n > INT32_MAX) return DPZ_ERR_UNSUPPORTED;
  std::lock_guard<std::mutex> lock(g_fft_mu);
  FftPlan p;
  const int rc = fft_plan(n, dir, &p);
  if (rc != DPZ_OK) return rc;
  if (p.work > 0 && (!ws || ws_bytes < p.work)) return DPZ_ERR_WORKSPACE;
  if (hipfftSetWorkArea(p.h, p.work > 0 ? ws : nullptr) != HIPFFT_SUCCESS ||
      hipfftSetStream(p.h, st) != HIPFFT_SUCCESS)
    return DPZ_ERR_INTERNAL;
  const hipfftResult r =
      dir == 0 ? hipfftExecR2C(p.h, static_cast<hipfftReal*>(in), static_cast<hipfftComplex*>(out))
               : hipfftExecC2R(p.h, static_cast<hipfftComplex*>(in), static_cast<hipfftReal*>(out));
  return r == HIPFFT_SUCCESS ? DPZ_OK : DPZ_ERR_INTERNAL;
}

}  // namespace dpz

using namespace dpz;

extern "C" int64_t dpz_fft_workspace_bytes(int64_t n) {
  if (n < 2 || n > INT32_MAX) return -1;
  std::lock_guard<std::mutex> lock(g_fft_mu);
  FftPlan a, b;
  if (fft_plan(n, 0, &a) != DPZ_OK || fft_plan(n, 1, &b) != DPZ_OK) return -1;
  const size_t w = a.work > b.work ? a.work : b.work;
  return (int64_t)(w > 0 ? w : 0);
}

extern "C" int dpz_rfft(const float* x, int64_t n, float* out, void* ws, size_t ws_bytes,
                        dpz_stream_t stream) {
  if (!x || !out || n < 2) return DPZ_ERR_ARG;
  // out-of-place R2C leaves its input untouched
  return fft_exec(n, 0, const_cast<float*>(x), out, ws, ws_bytes, static_cast<hipStream_t>(stream));
}

extern "C" int dpz_irfft(float* coeffs, int64_t n, float* out, void* ws, size_t ws_bytes,
                         dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!coeffs || !out || n < 2) return DPZ_ERR_ARG;
  const int rc = fft_exec(n, 1, coeffs, out, ws, ws_bytes, st);
  if (rc != DPZ_OK) return rc;
  DPZ_TIMED(DPZ_KT_FFT_SCALE, st, scale_kernel<<<grid_for(n), 256, 0, st>>>(out, n, 1.0f / (float)n));
  return DPZ_OK;
}

extern "C" int dpz_cplx_key(const float* change, float* acc, int acc_mode, int64_t m, float* key,
                            dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (m < 0 || (m > 0 && (!change || !key))) return DPZ_ERR_ARG;
  if (acc_mode != DPZ_ACC_NONE && !acc) return DPZ_ERR_ARG;
  if (m == 0) return DPZ_OK;
  const float2* c = reinterpret_cast<const float2*>(change);
  float2* a = reinterpret_cast<float2*>(acc);
  switch (acc_mode) {
    case DPZ_ACC_NONE:
      DPZ_TIMED(DPZ_KT_CPLX, st, cplx_key_kernel<DPZ_ACC_NONE><<<grid_for(m), 256, 0, st>>>(c, a, m, key));
      break;
    case DPZ_ACC_ACCUMULATE:
      DPZ_TIMED(DPZ_KT_CPLX, st, cplx_key_kernel<DPZ_ACC_ACCUMULATE><<<grid_for(m), 256, 0, st>>>(c, a, m, key));
      break;
    case DPZ_ACC_ADD:
      DPZ_TIMED(DPZ_KT_CPLX, st, cplx_key_kernel<DPZ_ACC_ADD><<<grid_for(m), 256, 0, st>>>(c, a, m, key));
      break;
    default:
      return DPZ_ERR_ARG;
  }
  return DPZ_OK;
}

extern "C" int dpz_cplx_gather(const float* src, int64_t m, const int32_t* idx, int64_t k,
                               float* out, float* acc, dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (m < 0 || k < 0 || (k > 0 && (!src || !idx || !out))) return DPZ_ERR_ARG;
  if (k == 0) return DPZ_OK;
  DPZ_TIMED(DPZ_KT_CPLX, st,
            cplx_gather_kernel<<<grid_for(k), 256, 0, st>>>(
                reinterpret_cast<const float2*>(src), m, idx, k, reinterpret_cast<float2*>(out),
                reinterpret_cast<float2*>(acc)));
  return DPZ_OK;
}

extern "C" int dpz_cplx_pair_indices(const int32_t* idx, int64_t k, int32_t* pair,
                                     dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (k < 0 || (k > 0 && (!idx || !pair))) return DPZ_ERR_ARG;
  if (k == 0) return DPZ_OK;
  if (!aligned16(pair) && (reinterpret_cast<uintptr_t>(pair) & 7u)) return DPZ_ERR_ARG;
  DPZ_TIMED(DPZ_KT_CPLX, st, cplx_pair_idx_kernel<<<grid_for(k), 256, 0, st>>>(idx, k, pair));
  return DPZ_OK;
}
