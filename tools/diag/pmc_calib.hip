// Calibration of rocprofv3's FETCH_SIZE for the load widths the top-k compact uses
// (MI355X_MICROARCH.md § HBM: FETCH_SIZE reports 1/2 of a 16-byte-per-lane streaming read; other
// widths are uncalibrated).  Each kernel streams the same 512 MiB (twice the Infinity Cache) with
// a different per-lane width and writes one word per block; run under
//   rocprofv3 --pmc FETCH_SIZE -- ./pmc_calib
// and compare each kernel's FETCH_SIZE with the 536,870,912 bytes it reads.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr size_t BYTES = size_t(512) << 20;

__global__ void __launch_bounds__(256) read_b4(const uint32_t* __restrict__ p, size_t n,
                                                uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    acc ^= p[i];
  if (acc == 0x9E3779B9u) out[blockIdx.x] = acc;  // never true for the zero-filled input
}

__global__ void __launch_bounds__(256) read_b8(const uint2* __restrict__ p, size_t n,
                                                uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const uint2 v = p[i];
    acc ^= v.x ^ v.y;
  }
  if (acc == 0x9E3779B9u) out[blockIdx.x] = acc;
}

__global__ void __launch_bounds__(256) read_b16(const uint4* __restrict__ p, size_t n,
                                                 uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9E3779B9u) out[blockIdx.x] = acc;
}

// short contiguous runs (64 words) at scattered run starts: a compact-like list read
__global__ void __launch_bounds__(256) read_runs(const uint32_t* __restrict__ p, size_t n,
                                                  uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  const size_t runs = n / 64;
  for (size_t r = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < runs;
       r += (size_t)gridDim.x * 4) {
    const size_t q = (r * 2654435761ull) % runs;  // a permutation of the runs (runs odd-coprime)
    acc ^= p[q * 64 + (threadIdx.x & 63)];
  }
  if (acc == 0x9E3779B9u) out[blockIdx.x] = acc;
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main() {
  void* buf = nullptr;
  uint32_t* out = nullptr;
  CK(hipMalloc(&buf, BYTES));
  CK(hipMalloc(&out, 4096 * sizeof(uint32_t)));
  CK(hipMemset(buf, 0, BYTES));
  const unsigned grid = 2048;
  for (int rep = 0; rep < 3; ++rep) {
    read_b4<<<grid, 256>>>(static_cast<const uint32_t*>(buf), BYTES / 4, out);
    read_b8<<<grid, 256>>>(static_cast<const uint2*>(buf), BYTES / 8, out);
    read_b16<<<grid, 256>>>(static_cast<const uint4*>(buf), BYTES / 16, out);
    read_runs<<<grid, 256>>>(static_cast<const uint32_t*>(buf), BYTES / 4, out);
  }
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  std::printf("read %zu bytes per kernel\n", BYTES);
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
