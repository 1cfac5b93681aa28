// Micro-benchmark: what a plain fp32 copy (the replace decode's 4N read + 4N write) and a
// two-stream read (the filter's x, x0) reach on MI355X, by launch geometry and cache policy.
// Buffers rotate over NSET independent sets so the working set is > 2x the 256 MiB L3.
// Build: hipcc --offload-arch=gfx950 -O3 -o copy_bw copy_bw.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef float v4f __attribute__((ext_vector_type(4)));

template <int U, int NT>
__global__ void __launch_bounds__(256) copy_gs(const v4f* __restrict__ a, v4f* __restrict__ b,
                                               int64_t n4) {
  const int64_t stride = (int64_t)gridDim.x * 256 * U;
  for (int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x; base < n4; base += stride) {
    v4f v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t q = base + u * 256;
      if (q < n4) v[u] = (NT & 1) ? __builtin_nontemporal_load(&a[q]) : a[q];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t q = base + u * 256;
      if (q < n4) {
        if (NT & 2) __builtin_nontemporal_store(v[u], &b[q]);
        else b[q] = v[u];
      }
    }
  }
}

template <int U, int NT>
__global__ void __launch_bounds__(256) read2_gs(const v4f* __restrict__ a,
                                                const v4f* __restrict__ c, int64_t n4,
                                                uint32_t* out) {
  const int64_t stride = (int64_t)gridDim.x * 256 * U;
  uint32_t cnt = 0;
  for (int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x; base < n4; base += stride) {
    v4f v[U], w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t q = base + u * 256;
      if (q < n4) {
        v[u] = (NT & 1) ? __builtin_nontemporal_load(&a[q]) : a[q];
        w[u] = (NT & 1) ? __builtin_nontemporal_load(&c[q]) : c[q];
      } else {
        v[u] = w[u] = (v4f){0, 0, 0, 0};
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      v4f d = v[u] - w[u];
      cnt += (__float_as_uint(d.x) & 0x7FFFFFFFu) > 0x3F800000u;
      cnt += (__float_as_uint(d.y) & 0x7FFFFFFFu) > 0x3F800000u;
      cnt += (__float_as_uint(d.z) & 0x7FFFFFFFu) > 0x3F800000u;
      cnt += (__float_as_uint(d.w) & 0x7FFFFFFFu) > 0x3F800000u;
    }
  }
  if (cnt == 0xFFFFFFFFu) out[0] = cnt;
}

// each WAVE copies its own contiguous segment of R elements (the replace / filter geometry)
template <int U, int NT>
__global__ void __launch_bounds__(256) copy_waveseg(const v4f* __restrict__ a, v4f* __restrict__ b,
                                                    int64_t n4, int64_t R4) {
  const int lane = threadIdx.x & 63;
  const int64_t seg = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t beg = seg * R4, end = beg + R4 < n4 ? beg + R4 : n4;
  for (int64_t base = beg; base < end; base += 64 * U) {
    v4f v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t q = base + u * 64 + lane;
      if (q < end) v[u] = (NT & 1) ? __builtin_nontemporal_load(&a[q]) : a[q];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t q = base + u * 64 + lane;
      if (q < end) {
        if (NT & 2) __builtin_nontemporal_store(v[u], &b[q]);
        else b[q] = v[u];
      }
    }
  }
}

// each BLOCK copies its own contiguous segment of R elements, its 4 waves side by side
template <int U, int NT>
__global__ void __launch_bounds__(256) copy_blockseg(const v4f* __restrict__ a, v4f* __restrict__ b,
                                                     int64_t n4, int64_t R4) {
  const int64_t beg = (int64_t)blockIdx.x * R4, end = beg + R4 < n4 ? beg + R4 : n4;
  for (int64_t base = beg; base < end; base += 256 * U) {
    v4f v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t q = base + u * 256 + threadIdx.x;
      if (q < end) v[u] = (NT & 1) ? __builtin_nontemporal_load(&a[q]) : a[q];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t q = base + u * 256 + threadIdx.x;
      if (q < end) {
        if (NT & 2) __builtin_nontemporal_store(v[u], &b[q]);
        else b[q] = v[u];
      }
    }
  }
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 11000000;
  const int NSET = 8;
  const int64_t n4 = n / 4;
  float *A[NSET], *B[NSET];
  for (int s = 0; s < NSET; ++s) {
    CK(hipMalloc(&A[s], n * 4));
    CK(hipMalloc(&B[s], n * 4));
    CK(hipMemset(A[s], 0x3c, n * 4));
    CK(hipMemset(B[s], 0x3d, n * 4));
  }
  uint32_t* out;
  CK(hipMalloc(&out, 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int REPS = 64;
  auto bench = [&](const char* name, int grid, auto fn, double bytes) {
    for (int r = 0; r < 2 * NSET; ++r) fn(r % NSET, grid);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < REPS; ++r) fn(r % NSET, grid);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / REPS;
    printf("%-34s grid %6d  %8.2f us  %7.1f GB/s\n", name, grid, us, bytes / us / 1e3);
  };
#define COPY(U, NT)                                                                            \
  for (int grid : {1024, 2048, 4096, 8192, (int)((n4 + 256 * U - 1) / (256 * U))}) {          \
    char nm[64];                                                                               \
    snprintf(nm, sizeof nm, "copy U=%d nt=%d", U, NT);                                         \
    bench(nm, grid, [&](int s, int g) {                                                        \
      copy_gs<U, NT><<<g, 256>>>((const v4f*)A[s], (v4f*)B[s], n4); }, 8.0 * n);              \
  }
#define READ2(U, NT)                                                                           \
  for (int grid : {1024, 2048, 4096, (int)((n4 + 256 * U - 1) / (256 * U))}) {                \
    char nm[64];                                                                               \
    snprintf(nm, sizeof nm, "read2 U=%d nt=%d", U, NT);                                        \
    bench(nm, grid, [&](int s, int g) {                                                        \
      read2_gs<U, NT><<<g, 256>>>((const v4f*)A[s], (const v4f*)B[s], n4, out); }, 8.0 * n);  \
  }
  if (argc > 2) {
    COPY(4, 3) COPY(8, 3)
    for (int64_t R : {1600LL, 6400LL, 25600LL}) {
      const int64_t R4 = R / 4;
      const int64_t W = (n4 + R4 - 1) / R4;
      char nm[64];
      snprintf(nm, sizeof nm, "waveseg U=4 nt=3 R=%lld", (long long)R);
      bench(nm, (int)((W + 3) / 4), [&](int s, int g) {
        copy_waveseg<4, 3><<<g, 256>>>((const v4f*)A[s], (v4f*)B[s], n4, R4); }, 8.0 * n);
      snprintf(nm, sizeof nm, "waveseg U=8 nt=3 R=%lld", (long long)R);
      bench(nm, (int)((W + 3) / 4), [&](int s, int g) {
        copy_waveseg<8, 3><<<g, 256>>>((const v4f*)A[s], (v4f*)B[s], n4, R4); }, 8.0 * n);
      snprintf(nm, sizeof nm, "blockseg U=4 nt=3 R=%lld", (long long)R);
      bench(nm, (int)W, [&](int s, int g) {
        copy_blockseg<4, 3><<<g, 256>>>((const v4f*)A[s], (v4f*)B[s], n4, R4); }, 8.0 * n);
    }
    return 0;
  }
  COPY(2, 0) COPY(4, 0) COPY(8, 0) COPY(4, 3) COPY(8, 3) COPY(8, 1) COPY(8, 2) COPY(16, 3)
  READ2(2, 0) READ2(4, 0) READ2(4, 1) READ2(8, 1) READ2(2, 1)
  return 0;
}
