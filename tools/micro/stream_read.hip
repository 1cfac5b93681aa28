// Micro-benchmark: HBM read geometry for the top-k filter (two fp32 streams x, x0 -> key).
// Variants (all read 8N bytes, count keys >= a threshold so the loads stay live):
//   seg<G>   : one wave per contiguous segment of R elements, G float4 groups per lane per
//              iteration (the filter's geometry is G = 4, R = 1344 at N = 11M)
//   grid<U>  : grid-stride over the whole array, U float4 per lane per iteration
// Buffers rotate over NSET independent (x, x0) pairs so the working set is > 2x the 256 MiB L3.
// Build: hipcc --offload-arch=gfx950 -O3 -o stream_read stream_read.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ uint32_t keyof(float a, float b) {
  return __float_as_uint(a - b) & 0x7FFFFFFFu;
}

template <int G>
__global__ void __launch_bounds__(256) seg_kernel(const float* __restrict__ x,
                                                  const float* __restrict__ x0, int64_t n,
                                                  int64_t R, uint32_t thr, uint32_t* out) {
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t seg = (int64_t)blockIdx.x * 4 + wid;
  const int64_t beg = seg * R;
  const int64_t end = beg + R < n ? beg + R : n;
  uint32_t c = 0;
  for (int64_t base = beg; base < end; base += G * 256) {
    float4 a[G], b[G];
#pragma unroll
    for (int q = 0; q < G; ++q) {
      const int64_t i0 = base + q * 256 + lane * 4;
      if (i0 + 3 < end) {
        a[q] = *reinterpret_cast<const float4*>(x + i0);
        b[q] = *reinterpret_cast<const float4*>(x0 + i0);
      } else {
        a[q] = make_float4(0, 0, 0, 0);
        b[q] = a[q];
      }
    }
#pragma unroll
    for (int q = 0; q < G; ++q) {
      c += keyof(a[q].x, b[q].x) >= thr;
      c += keyof(a[q].y, b[q].y) >= thr;
      c += keyof(a[q].z, b[q].z) >= thr;
      c += keyof(a[q].w, b[q].w) >= thr;
    }
  }
  if (lane == 0) out[seg] = c;
}

// the filter's end-of-block histogram flush, three ways: FLUSH 0 none, 1 atomics into 16 copies
// of 257 bins (the current filter), 2 plain row stores (257 per block)
template <int FLUSH>
__global__ void __launch_bounds__(256) segflush_kernel(const float* __restrict__ x,
                                                       const float* __restrict__ x0, int64_t n,
                                                       int64_t R, uint32_t thr, uint32_t* out,
                                                       uint32_t* hist) {
  __shared__ uint32_t h[257];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int b = threadIdx.x; b < 257; b += 256) h[b] = 0;
  __syncthreads();
  const int64_t seg = (int64_t)blockIdx.x * 4 + wid;
  const int64_t beg = seg * R;
  const int64_t end = beg + R < n ? beg + R : n;
  for (int64_t base = beg; base < end; base += 4 * 256) {
    float4 a[4], b[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t i0 = base + q * 256 + lane * 4;
      if (i0 + 3 < end) {
        a[q] = *reinterpret_cast<const float4*>(x + i0);
        b[q] = *reinterpret_cast<const float4*>(x0 + i0);
      } else {
        a[q] = make_float4(0, 0, 0, 0);
        b[q] = a[q];
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t k4[4] = {keyof(a[q].x, b[q].x), keyof(a[q].y, b[q].y), keyof(a[q].z, b[q].z),
                              keyof(a[q].w, b[q].w)};
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (k4[e] >= thr) atomicAdd(&h[(k4[e] >> 13) & 255], 1u);
    }
  }
  __syncthreads();
  if (FLUSH == 1) {
    uint32_t* g = hist + (blockIdx.x & 15) * 272;
    for (int b = threadIdx.x; b < 257; b += 256)
      if (h[b]) atomicAdd(&g[b], h[b]);
  } else if (FLUSH == 2) {
    uint32_t* row = hist + (int64_t)blockIdx.x * 257;
    for (int b = threadIdx.x; b < 257; b += 256) row[b] = h[b];
  } else {
    if (threadIdx.x == 0) out[blockIdx.x] = h[0];
  }
}

template <int U>
__global__ void __launch_bounds__(256) grid_kernel(const float* __restrict__ x,
                                                   const float* __restrict__ x0, int64_t n,
                                                   uint32_t thr, uint32_t* out) {
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * 256;
  uint32_t c = 0;
  for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < n4; g += stride * U) {
    float4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t gi = g + u * stride;
      if (gi < n4) {
        a[u] = reinterpret_cast<const float4*>(x)[gi];
        b[u] = reinterpret_cast<const float4*>(x0)[gi];
      } else {
        a[u] = make_float4(0, 0, 0, 0);
        b[u] = a[u];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      c += keyof(a[u].x, b[u].x) >= thr;
      c += keyof(a[u].y, b[u].y) >= thr;
      c += keyof(a[u].z, b[u].z) >= thr;
      c += keyof(a[u].w, b[u].w) >= thr;
    }
  }
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = c;
}

// one wave per segment, but the segment is streamed with a 2-deep software pipeline: the next
// iteration's loads are issued before the current one is consumed
template <int G>
__global__ void __launch_bounds__(256) segpipe_kernel(const float* __restrict__ x,
                                                      const float* __restrict__ x0, int64_t n,
                                                      int64_t R, uint32_t thr, uint32_t* out) {
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t seg = (int64_t)blockIdx.x * 4 + wid;
  const int64_t beg = seg * R;
  const int64_t end = beg + R < n ? beg + R : n;
  uint32_t c = 0;
  float4 a[G], b[G];
  auto load = [&](int64_t base) {
#pragma unroll
    for (int q = 0; q < G; ++q) {
      const int64_t i0 = base + q * 256 + lane * 4;
      if (i0 + 3 < end) {
        a[q] = *reinterpret_cast<const float4*>(x + i0);
        b[q] = *reinterpret_cast<const float4*>(x0 + i0);
      } else {
        a[q] = make_float4(0, 0, 0, 0);
        b[q] = a[q];
      }
    }
  };
  load(beg);
  for (int64_t base = beg; base < end; base += G * 256) {
    float4 ca[G], cb[G];
#pragma unroll
    for (int q = 0; q < G; ++q) { ca[q] = a[q]; cb[q] = b[q]; }
    if (base + G * 256 < end) load(base + G * 256);
#pragma unroll
    for (int q = 0; q < G; ++q) {
      c += keyof(ca[q].x, cb[q].x) >= thr;
      c += keyof(ca[q].y, cb[q].y) >= thr;
      c += keyof(ca[q].z, cb[q].z) >= thr;
      c += keyof(ca[q].w, cb[q].w) >= thr;
    }
  }
  if (lane == 0) out[seg] = c;
}

__global__ void init_kernel(float* x, float* x0, int64_t n, uint32_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    const float u1 = (float)(z & 0xFFFFFF) / 16777216.0f, u2 = (float)((z >> 24) & 0xFFFFFF) / 16777216.0f;
    x[i] = 2.0f * u1 - 1.0f;
    x0[i] = x[i] - 0.01f * (2.0f * u2 - 1.0f);
  }
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 11000000;
  const int NSET = argc > 2 ? atoi(argv[2]) : 8;
  const int REPS = 40;
  std::vector<float*> xs(NSET), x0s(NSET);
  for (int s = 0; s < NSET; ++s) {
    CK(hipMalloc(&xs[s], n * 4));
    CK(hipMalloc(&x0s[s], n * 4));
    init_kernel<<<4096, 256>>>(xs[s], x0s[s], n, 17u + s);
  }
  uint32_t* out;
  CK(hipMalloc(&out, 1 << 22));
  uint32_t* hist;
  CK(hipMalloc(&hist, 16 << 20));
  CK(hipMemset(hist, 0, 16 << 20));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch) {
    for (int w = 0; w < 3; ++w) launch(w % NSET);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < REPS; ++r) launch(r % NSET);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / REPS;
    printf("%-28s %8.2f us  %7.1f GB/s\n", name, us, 8.0 * n / us / 1e3);
  };
  // |x - x0| ~ U(0, 0.01): keys >= 0.0098 are the top ~2 % (the filter's candidate rate)
  const float fthr = 0.0098f;
  const uint32_t thr = *reinterpret_cast<const uint32_t*>(&fthr);
  for (int64_t R : {1344LL, 2688LL}) {
    const int64_t W = (n + R - 1) / R;
    const unsigned nb = (unsigned)((W + 3) / 4);
    char nm[64];
    snprintf(nm, sizeof nm, "flush none R=%lld", (long long)R);
    run(nm, [&](int s) { segflush_kernel<0><<<nb, 256>>>(xs[s], x0s[s], n, R, thr, out, hist); });
    snprintf(nm, sizeof nm, "flush atomics16 R=%lld", (long long)R);
    run(nm, [&](int s) { segflush_kernel<1><<<nb, 256>>>(xs[s], x0s[s], n, R, thr, out, hist); });
    snprintf(nm, sizeof nm, "flush rows R=%lld", (long long)R);
    run(nm, [&](int s) { segflush_kernel<2><<<nb, 256>>>(xs[s], x0s[s], n, R, thr, out, hist); });
  }
  for (int64_t R : {1344LL, 2688LL, 5376LL, 10752LL}) {
    const int64_t W = (n + R - 1) / R;
    const unsigned nb = (unsigned)((W + 3) / 4);
    char nm[64];
    snprintf(nm, sizeof nm, "seg<4> R=%lld W=%lld", (long long)R, (long long)W);
    run(nm, [&](int s) { seg_kernel<4><<<nb, 256>>>(xs[s], x0s[s], n, R, thr, out); });
    snprintf(nm, sizeof nm, "seg<2> R=%lld", (long long)R);
    run(nm, [&](int s) { seg_kernel<2><<<nb, 256>>>(xs[s], x0s[s], n, R, thr, out); });
    snprintf(nm, sizeof nm, "segpipe<2> R=%lld", (long long)R);
    run(nm, [&](int s) { segpipe_kernel<2><<<nb, 256>>>(xs[s], x0s[s], n, R, thr, out); });
    snprintf(nm, sizeof nm, "segpipe<4> R=%lld", (long long)R);
    run(nm, [&](int s) { segpipe_kernel<4><<<nb, 256>>>(xs[s], x0s[s], n, R, thr, out); });
  }
  for (unsigned g : {1024u, 2048u, 4096u}) {
    char nm[64];
    snprintf(nm, sizeof nm, "grid<2> blocks=%u", g);
    run(nm, [&](int s) { grid_kernel<2><<<g, 256>>>(xs[s], x0s[s], n, thr, out); });
    snprintf(nm, sizeof nm, "grid<4> blocks=%u", g);
    run(nm, [&](int s) { grid_kernel<4><<<g, 256>>>(xs[s], x0s[s], n, thr, out); });
  }
  return 0;
}
