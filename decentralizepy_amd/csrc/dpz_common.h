// Shared device helpers for the dpz codec kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/dpz_codec.h"
#include "dpz_knobs.h"

#define DPZ_WAVE 64

#define DPZ_HIP_TRY(expr)                                   \
  do {                                                      \
    hipError_t _e = (expr);                                 \
    if (_e != hipSuccess) return (int)_e;                   \
  } while (0)

#define DPZ_LAUNCH_CHECK() DPZ_HIP_TRY(hipGetLastError())

namespace dpz {
// dpz_timing.hip: optional per-kernel event timing (no-ops unless dpz_timing_enable(1))
int timing_begin(int id, hipStream_t st);
void timing_end(int slot, hipStream_t st);
}  // namespace dpz

// launch + error check, bracketed by timing events when timing is enabled
#define DPZ_TIMED(id, st, ...)                          \
  do {                                                  \
    const int _dpz_tslot = ::dpz::timing_begin(id, st); \
    __VA_ARGS__;                                        \
    DPZ_LAUNCH_CHECK();                                 \
    ::dpz::timing_end(_dpz_tslot, st);                  \
  } while (0)

namespace dpz {

// |c| as an order-preserving uint32 key: sign cleared, every NaN -> 0x7FC00000 so that NaNs
// rank above +inf and tie with each other (torch.topk treats NaN as the largest value).
__device__ __forceinline__ uint32_t key_of(float c) {
  uint32_t b = __float_as_uint(c) & 0x7FFFFFFFu;
  return b > 0x7F800000u ? 0x7FC00000u : b;
}

// Exclusive prefix of `v` over the 64 lanes of a wave plus the wave total (in *total).
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t* total) {
  const int lane = threadIdx.x & 63;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  *total = __shfl(x, 63, 64);
  return x - v;
}

// Block-wide exclusive scan (blockDim.x multiple of 64, <= 1024). `wsum` is LDS scratch of at
// least 16 words. Returns the exclusive prefix; *total gets the block sum. Contains barriers:
// every thread of the block must call it.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* wsum, uint32_t* total) {
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nw = blockDim.x >> 6;
  uint32_t wt;
  uint32_t ex = wave_excl_scan(v, &wt);
  if (lane == 0) wsum[wid] = wt;
  __syncthreads();
  uint32_t off = 0, tot = 0;
  for (int w = 0; w < nw; ++w) {
    uint32_t s = wsum[w];
    off += (w < wid) ? s : 0u;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return ex + off;
}

// Block-wide exclusive scan on 64-bit values (same contract as block_excl_scan).
__device__ __forceinline__ uint64_t block_excl_scan64(uint64_t v, uint64_t* wsum, uint64_t* total) {
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nw = blockDim.x >> 6;
  uint64_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint64_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  uint64_t off = 0, tot = 0;
  for (int w = 0; w < nw; ++w) {
    uint64_t s = wsum[w];
    off += (w < wid) ? s : 0ull;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return x - v + off;
}

__host__ __device__ __forceinline__ bool aligned16(const void* p) {
  return (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
}

// A payload value as stored: fp32, or (DPZ_TOPK_VAL_FP16) fp16 rounded to nearest even, the
// torch.Tensor.half() conversion (overflow -> inf, NaN stays NaN), in the same slot order.
__device__ __forceinline__ void store_val(float* val_out, int val_h, int64_t pos, float v) {
  if (val_h) {
    const _Float16 h = (_Float16)v;
    reinterpret_cast<uint16_t*>(val_out)[pos] = __builtin_bit_cast(uint16_t, h);
  } else {
    val_out[pos] = v;
  }
}

// The Metro-Hastings fold's value at an element no payload hits (every term is the local value
// x): fl(...fl(fl(x*w[0]) + fl(x*w[1])) ... + fl(x*ws)), the reference's fp32 order
// (sharing/Sharing.py:156-190; the library is compiled with -ffp-contract=off).  Written by the
// encoder's filter while it streams x (dpz_topk_encode_foldbase) so that the decode only
// rewrites the elements its payloads hit (DPZ_FOLD_BASE_READY).
constexpr int FOLDBASE_MAXW = 16;
struct FoldBase {
  int nw;                  // payload weights, 1 .. FOLDBASE_MAXW
  float w[FOLDBASE_MAXW];
  float ws;                // the self weight
  __device__ __forceinline__ float of(float x) const {
    float t = x * w[0];
    for (int p = 1; p < nw; ++p) t = t + x * w[p];
    return t + x * ws;
  }
};

}  // namespace dpz
