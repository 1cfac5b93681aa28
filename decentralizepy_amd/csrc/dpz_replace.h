// Replace-only decode of ONE sparse payload (reference sharing/PartialModel.py:257-303,
// `T = cat(local); T[idx] = params`), as a device function on payload-entry chunks, shared by the
// standalone replace kernel (dpz_fold.hip) and the encoder's co-scheduled decode (a replace job
// carried by the latency-bound top-k kernels in blocks of their own, dpz_topk_sampled.hip).
//
// Chunk c owns payload entries [RP_E c, RP_E c + RP_E) and the element range from its first
// entry's index to the next chunk's first entry's index (chunk 0 from 0, the last chunk to n):
// a contiguous partition of [0, n) known after one load, so no tile-offset pre-pass and no
// chunk's scatter lands in another chunk's range.  The chunk copies its range local -> out
// (float4 body, non-temporal), then scatters its entries' values.
#pragma once
#include "dpz_common.h"

namespace dpz {

#ifndef DPZ_RP_E
#define DPZ_RP_E 64
#endif
constexpr int RP_E = DPZ_RP_E;  // payload entries per chunk (one 256-thread sub-block)
#ifndef DPZ_RP_U
#define DPZ_RP_U 8
#endif
constexpr int RP_U = DPZ_RP_U;  // float4 loads per thread in flight in the range copy
typedef float rp_v4f __attribute__((ext_vector_type(4)));

// Non-temporal (streaming) policy of the range copy: 2 = nt loads of local and nt stores of out
// (measured on MI355X in the encode+decode step: C2 570 -> 606 GiB/s together with the filter's
// nt loads; the once-touched 4N bytes no longer evict the next kernel's inputs from the L3),
// 1 = nt stores only, 0 = default policy.
#ifndef DPZ_REPLACE_NT
#define DPZ_REPLACE_NT 2
#endif

struct ReplaceJob {
  const float* local;
  const int32_t* idx;
  const float* val;
  int64_t k, n;
  float* out;
  int64_t c0, c1;  // chunks [c0, c1) of this launch
  int add;         // 0: out = local with entries replaced; 1: out = local + T (T zero-based)
  int64_t off;     // payload indices are global; element i of local / out is global off + i
                   // (a rank's slice of a sharded model; entries outside [0, n) are skipped)
};

static inline int64_t replace_chunks(int64_t k) { return (k + RP_E - 1) / RP_E; }

// One 256-thread sub-block (t = its thread index) runs chunk c when `valid`.  Contains exactly
// one __syncthreads(): every thread of the enclosing block must call it (valid or not).
__device__ __forceinline__ void replace_chunk(const ReplaceJob& j, int64_t c, bool valid, int t) {
  int64_t my_i = -1;
  float my_v = 0.0f;
  if (valid) {
    const float* __restrict__ local = j.local;
    float* __restrict__ out = j.out;
    const int64_t k = j.k, n = j.n;
    const int64_t e0 = c * RP_E;
    const int64_t e1 = (e0 + RP_E < k) ? e0 + RP_E : k;
    int64_t a = c == 0 ? 0 : (int64_t)j.idx[e0] - j.off;
    int64_t b = e1 >= k ? n : (int64_t)j.idx[e1] - j.off;
    // an invalid payload (indices outside [0, n)) must not fault: clamp the range
    a = a < 0 ? 0 : (a > n ? n : a);
    b = b < 0 ? 0 : (b > n ? n : b);
    if (t < e1 - e0) {
      my_i = (int64_t)j.idx[e0 + t] - j.off;
      my_v = j.val[e0 + t];
    }
    if (a < b) {
      const int64_t a4 = (a + 3) & ~int64_t(3);
      const int64_t b4 = b & ~int64_t(3);
      if (a4 < b4) {
        if (t < a4 - a) out[a + t] = j.add ? local[a + t] + 0.0f : local[a + t];
        if (t < b - b4) out[b4 + t] = j.add ? local[b4 + t] + 0.0f : local[b4 + t];
        const rp_v4f* __restrict__ lv = reinterpret_cast<const rp_v4f*>(local);
        rp_v4f* __restrict__ ov = reinterpret_cast<rp_v4f*>(out);
        const int64_t q1 = b4 >> 2;
        // replace: a bit copy; add: out = local + 0.0 off the entries, as the reference's dense
        // `local + T` (fl(-0 + +0) = +0, NaNs quieted) — a uniform branch per launch
        const bool add = j.add != 0;
        const rp_v4f z = {0.f, 0.f, 0.f, 0.f};
        // passes of RP_U float4 per thread: every load of a pass is issued before its stores
        // (guarded, no remainder loop of dependent load -> store trips)
        for (int64_t base = (a4 >> 2) + t; base < q1; base += RP_U * 256) {
          rp_v4f v[RP_U];
#pragma unroll
          for (int u = 0; u < RP_U; ++u) {
            const int64_t q = base + u * 256;
            if (q < q1) {
#if DPZ_REPLACE_NT >= 2
              v[u] = __builtin_nontemporal_load(&lv[q]);
#else
              v[u] = lv[q];
#endif
            }
          }
#pragma unroll
          for (int u = 0; u < RP_U; ++u) {
            const int64_t q = base + u * 256;
            if (q < q1) {
              const rp_v4f w = add ? v[u] + z : v[u];
#if DPZ_REPLACE_NT >= 1
              __builtin_nontemporal_store(w, &ov[q]);
#else
              ov[q] = w;
#endif
            }
          }
        }
      } else {
        for (int64_t i = a + t; i < b; i += 256) out[i] = j.add ? local[i] + 0.0f : local[i];
      }
    }
  }
  __syncthreads();  // the range copy is in place before this chunk's entries overwrite it
  if (my_i >= 0 && my_i < j.n) j.out[my_i] = j.add ? j.local[my_i] + my_v : my_v;
}

// A whole block of blockDim.x (a multiple of 256) threads: sub-block s runs chunk
// j.c0 + p * (blockDim.x / 256) + s.
__device__ __forceinline__ void replace_block(const ReplaceJob& j, int64_t p) {
  const int per = (int)(blockDim.x >> 8);
  const int64_t c = j.c0 + p * per + (threadIdx.x >> 8);
  replace_chunk(j, c, c < j.c1, (int)(threadIdx.x & 255));
}

// host: the standalone replace kernel over chunks [j.c0, j.c1) (dpz_fold.hip)
int launch_replace(const ReplaceJob& j, hipStream_t st);

}  // namespace dpz
