// Replace-only decode of ONE sparse payload (reference sharing/PartialModel.py:257-303,
// `T = cat(local); T[idx] = params`), as a device function on payload-entry chunks, shared by the
// standalone replace kernel (dpz_fold.hip) and the encoder's co-scheduled decode (a replace job
// carried by the latency-bound top-k kernels in blocks of their own, dpz_topk_sampled.hip).
//
// Chunk c owns payload entries [RP_E c, RP_E c + RP_E) and the element range from its first
// entry's index to the next chunk's first entry's index (chunk 0 from 0, the last chunk to n):
// a contiguous partition of [0, n) known after one load, so no tile-offset pre-pass and no
// chunk's entries land in another chunk's range.  The chunk streams its range local -> out
// (float4, non-temporal loads and stores) and merges its entries' values into the loaded
// registers before the store (a binary search over the entries held one per lane).
#pragma once
#include "dpz_common.h"

namespace dpz {

#ifndef DPZ_RP_E
#define DPZ_RP_E 16
#endif
constexpr int RP_E = DPZ_RP_E;  // payload entries per chunk (one wave's unit of work)
static_assert(RP_E >= 1 && RP_E <= 64, "a chunk's entries are held one per lane");
#ifndef DPZ_RP_U
#define DPZ_RP_U 4
#endif
constexpr int RP_U = DPZ_RP_U;  // float4 loads per lane in flight in the range copy
typedef float rp_v4f __attribute__((ext_vector_type(4)));

// Non-temporal (streaming) policy of the range copy: 2 = nt loads of local and nt stores of out
// (the once-touched 4N bytes do not evict the next kernel's inputs from the L3), 1 = nt stores
// only, 0 = default policy.
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
  int scatter;     // 1: out already holds local (the encoder's filter copied it while streaming
                   // the same tensor): only the entries are written, 64 per chunk (replace only)
};

static inline int64_t replace_chunks(int64_t k) { return (k + RP_E - 1) / RP_E; }
static inline int64_t scatter_chunks(int64_t k) { return (k + 63) / 64; }

// A chunk's entries, one per lane: rel = index relative to the slice, clamped to [-1, n] (lanes
// past the chunk's end hold INT32_MAX), ev = value; bnext = the next chunk's first index (the
// end of this chunk's range) or n.  Issued as loads only: a caller may keep them in flight.
struct RpChunk {
  int32_t rel;
  float ev;
  int64_t bnext;
};

__device__ __forceinline__ RpChunk rp_load(const ReplaceJob& j, int64_t c, int lane) {
  RpChunk r{INT32_MAX, 0.0f, j.n};
  const int64_t e0 = c * RP_E;
  const int64_t e1 = (e0 + RP_E < j.k) ? e0 + RP_E : j.k;
  if (lane < e1 - e0) {
    const int64_t v = (int64_t)j.idx[e0 + lane] - j.off;
    r.rel = (int32_t)(v < -1 ? -1 : (v > j.n ? j.n : v));  // outside the slice: never an element
    r.ev = j.val[e0 + lane];
  }
  if (e1 < j.k) r.bnext = (int64_t)j.idx[e1] - j.off;
  return r;
}

// One scalar element i (valid) merged with the chunk's entries: replace -> the entry's value,
// add -> local + value (local + 0.0 off the entries).  Wave-uniform call.
__device__ __forceinline__ float rp_scalar(const RpChunk& ch, const float* local, int64_t i,
                                           bool valid, bool add) {
  const float raw = valid ? local[i] : 0.0f;
  float w = add ? raw + 0.0f : raw;
  const int32_t key = valid ? (int32_t)i : INT32_MIN;
  for (int p = 0; p < RP_E; ++p) {  // RP_E readlanes, one scalar element: head / tail only
    const int32_t ie = __builtin_amdgcn_readlane(ch.rel, p);
    const float iv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ch.ev), p));
    if (valid && ie == key) w = add ? raw + iv : iv;
  }
  return w;
}

// Chunk c streamed by one wave: out[a, b) = local[a, b) with the chunk's entries merged in
// registers before the store (each output line is written once, whole).  [a, b) runs from the
// chunk's first entry (0 for chunk 0) to the next chunk's first entry (n for the last): a
// contiguous partition of [0, n), clamped so an invalid payload cannot fault.
__device__ __forceinline__ void rp_stream(const ReplaceJob& j, int64_t c, int lane,
                                          const RpChunk& ch) {
  const float* __restrict__ local = j.local;
  float* __restrict__ out = j.out;
  const int64_t n = j.n;
  int64_t a = c == 0 ? 0 : (int64_t)__builtin_amdgcn_readlane(ch.rel, 0);
  int64_t b = ch.bnext;
  a = a < 0 ? 0 : (a > n ? n : a);
  b = b < 0 ? 0 : (b > n ? n : b);
  if (a >= b) return;
  const bool add = j.add != 0;
  // the float4 body starts and ends on 128-byte lines (32 elements): every wave-instruction
  // reads and writes 8 whole lines, the ragged ends are scalar
  const int64_t a4 = (a + 31) & ~int64_t(31);
  const int64_t b4 = b & ~int64_t(31);
  if (a4 >= b4) {  // short range: scalar elements
    for (int64_t base = a; base < b; base += 64) {
      const int64_t i = base + lane;
      const float w = rp_scalar(ch, local, i, i < b, add);
      if (i < b) out[i] = w;
    }
    return;
  }
  {  // head [a, a4): lanes 0..30, tail [b4, b): lanes 32..62
    const bool head = lane < a4 - a;
    const bool tail = lane >= 32 && lane - 32 < b - b4;
    const int64_t i = head ? a + lane : (tail ? b4 + (lane - 32) : a);
    const float w = rp_scalar(ch, local, i, head || tail, add);
    if (head || tail) out[i] = w;
  }
  const rp_v4f* __restrict__ lv = reinterpret_cast<const rp_v4f*>(local);
  rp_v4f* __restrict__ ov = reinterpret_cast<rp_v4f*>(out);
  const int64_t q0 = a4 >> 2, q1 = b4 >> 2;
  const rp_v4f z = {0.f, 0.f, 0.f, 0.f};
  // passes of RP_U float4 per lane: every load of a pass is issued before its merges / stores
  for (int64_t base = q0; base < q1; base += RP_U * 64) {
    rp_v4f v[RP_U];
#pragma unroll
    for (int u = 0; u < RP_U; ++u) {
      const int64_t q = base + u * 64 + lane;
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
      const int64_t qw = base + u * 64;  // the wave's 64 groups: elements [4 qw, 4 qw + 256)
      if (qw >= q1) break;
      const int64_t q = qw + lane;
      const bool in = q < q1;
      const rp_v4f x = add ? v[u] + z : v[u];  // add: local + 0.0 off the entries
      float w[4] = {x.x, x.y, x.z, x.w};
      // the entries inside the window are the lanes [p0, p1) (sorted: two ballots), applied
      // one by one from scalar registers by the lane that holds the element
      const int32_t ws = (int32_t)(4 * qw);
      const int p0 = __popcll(__ballot(ch.rel < ws));
      const int p1 = __popcll(__ballot(ch.rel < ws + 256));
      for (int p = p0; p < p1; ++p) {
        const int32_t o = __builtin_amdgcn_readlane(ch.rel, p) - ws;
        const float iv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ch.ev), p));
        if (in && (o >> 2) == lane) {
          const int e = o & 3;
          const float r = e == 0 ? v[u].x : e == 1 ? v[u].y : e == 2 ? v[u].z : v[u].w;
          const float nv = add ? r + iv : iv;
          w[0] = e == 0 ? nv : w[0];
          w[1] = e == 1 ? nv : w[1];
          w[2] = e == 2 ? nv : w[2];
          w[3] = e == 3 ? nv : w[3];
        }
      }
      if (in) {
        const rp_v4f r = {w[0], w[1], w[2], w[3]};
#if DPZ_REPLACE_NT >= 1
        __builtin_nontemporal_store(r, &ov[q]);
#else
        ov[q] = r;
#endif
      }
    }
  }
}

// A whole block of blockDim.x (a multiple of 64) threads runs chunks j.c0 + p * waves + wave
// (the co-scheduled decode inside the encoder's launches): no barrier, waves independent.
__device__ __forceinline__ void replace_block(const ReplaceJob& j, int64_t p) {
  const int per = (int)(blockDim.x >> 6);
  const int64_t c = j.c0 + p * per + (threadIdx.x >> 6);
  if (c >= j.c1) return;
  const int lane = threadIdx.x & 63;
  if (j.scatter) {
    // out[idx[e]] = val[e] for the chunk's 64 entries; of equal (adjacent, the indices are
    // sorted) indices the last entry wins, as in the sequential `T[idx] = params`
    const int64_t e = c * 64 + lane;
    if (e < j.k) {
      const int64_t i = (int64_t)j.idx[e] - j.off;
      const bool last = e + 1 >= j.k || j.idx[e + 1] != j.idx[e];
      if (last && i >= 0 && i < j.n) j.out[i] = j.val[e];
    }
    return;
  }
  const RpChunk ch = rp_load(j, c, lane);
  rp_stream(j, c, lane, ch);
}

// host: the standalone replace kernel over chunks [j.c0, j.c1) (dpz_fold.hip)
int launch_replace(const ReplaceJob& j, hipStream_t st);

}  // namespace dpz
