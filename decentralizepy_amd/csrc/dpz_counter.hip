// The share counter kept as a ring of sent index lists, applied on read (dpz_counter_flush).
//
// Reference: sharing/PartialModel.py:205-207 (`shared_parameters_counter[indices] += 1` every
// round) whose only reader is the node's end-of-run dump (node/DPSGDNode.py:186-194).  Updating
// the int32 counter in the encode costs one scattered read-modify-write per selected index: at
// 1 % density nearly every index owns its 128-byte line, ~95 bytes of HBM traffic each (compact's
// PMC at 64 MiB: 19.3 MB for 3.4 MB of payload).  Instead the plugin keeps each round's payload
// indices (already written: the wire payload itself) in a device ring and folds the ring into the
// counter when it is read or full:
//   SCATTER : one atomic per ring entry (few entries: cheaper than touching the whole counter)
//   SWEEP   : one block per tile of CT counters: the tile is read into LDS, every ring segment's
//             entries inside the tile (a binary-searched contiguous range: each segment is a
//             strictly ascending payload) are added with LDS atomics, the tile is written back —
//             8n coalesced bytes + 4 per entry, whatever the number of rounds in the ring.
#include "dpz_common.h"

namespace dpz {
namespace {

constexpr int CT = 8192;     // counters per sweep tile (32 KB of LDS)
constexpr int CSEGS = 64;    // ring segments per sweep launch (their offsets are kernel arguments)

struct SegTab {
  int64_t off[CSEGS + 1];    // segment r = ring[off[r], off[r + 1])
  int m;
};

__global__ void __launch_bounds__(256) counter_scatter_kernel(int32_t* __restrict__ counter,
                                                              int64_t n,
                                                              const int32_t* __restrict__ ring,
                                                              int64_t total) {
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < total;
       j += (int64_t)gridDim.x * 256) {
    const uint32_t i = (uint32_t)ring[j];
    if ((int64_t)i < n) atomicAdd(&counter[i], 1);
  }
}

// first position p in [b, e) with ring[p] >= v (ring[b, e) ascending)
__device__ __forceinline__ int64_t lower_pos(const int32_t* __restrict__ ring, int64_t b,
                                             int64_t e, int64_t v) {
  while (b < e) {
    const int64_t mid = b + ((e - b) >> 1);
    if ((int64_t)ring[mid] < v) b = mid + 1;
    else e = mid;
  }
  return b;
}

__global__ void __launch_bounds__(256) counter_sweep_kernel(int32_t* __restrict__ counter,
                                                            int64_t n,
                                                            const int32_t* __restrict__ ring,
                                                            const SegTab tab) {
  __shared__ int32_t tile[CT];
  __shared__ int64_t sb[CSEGS], se[CSEGS];
  const int m = tab.m;
  const int t = threadIdx.x;
  const int64_t t0 = (int64_t)blockIdx.x * CT;
  const int64_t t1 = t0 + CT < n ? t0 + CT : n;
  const int cnt = (int)(t1 - t0);
  const bool full = cnt == CT && (reinterpret_cast<uintptr_t>(counter) & 15u) == 0;
  // the tile's counters first (their loads in flight while the segment ranges are searched)
  if (full) {
    const int4* src = reinterpret_cast<const int4*>(counter + t0);
#pragma unroll
    for (int q = 0; q < CT / 1024; ++q) reinterpret_cast<int4*>(tile)[t + 256 * q] = src[t + 256 * q];
  } else {
    for (int i = t; i < cnt; i += 256) tile[i] = counter[t0 + i];
  }
  if (t < m) {  // segment t's entries inside [t0, t1): one contiguous range (ascending)
    const int64_t b = tab.off[t], e = tab.off[t + 1];
    const int64_t lo = lower_pos(ring, b, e, t0);
    sb[t] = lo;
    se[t] = lower_pos(ring, lo, e, t1);
  }
  __syncthreads();
  for (int r = 0; r < m; ++r) {
    const int64_t b = sb[r], e = se[r];
    for (int64_t j = b + t; j < e; j += 256) {
      // inside the tile by the search when the segment is ascending; checked all the same (a
      // caller's unsorted segment must not write outside the tile)
      const int64_t i = (int64_t)ring[j] - t0;
      if (i >= 0 && i < cnt) atomicAdd(&tile[i], 1);
    }
  }
  __syncthreads();
  if (full) {
    int4* dst = reinterpret_cast<int4*>(counter + t0);
#pragma unroll
    for (int q = 0; q < CT / 1024; ++q) dst[t + 256 * q] = reinterpret_cast<const int4*>(tile)[t + 256 * q];
  } else {
    for (int i = t; i < cnt; i += 256) counter[t0 + i] = tile[i];
  }
}

}  // namespace
}  // namespace dpz

using namespace dpz;

extern "C" int dpz_counter_flush(int32_t* counter, int64_t n, const int32_t* ring,
                                 const int64_t* seg_off, int m, int mode, dpz_stream_t stream) {
  if (n < 0 || m < 0 || n >= (int64_t(1) << 31)) return DPZ_ERR_ARG;
  if (mode < DPZ_COUNTER_AUTO || mode > DPZ_COUNTER_SWEEP) return DPZ_ERR_ARG;
  if (m == 0 || n == 0) return DPZ_OK;
  if (!seg_off || seg_off[0] != 0) return DPZ_ERR_ARG;
  for (int r = 0; r < m; ++r)
    if (seg_off[r + 1] < seg_off[r] || seg_off[r + 1] - seg_off[r] > n) return DPZ_ERR_ARG;
  const int64_t total = seg_off[m];
  if (total == 0) return DPZ_OK;
  if (!counter || !ring) return DPZ_ERR_ARG;
  hipStream_t st = static_cast<hipStream_t>(stream);
  // an entry scattered costs ~one 128-byte line read-modify-write (~95 B measured, compact's PMC);
  // a sweep reads and writes the counter once (8n) and reads every entry (4 B)
  bool sweep = mode == DPZ_COUNTER_SWEEP;
  if (mode == DPZ_COUNTER_AUTO) sweep = (double)total * 91.0 > 8.0 * (double)n;
  if (sweep) {
    const int64_t tiles = (n + CT - 1) / CT;
    for (int r0 = 0; r0 < m; r0 += CSEGS) {  // CSEGS segments per pass over the counter
      SegTab tab{};
      tab.m = m - r0 < CSEGS ? m - r0 : CSEGS;
      for (int r = 0; r <= tab.m; ++r) tab.off[r] = seg_off[r0 + r];
      DPZ_TIMED(DPZ_KT_COUNTER, st,
                counter_sweep_kernel<<<(unsigned)tiles, 256, 0, st>>>(counter, n, ring, tab));
    }
  } else {
    int64_t g = (total + 255) / 256;
    if (g > 8192) g = 8192;
    DPZ_TIMED(DPZ_KT_COUNTER, st,
              counter_scatter_kernel<<<(unsigned)g, 256, 0, st>>>(counter, n, ring, total));
  }
  return DPZ_OK;
}
