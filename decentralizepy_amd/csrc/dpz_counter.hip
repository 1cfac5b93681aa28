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
//   SWEEP   : a bounds pass over the entries (where each segment enters each tile: a segment is a
//             strictly ascending payload), then one block per tile of CT counters: the tile is
//             read into LDS, every segment's entries inside it (a contiguous range) are added
//             with LDS atomics, the tile is written back — 8n coalesced bytes + 8 per entry,
//             whatever the number of rounds in the ring.
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

// bounds[r * (tiles + 1) + t] = the first position q of segment r (relative to its start) whose
// index is >= t * CT, for t = 0 .. tiles: entry q writes the tiles its index opens (those after
// the previous entry's tile up to its own), the segment's last entry the tiles after it — every
// word once for an ascending segment.  Replaces a per-tile binary search (a chain of ~17
// dependent loads per segment in every sweep block).
__global__ void __launch_bounds__(256) counter_bounds_kernel(const int32_t* __restrict__ ring,
                                                             const SegTab tab, int64_t tiles,
                                                             int32_t* __restrict__ bounds) {
  const int r = blockIdx.y;
  const int64_t b = tab.off[r], len = tab.off[r + 1] - b;
  int32_t* br = bounds + (int64_t)r * (tiles + 1);
  if (len == 0) {
    for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t <= tiles;
         t += (int64_t)gridDim.x * 256)
      br[t] = 0;
    return;
  }
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < len;
       q += (int64_t)gridDim.x * 256) {
    const int64_t tv = (int64_t)(uint32_t)ring[b + q] / CT;
    const int64_t tp = q > 0 ? (int64_t)(uint32_t)ring[b + q - 1] / CT : -1;
    const int64_t hi = tv < tiles ? tv : tiles;
    for (int64_t t = tp + 1; t <= hi; ++t) br[t] = (int32_t)q;
    if (q == len - 1)
      for (int64_t t = (tv + 1 > tp + 1 ? tv + 1 : tp + 1); t <= tiles; ++t) br[t] = (int32_t)len;
  }
}

__global__ void __launch_bounds__(256) counter_sweep_kernel(int32_t* __restrict__ counter,
                                                            int64_t n,
                                                            const int32_t* __restrict__ ring,
                                                            const SegTab tab, int64_t tiles,
                                                            const int32_t* __restrict__ bounds) {
  __shared__ int32_t tile[CT];
  __shared__ int64_t sb[CSEGS];
  __shared__ int32_t pre[CSEGS + 1];  // the tile's entries of segments < r: pre[r]
  const int m = tab.m;
  const int t = threadIdx.x;
  const int64_t t0 = (int64_t)blockIdx.x * CT;
  const int64_t t1 = t0 + CT < n ? t0 + CT : n;
  const int cnt = (int)(t1 - t0);
  const bool full = cnt == CT && (reinterpret_cast<uintptr_t>(counter) & 15u) == 0;
  // segment t's entries inside [t0, t1): one contiguous range of an ascending segment (clamped
  // to the segment: bounds of a segment that is not ascending are not trusted)
  int64_t lo = 0, hi = 0;
  if (t < m) {
    const int64_t len = tab.off[t + 1] - tab.off[t];
    const int32_t* br = bounds + (int64_t)t * (tiles + 1) + blockIdx.x;
    int64_t a = br[0], e = br[1];
    a = a < 0 ? 0 : (a > len ? len : a);
    e = e < a ? a : (e > len ? len : e);
    lo = tab.off[t] + a;
    hi = tab.off[t] + e;
  }
  if (full) {
    const int4* src = reinterpret_cast<const int4*>(counter + t0);
#pragma unroll
    for (int q = 0; q < CT / 1024; ++q) reinterpret_cast<int4*>(tile)[t + 256 * q] = src[t + 256 * q];
  } else {
    for (int i = t; i < cnt; i += 256) tile[i] = counter[t0 + i];
  }
  // the tile's entries of all segments as ONE index space [0, total): a wave scan of the
  // per-segment counts (m <= 64), then every thread takes entries j, j + 256, ... — the ring
  // loads are independent (a loop per segment had put one load round trip per segment in
  // series: 64 rounds, ~50 us per launch)
  if (t < 64) {
    const int32_t c = t < m ? (int32_t)(hi - lo) : 0;
    int32_t v = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int32_t u = __shfl_up(v, d, 64);
      if (t >= d) v += u;
    }
    if (t < m) {
      sb[t] = lo;
      pre[t] = v - c;
    }
    if (t == 63) pre[m] = v;
  }
  __syncthreads();
  const int32_t total = pre[m];
  constexpr int U = 4;
  for (int32_t j0 = t; j0 < total; j0 += 256 * U) {
    int32_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int32_t j = j0 + 256 * u;
      v[u] = -1;
      if (j < total) {
        int a = 0, b = m - 1;  // the segment r with pre[r] <= j < pre[r + 1]
        while (a < b) {
          const int c = (a + b + 1) >> 1;
          if (pre[c] <= j) a = c; else b = c - 1;
        }
        v[u] = ring[sb[a] + (j - pre[a])];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      // inside the tile for an ascending segment; checked all the same (a caller's unsorted
      // segment must not write outside the tile)
      const int64_t i = (int64_t)v[u] - t0;
      if (v[u] >= 0 && i >= 0 && i < cnt) atomicAdd(&tile[i], 1);
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

extern "C" size_t dpz_counter_flush_workspace_bytes(int64_t n) {
  const int64_t tiles = (n > 0 ? n : 1) / CT + 1;
  return (size_t)CSEGS * (size_t)(tiles + 1) * sizeof(int32_t);
}

extern "C" int dpz_counter_flush(int32_t* counter, int64_t n, const int32_t* ring,
                                 const int64_t* seg_off, int m, int mode, void* ws,
                                 size_t ws_bytes, dpz_stream_t stream) {
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
  // a sweep reads and writes the counter once (8n) and reads every entry twice (8 B)
  bool sweep = mode == DPZ_COUNTER_SWEEP;
  if (mode == DPZ_COUNTER_AUTO) sweep = (double)total * 87.0 > 8.0 * (double)n;
  if (sweep) {
    if (!ws || ws_bytes < dpz_counter_flush_workspace_bytes(n)) return DPZ_ERR_WORKSPACE;
    const int64_t tiles = (n + CT - 1) / CT;
    int32_t* bounds = static_cast<int32_t*>(ws);
    for (int r0 = 0; r0 < m; r0 += CSEGS) {  // CSEGS segments per pass over the counter
      SegTab tab{};
      tab.m = m - r0 < CSEGS ? m - r0 : CSEGS;
      for (int r = 0; r <= tab.m; ++r) tab.off[r] = seg_off[r0 + r];
      int64_t longest = 0;
      for (int r = 0; r < tab.m; ++r)
        if (tab.off[r + 1] - tab.off[r] > longest) longest = tab.off[r + 1] - tab.off[r];
      int64_t gx = (longest + 255) / 256;
      gx = gx < 1 ? 1 : (gx > 1024 ? 1024 : gx);
      DPZ_TIMED(DPZ_KT_COUNTER, st,
                counter_bounds_kernel<<<dim3((unsigned)gx, (unsigned)tab.m), 256, 0, st>>>(
                    ring, tab, tiles, bounds));
      DPZ_TIMED(DPZ_KT_COUNTER, st,
                counter_sweep_kernel<<<(unsigned)tiles, 256, 0, st>>>(counter, n, ring, tab, tiles,
                                                                      bounds));
    }
  } else {
    int64_t g = (total + 255) / 256;
    if (g > 8192) g = 8192;
    DPZ_TIMED(DPZ_KT_COUNTER, st,
              counter_scatter_kernel<<<(unsigned)g, 256, 0, st>>>(counter, n, ring, total));
  }
  return DPZ_OK;
}
