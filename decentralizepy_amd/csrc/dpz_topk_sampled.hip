// Sampled single-read top-k (k <= n/16).  See dpz_topk.hip for the contract.
//
// Work unit = one WAVE streaming one contiguous "wave segment" of R elements: ordered compaction
// inside a segment is a ballot + mbcnt prefix (no LDS scan, no barriers in the streaming loop),
// so the 32 waves of a CU drift apart and keep HBM busy.  Five kernels per call:
//   sample  : 64 blocks histogram 65,536 sampled keys (1024 chunks x 64) into chist[key >> 20];
//             zero this call's window-histogram copies and boundary sub-list counters
//   filter  : per block, wave 0 turns chist into the key window [lo, hi) while every wave's first
//             loads are in flight; each wave streams its segment once (x, x0[, acc] -> key),
//             appends keys >= lo in index order to its candidate list (idx, key; staged in LDS
//             and flushed in coalesced chunks) and bins them into a 256-bin window histogram in
//             LDS, folded into copy (block % 16) of the global histogram with atomics
//   select  : 32 segments per block: sum the 16 copies, threshold bin b* (wave 0), per filter
//             block the count above b*, bin-b* entries staged in LDS and appended to sub-list
//             (block % 16) with one atomic (a contended device-scope atomic costs ~20 ns per
//             arrival on MI355X, so no single global counter anywhere)
//   resolve : 1 block: radix select over the ~k/256 boundary entries -> exact threshold T and
//             tie cut (lowest index); every filter block's output offset (scan of above +
//             selected boundary counts over <= 2048 blocks); checks the total == k
//   compact : per filter block: each wave counts, takes its offset inside the block's range and
//             writes its selected (idx, vals_src[idx]) in index order (+ counter / rewind)
// A miss (window does not bracket the k-th key / boundary overflow) sets ctrl->status and compact
// writes nothing; the host then runs the exact path.  A segment whose candidates overflow its
// list is DENSE and re-reads its input range in select / compact (still exact).
#include <cstdio>
#include <cstdlib>

#include "dpz_topk.h"

namespace dpz {

// x / x0 are streamed once by the filter: non-temporal loads (1) keep them from displacing the
// step's other working set in L2 / the L3 (filter 29 -> 21 us in the C2 step on MI355X).
#ifndef DPZ_FILTER_NT
#define DPZ_FILTER_NT 1
#endif

// ---- optional timing stamps (debug builds with -DDPZ_STAMPS only; s_memrealtime = 100 MHz) ----
#ifdef DPZ_STAMPS
__device__ unsigned long long g_stamps[64];
#define STAMP_MIN(i) do { if (threadIdx.x == 0) atomicMin(&g_stamps[i], __builtin_amdgcn_s_memrealtime()); } while (0)
#define STAMP_MAX(i) do { __syncthreads(); if (threadIdx.x == 0) atomicMax(&g_stamps[i], __builtin_amdgcn_s_memrealtime()); } while (0)
#define STAMP_ONE(i) do { if (threadIdx.x == 0) g_stamps[i] = __builtin_amdgcn_s_memrealtime(); } while (0)
// per-block phase stamps of one kernel (plain stores, no contention): g_bst[phase][block]
__device__ unsigned long long g_bst[16][4096];
#define STAMP_T0(i) do { if (threadIdx.x == 0 && blockIdx.x < 4096) g_bst[i][blockIdx.x] = __builtin_amdgcn_s_memrealtime(); } while (0)
// per-wave phase stamps of the filter: g_fst[phase][wave segment]
__device__ unsigned long long g_fst[6][8192];
#define STAMP_W(i) do { const int64_t _sg = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); if ((threadIdx.x & 63) == 0 && _sg < 8192) g_fst[i][_sg] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define STAMP_T0(i) do {} while (0)
#define STAMP_W(i) do {} while (0)
#define STAMP_MIN(i) do {} while (0)
#define STAMP_MAX(i) do {} while (0)
#define STAMP_ONE(i) do {} while (0)
#endif

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint32_t fine_bin(uint32_t key, uint32_t lo, uint32_t hi,
                                             uint32_t shift) {
  return key >= hi ? (uint32_t)HB : ((key - lo) >> shift);
}

__device__ __forceinline__ int64_t sample_pos(int c, int lane, int64_t n) {
  return ((int64_t)c * (n - SMP_CHUNK)) / (SMP_NCHUNK - 1) + lane;  // < 2^41: 64-bit is exact
}

// SMP_NCHUNK / (4 waves-per-block) blocks: 1024 chunks of 64 contiguous elements spread evenly
// over [0, n), four per wave.  nsb = the sample's own blocks (blockDim 256 or 1024: fewer,
// larger blocks fold into the global histogram with fewer same-address atomics per bin).
__device__ __forceinline__ void sampled_sample_kernel_body(KeySrc s, int64_t n, TopkCtrl* ctrl, uint32_t* chist, uint32_t* ghist, uint32_t* blcnt, ReplaceJob pj, int nsb, int val_h, const uint32_t BID) {
  if ((int)BID >= nsb) {  // co-scheduled replace decode (independent work)
    replace_block(pj, BID - nsb);
    return;
  }
  STAMP_MIN(0);
  STAMP_T0(13);
  __shared__ uint32_t h[CB];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nw = (int)(blockDim.x >> 6);
  float v[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t i = sample_pos((BID * nw + wave) * 4 + r, lane, n);
    float d = s.x0 ? (s.x[i] - s.x0[i]) : s.x[i];
    if (s.mode != DPZ_ACC_NONE) d = s.acc[i] + d;
    v[r] = d;
  }
  for (int b = threadIdx.x; b < CB; b += blockDim.x) h[b] = 0;
  // this call's window histogram copies and boundary sub-list counters start at zero
  for (int b = BID * blockDim.x + threadIdx.x; b < GH_COPIES * GH_STRIDE;
       b += nsb * blockDim.x)
    ghist[b] = 0;
  if (BID == 0) {
    if (threadIdx.x < NSUB) blcnt[threadIdx.x] = 0;
    if (threadIdx.x == 0) {
      ctrl->status = 0;
      ctrl->nbound = 0;
      ctrl->val_h = (uint32_t)val_h;
      ctrl->hinted = 0;
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 4; ++r) atomicAdd(&h[key_of(v[r]) >> CB_SHIFT], 1u);
  __syncthreads();
  for (int b = threadIdx.x; b < CB; b += blockDim.x) {
    const uint32_t c = h[b];
    if (c) atomicAdd(&chist[b], c);
  }
  STAMP_MAX(1);
  STAMP_T0(14);
}

__global__ void __launch_bounds__(1024) sampled_sample_kernel(KeySrc s, int64_t n, TopkCtrl* ctrl, uint32_t* chist, uint32_t* ghist, uint32_t* blcnt, ReplaceJob pj, int nsb, int val_h) {
  sampled_sample_kernel_body(s, n, ctrl, chist, ghist, blcnt, pj, nsb, val_h, (uint32_t)blockIdx.x);
}

// Block-level (256 threads): window [lo, hi) around the k-th key from the coarse sample histogram.
// Thread t holds the 8 bins cv = [2040-8t, 2047-8t] (ascending in memory).  Ranks r_lo / r_hi are
// 1-based, descending (window_ranks).  Result in win[0..2] after the call (barriers inside: every
// thread of the block must call it).
__device__ __forceinline__ void block_window(const uint4 (&cv)[2], uint32_t r_lo, uint32_t r_hi,
                                             uint32_t* win, uint32_t* wsum) {
  const int t = threadIdx.x;
  if (t == 0) {
    win[3] = 0xFFFFFFFFu;  // bin of rank r_lo
    win[2] = 0xFFFFFFFFu;  // bin of rank r_hi
  }
  const uint32_t hv8[8] = {cv[1].w, cv[1].z, cv[1].y, cv[1].x, cv[0].w, cv[0].z, cv[0].y, cv[0].x};
  uint32_t local = 0;
#pragma unroll
  for (int e = 0; e < 8; ++e) local += hv8[e];
  uint32_t tot;
  uint32_t before = block_excl_scan(local, wsum, &tot);  // barriers order the win[] init first
#pragma unroll
  for (int e = 0; e < 8; ++e) {  // descending: bin 2047-8t first
    const uint32_t bin = (uint32_t)(2047 - 8 * t - e);
    const uint32_t hv = hv8[e];
    if (r_lo <= (uint32_t)SMP_N && before < r_lo && r_lo <= before + hv) win[3] = bin;
    if (r_hi >= 1 && before < r_hi && r_hi <= before + hv) win[2] = bin;
    before += hv;
  }
  __syncthreads();
  if (t == 0) {
    const uint32_t blo = win[3], bhi = win[2];
    const uint32_t lo = (blo != 0xFFFFFFFFu) ? (blo << CB_SHIFT) : 0u;
    const uint64_t h64 = (bhi != 0xFFFFFFFFu) ? ((uint64_t)(bhi + 1) << CB_SHIFT) : (1ull << 31);
    const uint32_t hi = (uint32_t)(h64 > (1ull << 31) ? (1ull << 31) : h64);
    const uint32_t width = hi - lo;
    uint32_t sft = 0;
    while ((((uint64_t)width + (1ull << sft) - 1) >> sft) > (uint64_t)HB) ++sft;
    win[0] = lo;
    win[1] = hi;
    win[2] = sft;
  }
  __syncthreads();
}

// Sample ranks (1-based, descending) that bracket the k-th key with a 6-sigma + 16 margin: the
// k-th largest of n sits near rank k * SMP_N / n of the SMP_N samples (binomial sd ~ sqrt).
static inline void window_ranks(int64_t n, int64_t k, uint32_t* r_lo, uint32_t* r_hi) {
  const double r_est = (double)k * SMP_N / (double)n;
  const double sd = sqrt(r_est);
  const double rlo_d = ceil(r_est + 6.0 * sd + 16.0);
  const double rhi_d = floor(r_est - 6.0 * sd - 16.0);
  *r_lo = rlo_d > SMP_N ? (uint32_t)SMP_N + 1 : (uint32_t)rlo_d;
  // at least rank 1 (the largest sample): an open-ended window [lo, 2^31) would make each of
  // the 256 fine bins an octave wide and overflow the boundary list at small alpha (C5); keys
  // above the largest sample's coarse bin are ~n / SMP_N elements, far fewer than k there
  *r_hi = rhi_d < 1.0 ? 1u : (uint32_t)rhi_d;
}

// Per-wave candidate list append through an LDS stage, flushed in coalesced 64-lane chunks.
struct WaveList {
  uint32_t* gidx;   // this segment's global candidate list
  uint32_t* gkey;
  float* gval;      // candidate values x[idx] (nullptr: not carried, compact gathers vals_src)
  uint32_t* stg;    // this wave's LDS stage: [0, STAGE) idx, [STAGE, 2 STAGE) key, then value
                    // (one base register; the offsets fold into the ds instructions)
  uint32_t staged;  // entries in the stage (wave-uniform)
  uint32_t flushed; // entries already in the global list (wave-uniform)

  // write the stage to the global list (if `write`) and bin its keys into the window histogram
  __device__ __forceinline__ void flush(int lane, bool write, uint32_t* h, uint32_t lo, uint32_t hi,
                                        uint32_t shift) {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // this wave's LDS stage writes done
    __builtin_amdgcn_wave_barrier();
    for (uint32_t j = lane; j < staged; j += 64) {
      const uint32_t key = stg[STAGE + j];
      atomicAdd(&h[fine_bin(key, lo, hi, shift)], 1u);
      if (write) {
        gidx[flushed + j] = stg[j];
        gkey[flushed + j] = key;
        if (gval) gval[flushed + j] = __uint_as_float(stg[2 * STAGE + j]);
      }
    }
    __builtin_amdgcn_wave_barrier();
    flushed += staged;
    staged = 0;
  }
};

// A wave's G float4 groups [base, base + G*256): every load is issued before any is used, so
// G x (2 or 3) 16-byte loads per lane are in flight at once; full groups take a branch-free path.
template <bool VEC, bool ACC, int G>
__device__ __forceinline__ void load_groups(const KeySrc& s, int64_t base, int64_t end, int lane,
                                            Raw4 (&raw)[G]) {
  if (VEC && base + G * 256 <= end) {
    const bool rekey = ACC && s.mode == DPZ_ACC_ACCUMULATE && s.rekey;
#pragma unroll
    for (int q = 0; q < G; ++q) {
      const int64_t i0 = base + q * 256 + lane * 4;
      raw[q].cnt = 4;
      if (!rekey) {
#if DPZ_FILTER_NT
        typedef float v4f __attribute__((ext_vector_type(4)));
        const v4f va = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(s.x + i0));
        raw[q].a = make_float4(va.x, va.y, va.z, va.w);
        if (s.x0) {
          const v4f vb = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(s.x0 + i0));
          raw[q].b = make_float4(vb.x, vb.y, vb.z, vb.w);
        }
#else
        raw[q].a = *reinterpret_cast<const float4*>(s.x + i0);
        if (s.x0) raw[q].b = *reinterpret_cast<const float4*>(s.x0 + i0);
#endif
      }
      if (ACC && s.mode != DPZ_ACC_NONE) raw[q].q = *reinterpret_cast<const float4*>(s.acc + i0);
    }
  } else {
#pragma unroll
    for (int q = 0; q < G; ++q) {
      const int64_t i0 = base + q * 256 + lane * 4;
      raw[q].cnt = 0;
      if (i0 < end) load_raw4<VEC, ACC>(s, i0, end, raw[q]);
    }
  }
}

// B blocks x 256 threads; wave w of block b owns wave segment seg = 4b + w = [seg*R, +R) of [0, n).
template <bool VEC, bool ACC, int G>
__global__ void __launch_bounds__(256, ACC ? 4 : FOCC) sampled_filter_kernel(
    KeySrc s, int64_t n, uint32_t r_lo, uint32_t r_hi, int64_t W, int64_t R, int64_t CAP,
    TopkCtrl* ctrl, const uint32_t* __restrict__ chist, uint32_t* ghist, uint32_t* segcnt,
    uint32_t* cidx, uint32_t* ckey, float* cval, float* __restrict__ copy_out) {
  __shared__ uint32_t h[HBR];
  __shared__ uint32_t win[4];
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t st[4][3 * STAGE];
  STAMP_W(0);
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int b = threadIdx.x; b < HBR; b += 256) h[b] = 0;
  const int64_t seg = (int64_t)blockIdx.x * 4 + wid;
  const int64_t beg = seg * R;
  const int64_t end = (beg + R < n) ? beg + R : n;
  const bool store_acc = (s.mode == DPZ_ACC_ACCUMULATE) && !s.rekey;
  // The coarse sample histogram is loaded first (L2), then every wave's first G groups: loads
  // complete in issue order, so the block turns the histogram into the key window while the
  // stream loads are still in flight, and only then waits for them.
  uint4 cv[2];
  {
    const uint4* c4 = reinterpret_cast<const uint4*>(chist) + (510 - 2 * threadIdx.x);
    cv[0] = c4[0];
    cv[1] = c4[1];
  }
  Raw4 raw[G];
  load_groups<VEC, ACC, G>(s, beg, end, lane, raw);
  block_window(cv, r_lo, r_hi, win, wsum);
  STAMP_W(1);
  STAMP_W(2);
  const uint32_t lo = win[0], hi = win[1], shift = win[2];
  if (seg == 0 && lane == 0) {
    ctrl->lo = lo;
    ctrl->hi = hi;
    ctrl->shift = shift;
  }
  WaveList L{cidx + seg * CAP, ckey + seg * CAP, cval ? cval + seg * CAP : nullptr, st[wid], 0u,
             0u};
  uint32_t run = 0;
  bool dense = false;
  for (int64_t base = beg; base < end; base += G * 256) {
    if (base != beg) load_groups<VEC, ACC, G>(s, base, end, lane, raw);
#pragma unroll
    for (int q = 0; q < G; ++q) {
      uint32_t kq[4];
      const int cq = raw[q].cnt;
      if (copy_out) {  // fused replace decode over this same tensor: out = x while x streams by
        const int64_t i0 = base + q * 256 + lane * 4;
        if (VEC && cq == 4) {
          typedef float v4f __attribute__((ext_vector_type(4)));
          const v4f v = {raw[q].a.x, raw[q].a.y, raw[q].a.z, raw[q].a.w};
          __builtin_nontemporal_store(v, reinterpret_cast<v4f*>(copy_out + i0));
        } else {
          const float xv[4] = {raw[q].a.x, raw[q].a.y, raw[q].a.z, raw[q].a.w};
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (e < cq) copy_out[i0 + e] = xv[e];
        }
      }
      if (cq) finish_keys4<VEC, ACC>(s, base + q * 256 + lane * 4, store_acc, raw[q], kq);
      bool f[4];
      uint32_t pre = 0, tot = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        f[e] = e < cq && kq[e] >= lo;
        const uint64_t m = __ballot(f[e]);
        pre += mbcnt64(m);
        tot += (uint32_t)__popcll(m);
      }
      if (tot) {
        // candidates are staged in LDS and binned into the window histogram when the stage is
        // flushed (all lanes busy), not one divergent LDS atomic per element here
        if (!dense && run + tot <= (uint32_t)CAP && tot <= (uint32_t)STAGE) {
          const uint32_t i0 = (uint32_t)(base + q * 256 + lane * 4);
          if (L.staged + tot > STAGE) L.flush(lane, true, h, lo, hi, shift);
          uint32_t p = L.staged + pre;
          const float xv[4] = {raw[q].a.x, raw[q].a.y, raw[q].a.z, raw[q].a.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (f[e]) {
              L.stg[p] = i0 + e;
              L.stg[STAGE + p] = kq[e];
              L.stg[2 * STAGE + p] = __float_as_uint(xv[e]);  // x[i] (used when carried)
              ++p;
            }
          }
          L.staged += tot;
        } else {
          // segment list overflow (or one group denser than the stage): the segment turns DENSE
          // (select / compact re-read its input range); what was staged is binned, not written
          if (!dense) L.flush(lane, false, h, lo, hi, shift);
          dense = true;
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (f[e]) atomicAdd(&h[fine_bin(kq[e], lo, hi, shift)], 1u);
        }
        run += tot;
      }
    }
  }
  STAMP_W(3);
  if (!dense) L.flush(lane, true, h, lo, hi, shift);
  STAMP_W(4);
  __syncthreads();
  // fold the block's window histogram into copy b % 16 (non-returning atomics; ~B/16 arrivals
  // per address instead of B)
  uint32_t* gcopy = ghist + (blockIdx.x & (GH_COPIES - 1)) * GH_STRIDE;
  for (int b = threadIdx.x; b < HBR; b += 256) {
    const uint32_t v = h[b];
    if (v) atomicAdd(&gcopy[b], v);
  }
  if (lane == 0 && seg < W) segcnt[seg] = dense ? DENSE : run;
  STAMP_W(5);
}

// One float4 group's keys kq (valid elements e < cq, index i0 + e, values xv) into the wave's
// candidate list: keys >= lo are staged in index order (ballot + mbcnt), or counted into the
// window histogram once the segment is DENSE.
__device__ __forceinline__ void stage_group(WaveList& L, uint32_t* h, const uint32_t (&kq)[4],
                                            const float (&xv)[4], int cq, uint32_t i0, int lane,
                                            uint32_t lo, uint32_t hi, uint32_t shift, int64_t CAP,
                                            uint32_t& run, bool& dense) {
  bool f[4];
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    f[e] = e < cq && kq[e] >= lo;
    const uint64_t m = __ballot(f[e]);
    pre += mbcnt64(m);
    tot += (uint32_t)__popcll(m);
  }
  if (!tot) return;
  if (!dense && run + tot <= (uint32_t)CAP && tot <= (uint32_t)STAGE) {
    if (L.staged + tot > STAGE) L.flush(lane, true, h, lo, hi, shift);
    uint32_t p = L.staged + pre;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (f[e]) {
        L.stg[p] = i0 + e;
        L.stg[STAGE + p] = kq[e];
        L.stg[2 * STAGE + p] = __float_as_uint(xv[e]);
        ++p;
      }
    }
    L.staged += tot;
  } else {
    if (!dense) L.flush(lane, false, h, lo, hi, shift);
    dense = true;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (f[e]) atomicAdd(&h[fine_bin(kq[e], lo, hi, shift)], 1u);
  }
  run += tot;
}

// Software-pipelined filter for the PartialModel step (16-byte aligned operands, no
// accumulation; with or without the fused copy): every stream load is branch-free — lanes past
// the segment's last whole float4 read element 0 and are masked — so the compiler's wait counts
// track them, and D - 1 float4 groups (x and x0, 2 KB per wave each) stay in flight while a
// group is copied, keyed and staged: the loop is unrolled D times over D register buffers, so
// no register copy ever waits on a load.  (sampled_filter_kernel loads G groups, then waits for
// all of them — vmcnt(0) under its ragged-element branches — and has nothing in flight while it
// processes them.)  OCC waves per SIMD: the grid's W segments are all resident at once (8 at
// 8192 segments with D = 2; 4 at <= 4096 segments, where 128 registers hold deeper pipelines).
// The < 4 elements past the last whole float4 of [0, n) are handled after the loop, by the last
// segment.
// SRC: the key's operands — 0: |x|, 1: |x - x0|, 2: |acc + x| (DPZ_ACC_ADD without x0: the
// wavelet encode's W(x - x0) plus the accumulated changes, C3).
// CP: what the filter also writes as x streams by — 0 nothing, 1 copy_out = x (the fused replace
// decode), 2 copy_out = fb.of(x) (the Metro-Hastings fold's no-hit base, dpz_topk_encode_foldbase).
// Key window [lo, hi) around a prior threshold key T (DPZ_TOPK_HINT) and its fine-bin shift.
__device__ __forceinline__ void hint_window(uint32_t T, uint32_t* lo, uint32_t* hi,
                                            uint32_t* shift) {
  const float t = __uint_as_float(T);
  *lo = __float_as_uint(t * HINT_LO);
  const uint64_t h64 = (uint64_t)__float_as_uint(t * HINT_HI) + 1u;  // inf + 1 at most
  *hi = (uint32_t)(h64 > (1ull << 31) ? (1ull << 31) : h64);
  const uint32_t width = *hi - *lo;
  uint32_t sft = 0;
  while ((((uint64_t)width + (1ull << sft) - 1) >> sft) > (uint64_t)HB) ++sft;
  *shift = sft;
}

// XNT: x loaded non-temporal (true) or with the default policy (DPZ_TOPK_KEEP_X: the caller reads
// x again right after, e.g. a node's fold over its own model, which may then hit the Infinity
// Cache).  hsig != 0 (DPZ_TOPK_HINT): the window comes from the previous call's exact threshold
// (ctrl->hint_T, valid when ctrl->hint_sig == hsig) and no sample launch ran before this one —
// block 0 then does the sample launch's per-call resets (status, boundary sub-list counters; the
// window-histogram copies were left zero by the previous call's compact); an invalid prior makes
// the call miss at once (every block leaves, select and compact see the status).
template <int SRC, int CP, int D, int OCC, bool XNT>
__device__ __forceinline__ void sampled_filter_pipe_kernel_body(KeySrc s, int64_t n, uint32_t r_lo, uint32_t r_hi, int64_t W, int64_t R, int64_t CAP, TopkCtrl* ctrl, const uint32_t* __restrict__ chist, uint32_t* ghist, uint32_t* segcnt, uint32_t* cidx, uint32_t* ckey, float* cval, float* __restrict__ copy_out, FoldBase fb, uint32_t hsig, uint32_t* blcnt, int val_h, const uint32_t BID) {
  static_assert(D >= 2, "at least one group in flight");
  typedef float v4f __attribute__((ext_vector_type(4)));
  __shared__ uint32_t h[HBR];
  __shared__ uint32_t win[4];
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t st[4][3 * STAGE];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  STAMP_T0(5);
  for (int b = threadIdx.x; b < HBR; b += 256) h[b] = 0;
  const int64_t seg = (int64_t)BID * 4 + wid;
  const int64_t beg = seg * R;  // a multiple of 4 (R is); >= n for the grid's spare waves
  const int64_t end = (beg + R < n) ? beg + R : n;
  const int64_t end4 = beg < end ? beg + ((end - beg) & ~int64_t(3)) : beg;
  const v4f* __restrict__ xa = reinterpret_cast<const v4f*>(s.x);
  constexpr bool X0 = SRC != 0;  // a second operand stream (x0 or acc) in the B buffers
  const v4f* __restrict__ xb = reinterpret_cast<const v4f*>(SRC == 2 ? s.acc : s.x0);
  v4f A[D], B[D];
  // group j of the segment (256 elements) into buffer slot u
  auto ld = [&](int64_t j, int u) {
    const int64_t i0 = beg + j * 256 + lane * 4;
    const int64_t g4 = (i0 < end4 ? i0 : 0) >> 2;
    // x non-temporal, like x0 / acc: a runtime choice between a non-temporal and a plain load
    // (an xnt kernel argument, tried in round 4) compiled to ONE plain load — the hint was lost,
    // x stayed in the caches and the compact's counter updates slowed by 1-3 us (same-box A/B
    // against the round-3 build, tools/diag/enc_ab.py)
    if (XNT) A[u] = __builtin_nontemporal_load(xa + g4);
    else A[u] = xa[g4];
    if (X0) B[u] = __builtin_nontemporal_load(xb + g4);
  };
  // the window's inputs are loaded first, the first stream loads right after them, and only
  // then is anything waited on (a check of the prior before the stream loads would hold every
  // wave's first load behind its round trip)
  uint4 cv[2] = {};
  uint32_t hT = 0, hS = 0;
  if (hsig) {
    hT = ctrl->hint_T;
    hS = ctrl->hint_sig;
  } else {
    const uint4* c4 = reinterpret_cast<const uint4*>(chist) + (510 - 2 * threadIdx.x);
    cv[0] = c4[0];
    cv[1] = c4[1];
  }
#pragma unroll
  for (int u = 0; u < D - 1; ++u) ld(u, u);
  if (hsig) {
    const bool ok = hS == hsig && hT > 0u && hT < 0x7F800000u;
    if (!ok) {  // no usable prior window: the call misses (uniform over the grid)
      if (BID == 0 && threadIdx.x == 0) {
        ctrl->status = 1;
        ctrl->hinted = 1;
        ctrl->val_h = (uint32_t)val_h;
      }
      // the copy this launch owes (CP 1: the fused replace's out = x, whose payload entries the
      // compact launch still scatters; CP 2: the fold's no-hit base) is written all the same:
      // the re-run after the miss (dpz_topk_complete) encodes only, it has no copy slot
      if (CP != 0) {
        const int64_t ngc = (end4 - beg + 255) >> 8;
        for (int64_t j = 0; j < ngc; ++j) {
          const int64_t i0 = beg + j * 256 + lane * 4;
          if (i0 < end4) {
            const v4f a = xa[i0 >> 2];
            const v4f b = CP == 1 ? a : v4f{fb.of(a.x), fb.of(a.y), fb.of(a.z), fb.of(a.w)};
            __builtin_nontemporal_store(b, reinterpret_cast<v4f*>(copy_out) + (i0 >> 2));
          }
        }
        if (end4 < end && end4 + lane < end) {
          const float xv = s.x[end4 + lane];
          copy_out[end4 + lane] = CP == 1 ? xv : fb.of(xv);
        }
      }
      return;
    }
    if (BID == 0) {
      if (threadIdx.x < NSUB) blcnt[threadIdx.x] = 0;
      if (threadIdx.x == 0) {
        ctrl->status = 0;
        ctrl->nbound = 0;
        ctrl->val_h = (uint32_t)val_h;
        ctrl->hinted = 1;
      }
    }
  }
  uint32_t lo, hi, shift;
  if (hsig) {
    hint_window(hT, &lo, &hi, &shift);
  } else {
    block_window(cv, r_lo, r_hi, win, wsum);
    lo = win[0];
    hi = win[1];
    shift = win[2];
  }
  STAMP_T0(6);
  if (seg == 0 && lane == 0) {
    ctrl->lo = lo;
    ctrl->hi = hi;
    ctrl->shift = shift;
  }
  WaveList L{cidx + seg * CAP, ckey + seg * CAP, cval ? cval + seg * CAP : nullptr, st[wid], 0u,
             0u};
  uint32_t run = 0;
  bool dense = false;
  auto proc = [&](int64_t j, int u) {
    const int64_t i0 = beg + j * 256 + lane * 4;
    const int cq = i0 < end4 ? 4 : 0;
    if (CP == 1 && cq) __builtin_nontemporal_store(A[u], reinterpret_cast<v4f*>(copy_out) + (i0 >> 2));
    if (CP == 2 && cq) {
      const v4f b = {fb.of(A[u].x), fb.of(A[u].y), fb.of(A[u].z), fb.of(A[u].w)};
      __builtin_nontemporal_store(b, reinterpret_cast<v4f*>(copy_out) + (i0 >> 2));
    }
    const float xv[4] = {A[u].x, A[u].y, A[u].z, A[u].w};
    uint32_t kq[4];
    if (SRC == 1) {
      const float bv[4] = {B[u].x, B[u].y, B[u].z, B[u].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) kq[e] = key_of(xv[e] - bv[e]);
    } else if (SRC == 2) {
      const float bv[4] = {B[u].x, B[u].y, B[u].z, B[u].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) kq[e] = key_of(bv[e] + xv[e]);  // acc + change
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) kq[e] = key_of(xv[e]);
    }
    stage_group(L, h, kq, xv, cq, (uint32_t)i0, lane, lo, hi, shift, CAP, run, dense);
  };
  const int64_t ng = (end4 - beg + 255) >> 8;  // groups holding whole float4s
  for (int64_t j0 = 0; j0 < ng; j0 += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      ld(j0 + u + D - 1, (u + D - 1) % D);  // the group D - 1 ahead, into the slot just freed
      proc(j0 + u, u);
    }
  }
  if (end4 < end) {  // the last segment's ragged 1-3 elements
    const int64_t i = end4 + lane;
    const bool v = i < end;
    float xv[4] = {0.f, 0.f, 0.f, 0.f};
    uint32_t kq[4] = {0u, 0u, 0u, 0u};
    if (v) {
      xv[0] = s.x[i];
      kq[0] = key_of(SRC == 1 ? xv[0] - s.x0[i] : (SRC == 2 ? s.acc[i] + xv[0] : xv[0]));
      if (CP == 1) copy_out[i] = xv[0];
      if (CP == 2) copy_out[i] = fb.of(xv[0]);
    }
    // one element per lane: lane order is index order
    stage_group(L, h, kq, xv, v ? 1 : 0, (uint32_t)i, lane, lo, hi, shift, CAP, run, dense);
  }
  if (!dense) L.flush(lane, true, h, lo, hi, shift);
  __syncthreads();
  uint32_t* gcopy = ghist + (BID & (GH_COPIES - 1)) * GH_STRIDE;
  for (int b = threadIdx.x; b < HBR; b += 256) {
    const uint32_t v = h[b];
    if (v) atomicAdd(&gcopy[b], v);
  }
  if (lane == 0 && seg < W) segcnt[seg] = dense ? DENSE : run;
  STAMP_T0(7);
}

template <int SRC, int CP, int D, int OCC, bool XNT>
__global__ void __launch_bounds__(256, OCC) sampled_filter_pipe_kernel(KeySrc s, int64_t n, uint32_t r_lo, uint32_t r_hi, int64_t W, int64_t R, int64_t CAP, TopkCtrl* ctrl, const uint32_t* __restrict__ chist, uint32_t* ghist, uint32_t* segcnt, uint32_t* cidx, uint32_t* ckey, float* cval, float* __restrict__ copy_out, FoldBase fb, uint32_t hsig, uint32_t* blcnt, int val_h) {
  sampled_filter_pipe_kernel_body<SRC, CP, D, OCC, XNT>(s, n, r_lo, r_hi, W, R, CAP, ctrl, chist, ghist, segcnt, cidx, ckey, cval, copy_out, fb, hsig, blcnt, val_h, (uint32_t)blockIdx.x);
}

// Wave-level threshold bin from the global window histogram gh (LDS, HB fine bins + the
// above-window count `above`): lane l holds the HB/64 bins [HB - HB/64 (l + 1), HB - HB/64 l).
__device__ __forceinline__ bool wave_bstar(const uint32_t* gh, uint32_t above, uint32_t k,
                                           uint32_t* bstar, uint32_t* need) {
  constexpr int PL = HB / 64;
  const int lane = threadIdx.x & 63;
  uint32_t hv[PL];  // descending: hv[e] = bin HB - 1 - PL*lane - e
  const uint4* g4 = reinterpret_cast<const uint4*>(gh) + (HB / 4 - (PL / 4) * (lane + 1));
#pragma unroll
  for (int q = 0; q < PL / 4; ++q) {
    const uint4 v = g4[PL / 4 - 1 - q];
    hv[4 * q + 0] = v.w;
    hv[4 * q + 1] = v.z;
    hv[4 * q + 2] = v.y;
    hv[4 * q + 3] = v.x;
  }
  uint32_t local = 0;
#pragma unroll
  for (int e = 0; e < PL; ++e) local += hv[e];
  uint32_t tot;
  uint32_t before = wave_excl_scan(local, &tot) + above;
  uint32_t fb = 0xFFFFFFFFu, fn = 0;
#pragma unroll
  for (int e = 0; e < PL; ++e) {
    if (before < k && k <= before + hv[e]) {
      fb = (uint32_t)(HB - 1 - PL * lane - e);
      fn = k - before;
    }
    before += hv[e];
  }
  const uint64_t m = __ballot(fb != 0xFFFFFFFFu);
  const bool ok = (above < k) && (above + tot >= k) && m != 0;
  const int src = m ? (int)__ffsll((long long)m) - 1 : 0;
  *bstar = __shfl(fb, src, 64);
  *need = __shfl(fn, src, 64);
  return ok;
}

// ceil(W/32) blocks x 1024 (16 waves x 2 wave segments).  Sums the 16 window-histogram copies,
// finds the threshold bin b* (wave 0), counts each filter block's candidates above b*
// (blkabove) and appends the bin-b* entries, staged in LDS, to sub-list (block % 16) with one
// atomic per block.
template <bool VEC>
__device__ __forceinline__ void sampled_select_kernel_body(KeySrc s, int64_t n, int64_t k, int64_t W, int64_t B, int64_t R, int64_t CAP, TopkCtrl* ctrl, const uint32_t* __restrict__ ghist, const uint32_t* __restrict__ segcnt, const uint32_t* __restrict__ cidx, const uint32_t* __restrict__ ckey, uint32_t* blkabove, uint32_t* blcnt, uint32_t* blkey, uint32_t* blidx, ReplaceJob pj, const uint32_t BID) {
  {
    const int64_t own = (W + SEL_SEGS - 1) / SEL_SEGS;
    if ((int64_t)BID >= own) {  // co-scheduled replace decode
      replace_block(pj, (int64_t)BID - own);
      return;
    }
  }
  STAMP_MIN(6);
  STAMP_T0(8);
  __shared__ __attribute__((aligned(16))) uint32_t gh[GH_STRIDE];
  __shared__ uint32_t fbabove[SEL_SEGS / 4];
  __shared__ uint32_t lkey[SEL_LCAP], lidx[SEL_LCAP];
  __shared__ uint32_t lcnt, gbase, sb_bstar, sb_need, sb_ok;
  const int t = threadIdx.x, wid = t >> 6, lane = t & 63;
  const int64_t seg0 = (int64_t)BID * SEL_SEGS + wid * 2;
  const uint32_t cnt0 = seg0 < W ? segcnt[seg0] : 0u;
  const uint32_t cnt1 = seg0 + 1 < W ? segcnt[seg0 + 1] : 0u;
  // the first 64 entries of both lists are loaded with the counts and the histogram, not after
  // b* is known (CAP >= 64; entries past the count are ignored)
  constexpr int PFS = 4;  // chunks of 64 per segment held in registers
  uint32_t pk[2][PFS], pi[2][PFS];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int64_t sg = seg0 + u;
    pk[u][0] = sg < W ? ckey[sg * CAP + lane] : 0u;
    pi[u][0] = sg < W ? cidx[sg * CAP + lane] : 0u;
  }
  const uint32_t lo = ctrl->lo, hi = ctrl->hi, shift = ctrl->shift;
  // a hinted filter without a usable prior window reported a miss (checked once the first loads
  // are issued: nothing to select)
  const uint32_t fstatus = ctrl->status;
  // histogram copies (bins t and, for t == 0, the above-window bin HB), then chunks 1 .. PFS-1
  // of segments with more than 64 candidates — all loads issued before any sum is formed
  static_assert(HB == 1024, "select: one fine bin per thread + the above-window bin");
  uint32_t v[GH_COPIES], va[GH_COPIES];
#pragma unroll
  for (int c = 0; c < GH_COPIES; ++c) {
    v[c] = ghist[c * GH_STRIDE + t];
    va[c] = t == 0 ? ghist[c * GH_STRIDE + HB] : 0u;
  }
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int64_t sg = seg0 + u;
    const uint32_t cu = u ? cnt1 : cnt0;
#pragma unroll
    for (int c = 1; c < PFS; ++c) {
      const uint32_t j = c * 64u + lane;
      pk[u][c] = 0u;
      pi[u][c] = 0u;
      if (sg < W && cu != DENSE && j < cu) {
        pk[u][c] = ckey[sg * CAP + j];
        pi[u][c] = cidx[sg * CAP + j];
      }
    }
  }
  if (fstatus) return;  // uniform over the grid
  {
    uint32_t sum = 0, suma = 0;
#pragma unroll
    for (int c = 0; c < GH_COPIES; ++c) {
      sum += v[c];
      suma += va[c];
    }
    gh[t] = sum;
    if (t == 0) gh[HB] = suma;
  }
  STAMP_T0(12);
  if (t < SEL_SEGS / 4) fbabove[t] = 0;
  if (t == 0) lcnt = 0;
  __syncthreads();
  if (wid == 0) {
    uint32_t bstar, need;
    const bool ok = wave_bstar(gh, gh[HB], (uint32_t)k, &bstar, &need);
    if (lane == 0) {
      sb_bstar = bstar;
      sb_need = need;
      sb_ok = ok ? 1u : 0u;
    }
  }
  __syncthreads();
  if (!sb_ok) {  // identical in every block: the whole grid leaves
    if (BID == 0 && t == 0) ctrl->status = 1;
    return;
  }
  STAMP_T0(9);
  const uint32_t bstar = sb_bstar;
  if (BID == 0 && t == 0) {
    ctrl->bstar = bstar;
    ctrl->need = sb_need;
  }
  auto append = [&](bool in, uint32_t key, uint32_t idx) {
    const uint64_t m = __ballot(in);
    if (m) {
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(&lcnt, (uint32_t)__popcll(m));
      base = __shfl(base, 0, 64);
      if (in) {
        const uint32_t p = base + mbcnt64(m);
        if (p < SEL_LCAP) {
          lkey[p] = key;
          lidx[p] = idx;
        }
      }
    }
  };
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int64_t seg = seg0 + u;
    const uint32_t cnt = u ? cnt1 : cnt0;
    uint32_t above = 0;
    if (seg < W && cnt != DENSE) {
#pragma unroll
      for (int c = 0; c < PFS; ++c) {  // the chunks held in registers
        const uint32_t j = c * 64u + lane;
        if (c * 64u >= cnt) break;
        const uint32_t key = pk[u][c], idx = pi[u][c];
        const uint32_t b = j < cnt ? fine_bin(key, lo, hi, shift) : 0u;
        above += (uint32_t)__popcll(__ballot(j < cnt && b > bstar));
        append(j < cnt && b == bstar, key, idx);
      }
      // dense alpha: the chunks past them four at a time, every key load in flight together
      // (one chunk per iteration was one dependent round trip each); the index only for the
      // rare bin-b* entries
      for (uint32_t j0 = PFS * 64u; j0 < cnt; j0 += 4 * 64u) {
        uint32_t kg[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const uint32_t j = j0 + g * 64u + lane;
          kg[g] = ckey[seg * CAP + (j < cnt ? j : 0u)];
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const uint32_t j = j0 + g * 64u + lane;
          const bool v = j < cnt;
          const uint32_t b = v ? fine_bin(kg[g], lo, hi, shift) : 0u;
          above += (uint32_t)__popcll(__ballot(v && b > bstar));
          const bool ap = v && b == bstar;
          const uint32_t idx = ap ? cidx[seg * CAP + j] : 0u;
          append(ap, kg[g], idx);
        }
      }
    } else if (seg < W) {
      const int64_t beg = seg * R;
      const int64_t end = (beg + R < n) ? beg + R : n;
      for (int64_t i0 = beg + lane * 4; i0 - lane * 4 < end; i0 += 256) {
        uint32_t key[4];
        const int c = i0 < end ? load_keys4<VEC>(s, i0, end, false, key) : 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool valid = e < c && key[e] >= lo;
          const uint32_t b = valid ? fine_bin(key[e], lo, hi, shift) : 0u;
          above += (uint32_t)__popcll(__ballot(valid && b > bstar));
          append(valid && b == bstar, key[e], (uint32_t)(i0 + e));
        }
      }
    }
    if (lane == 0 && above) atomicAdd(&fbabove[(wid * 2 + u) >> 2], above);
  }
  __syncthreads();
  if (t < SEL_SEGS / 4) {
    const int64_t fb = (int64_t)BID * (SEL_SEGS / 4) + t;
    blkabove[fb] = fb < B ? fbabove[t] : 0u;  // zero-padded to a multiple of 8 (compact)
  }
  STAMP_T0(10);
  const uint32_t nl = lcnt;
  if (nl) {
    const int sub = (int)(BID & (NSUB - 1));
    if (t == 0) gbase = atomicAdd(&blcnt[sub], nl > SEL_LCAP ? (uint32_t)BCAP : nl);
    __syncthreads();
    const uint32_t gb = gbase;
    for (uint32_t j = t; j < nl && j < SEL_LCAP; j += 1024) {
      const uint32_t p = gb + j;
      if (p < SUBCAP) {
        blkey[sub * SUBCAP + p] = lkey[j];
        blidx[sub * SUBCAP + p] = lidx[j];
      }
    }
  }
  STAMP_T0(11);
}

template <bool VEC>
__global__ void __launch_bounds__(1024) sampled_select_kernel(KeySrc s, int64_t n, int64_t k, int64_t W, int64_t B, int64_t R, int64_t CAP, TopkCtrl* ctrl, const uint32_t* __restrict__ ghist, const uint32_t* __restrict__ segcnt, const uint32_t* __restrict__ cidx, const uint32_t* __restrict__ ckey, uint32_t* blkabove, uint32_t* blcnt, uint32_t* blkey, uint32_t* blidx, ReplaceJob pj) {
  sampled_select_kernel_body<VEC>(s, n, k, W, B, R, CAP, ctrl, ghist, segcnt, cidx, ckey, blkabove, blcnt, blkey, blidx, pj, (uint32_t)blockIdx.x);
}

// Boundary entry j (0 <= j < nb) of the 16 sub-lists: sub-list sb with subbase[sb] <= j.
__device__ __forceinline__ uint32_t bound_slot(const uint32_t* subbase, uint32_t j) {
  int sb = 0;
#pragma unroll
  for (int u = 1; u < NSUB; ++u) sb += subbase[u] <= j ? 1 : 0;
  return (uint32_t)sb * SUBCAP + (j - subbase[sb]);
}

// 256-thread block: the exact threshold key T and tie cut icut inside bin b* from the boundary
// sub-lists — the pivot is the need-th entry of bin b* in (key descending, index ascending)
// order; an entry of bin b* is selected iff it is not after the pivot (key > T, or key == T and
// idx <= icut).  One 8-bit digit pass over the offsets inside bin b* (~k/256 entries) leaves a
// handful in the pivot's digit; if at most 64, one wave ranks them against each other (register
// broadcasts) and the entry of rank rem - 1 is the pivot (ties cost nothing extra).  Otherwise
// (heavy ties, wide bins) radix select of T over the remaining digits, then of the tie cut on the
// index.  The first BLDS entries are staged in LDS, the rest are re-read (L2).
constexpr int BLDS = 1024;
struct Bound {
  const uint32_t* key;
  const uint32_t* idx;
  const uint32_t* subbase;  // LDS
  uint32_t* sk;             // LDS [BLDS]
  uint32_t* si;             // LDS [BLDS]
  uint32_t nb;
  __device__ __forceinline__ void load() {
    uint32_t kk[BLDS / 256], ii[BLDS / 256];
#pragma unroll
    for (int q = 0; q < BLDS / 256; ++q) {
      const uint32_t j = threadIdx.x + q * 256u;
      if (j < nb) {
        const uint32_t sl = bound_slot(subbase, j);
        kk[q] = key[sl];
        ii[q] = idx[sl];
      }
    }
#pragma unroll
    for (int q = 0; q < BLDS / 256; ++q) {
      const uint32_t j = threadIdx.x + q * 256u;
      if (j < nb) {
        sk[j] = kk[q];
        si[j] = ii[q];
      }
    }
    __syncthreads();
  }
  // f(key, idx) for every entry of this thread
  template <class F>
  __device__ __forceinline__ void each(F f) const {
    const uint32_t m = nb < (uint32_t)BLDS ? nb : (uint32_t)BLDS;
    for (uint32_t j = threadIdx.x; j < m; j += 256u) f(sk[j], si[j]);
    for (uint32_t j = threadIdx.x + BLDS; j < nb; j += 256u) {
      const uint32_t sl = bound_slot(subbase, j);
      f(key[sl], idx[sl]);
    }
  }
};

struct ResolveLds {
  uint32_t hist[256];
  uint32_t wsum[16];
  uint32_t sh[4];
  uint2 ent[64];
  uint32_t bcnt;
};

__device__ __forceinline__ void block_resolve(const Bound& bd, uint32_t need, uint32_t base,
                                              uint32_t shift, ResolveLds& L, uint32_t* T_out,
                                              uint32_t* icut_out) {
  const int t = threadIdx.x;
  // (A rank of every entry against all the others — O(nb^2) compares per thread, no digit
  // passes — measured 4-7 us per block instead of ~1.7: every one of the ~1024 blocks repeats
  // the resolve, so its VALU work is paid ~4 times on every SIMD.)
  const int d1 = shift >= 8 ? 8 : (int)shift;
  const int low1 = (int)shift - d1;
  const uint32_t m1 = (1u << d1) - 1u;
  L.hist[t] = 0;
  if (t == 0) L.bcnt = 0;
  __syncthreads();
  bd.each([&](uint32_t kv, uint32_t) { atomicAdd(&L.hist[((kv - base) >> low1) & m1], 1u); });
  __syncthreads();
  {
    const uint32_t hb = L.hist[255 - t];  // descending digit 255 - t
    uint32_t tot;
    const uint32_t before = block_excl_scan(hb, L.wsum, &tot);
    if (before < need && need <= before + hb) {
      L.sh[0] = 255 - t;
      L.sh[1] = need - before;
      L.sh[2] = hb;
    }
    __syncthreads();
  }
  const uint32_t dstar = L.sh[0], rem1 = L.sh[1], eq1 = L.sh[2];
  __syncthreads();
  if (eq1 <= 64) {
    bd.each([&](uint32_t kv, uint32_t iv) {
      if ((((kv - base) >> low1) & m1) == dstar) L.ent[atomicAdd(&L.bcnt, 1u)] = make_uint2(kv, iv);
    });
    __syncthreads();
    if (t < 64) {
      const uint2 me = t < (int)eq1 ? L.ent[t] : make_uint2(0u, 0xFFFFFFFFu);
      uint32_t rank = 0;
      for (uint32_t f = 0; f < eq1; ++f) {
        const uint32_t ok = __builtin_amdgcn_readlane(me.x, f);
        const uint32_t oi = __builtin_amdgcn_readlane(me.y, f);
        rank += (ok > me.x || (ok == me.x && oi < me.y)) ? 1u : 0u;
      }
      if (t < (int)eq1 && rank == rem1 - 1) {
        L.sh[0] = me.x;
        L.sh[1] = me.y;
      }
    }
    __syncthreads();
    *T_out = L.sh[0];
    *icut_out = L.sh[1];
    __syncthreads();
    return;
  }
  uint32_t prefix = 0, rem = need, eqcnt = bd.nb;
  for (int top = (int)shift; top > 0; top -= 8) {
    const int d = top >= 8 ? 8 : top;
    const int low = top - d;
    L.hist[t] = 0;
    __syncthreads();
    bd.each([&](uint32_t kv, uint32_t) {
      const uint32_t o = kv - base;
      if ((uint32_t)((uint64_t)o >> top) == (uint32_t)((uint64_t)prefix >> top))
        atomicAdd(&L.hist[(o >> low) & ((1u << d) - 1)], 1u);
    });
    __syncthreads();
    const uint32_t hb = L.hist[255 - t];
    uint32_t tot;
    const uint32_t before = block_excl_scan(hb, L.wsum, &tot);
    if (before < rem && rem <= before + hb) {
      L.sh[0] = 255 - t;
      L.sh[1] = rem - before;
      L.sh[2] = hb;
    }
    __syncthreads();
    prefix |= L.sh[0] << low;
    rem = L.sh[1];
    eqcnt = L.sh[2];
    __syncthreads();
  }
  const uint32_t T = base + prefix;
  uint32_t icut = 0xFFFFFFFFu;
  if (rem < eqcnt) {
    uint32_t ipre = 0, irem = rem;
    for (int top = 32; top > 0; top -= 8) {
      const int low = top - 8;
      L.hist[t] = 0;
      __syncthreads();
      bd.each([&](uint32_t kv, uint32_t iv) {
        if (kv == T && (top == 32 || (iv >> top) == (ipre >> top)))
          atomicAdd(&L.hist[(iv >> low) & 255u], 1u);
      });
      __syncthreads();
      const uint32_t hb = L.hist[t];  // ascending digit t
      uint32_t tot;
      const uint32_t before = block_excl_scan(hb, L.wsum, &tot);
      if (before < irem && irem <= before + hb) {
        L.sh[0] = t;
        L.sh[1] = irem - before;
      }
      __syncthreads();
      ipre |= L.sh[0] << low;
      irem = L.sh[1];
      __syncthreads();
    }
    icut = ipre;
  }
  *T_out = T;
  *icut_out = icut;
}

// Sum over the block of a pair of counters (each < 2^32), packed in 64 bits.
__device__ __forceinline__ uint64_t block_sum64(uint64_t v, uint64_t* wsum64) {
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  if (lane == 0) wsum64[wid] = v;
  __syncthreads();
  uint64_t tot = 0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) tot += wsum64[w];
  __syncthreads();
  return tot;
}

// DENSE segments (candidate list overflowed in the filter) re-read their input range: rare, kept
// out of line so the common path's register budget is not sized for it.
template <bool VEC>
__device__ __forceinline__ uint32_t dense_count(const KeySrc s, int64_t seg, int64_t R,
                                                          int64_t n, uint32_t lo, uint32_t T,
                                                          uint32_t icut) {
  const int lane = threadIdx.x & 63;
  const int64_t beg = seg * R;
  const int64_t end = (beg + R < n) ? beg + R : n;
  uint32_t mine = 0;
  for (int64_t i0 = beg + lane * 4; i0 - lane * 4 < end; i0 += 256) {
    uint32_t key[4];
    const int c = i0 < end ? load_keys4<VEC>(s, i0, end, false, key) : 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const bool f = e < c && key[e] >= lo &&
                     (key[e] > T || (key[e] == T && (uint32_t)(i0 + e) <= icut));
      mine += (uint32_t)__popcll(__ballot(f));
    }
  }
  return mine;
}

template <bool VEC>
__device__ __forceinline__ void dense_write(const KeySrc s, int64_t seg, int64_t R,
                                                      int64_t n, int64_t k, uint32_t lo,
                                                      uint32_t T, uint32_t icut, uint32_t run,
                                                      const float* vals_src, int32_t* idx_out,
                                                      float* val_out, int32_t* counter,
                                                      float* rewind, int val_h,
                                                      uint32_t* slrow) {
  const int lane = threadIdx.x & 63;
  const int64_t beg = seg * R;
  const int64_t end = (beg + R < n) ? beg + R : n;
  for (int64_t i0 = beg + lane * 4; i0 - lane * 4 < end; i0 += 256) {
    uint32_t key[4];
    const int c = i0 < end ? load_keys4<VEC>(s, i0, end, false, key) : 0;
    bool f[4];
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      f[e] = e < c && key[e] >= lo &&
             (key[e] > T || (key[e] == T && (uint32_t)(i0 + e) <= icut));
      const uint64_t m = __ballot(f[e]);
      pre += mbcnt64(m);
      tot += (uint32_t)__popcll(m);
    }
    uint32_t pos = run + pre;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (f[e]) {
        if (pos < (uint64_t)k) {
          const int64_t i = i0 + e;
          idx_out[pos] = (int32_t)i;
          store_val(val_out, val_h, pos, vals_src[i]);
          if (slrow) atomicOr(&slrow[(i - beg) >> 5], 1u << (i & 31));
          if (counter) atomicAdd(&counter[i], 1);
          if (rewind) rewind[i] = 0.0f;
        }
        ++pos;
      }
    }
    run += tot;
  }
}

// One block of 256 threads per CSEG = 4 SPW wave segments (SPW / 4 filter blocks... SPW per
// wave).  Prologue, redundantly in every block (no single-block launch in between — a launch
// boundary plus a one-CU kernel cost more than the ~15 KB of L2 reads per block): the exact T /
// icut from the boundary sub-lists, the block's output offset = above-b* counts of the earlier
// filter blocks + selected boundary entries before the block, and the check that the grand total
// is k.  Then per wave a count pass over its SPW segments, in-block offsets, and the ordered
// write of (idx, vals_src[idx]) with counter / rewind updates.  Block 0 re-zeroes the sample
// histogram and publishes T / icut / status.
// SPW = 8 (sparse alpha: ~20 candidates per segment): 256 blocks at 8192 segments, ONE per CU,
// so the redundant prologue (latency-bound LDS phases with barriers) is not shared four ways on
// every SIMD; every segment's first 64 candidates are loaded with the prologue.  SPW = 2 (dense
// alpha): four chunks of 64 per segment in registers, 4 blocks per CU.
// PLAIN (dense alpha, k > n/32): counter[idx] += 1 as a gathered read + plain store instead of a
// memory-side atomic.  The selected indices are unique, so no two lanes update one word; a wave
// instruction of atomics whose 64 lanes hit ~40 different lines runs at ~1/13 of the streaming
// rate (MI355X_MICROARCH.md, Global float atomics: "64 lanes in 64 different rows"), which made
// the C3 compact (k = 2.5 M) atomic-bound; scattered plain stores run at the streaming rate, and
// the gathers are issued while the threshold is being resolved.  At sparse alpha the atomics stay
// (reading every candidate's counter ahead measured slower at C2).
template <int SPW>
struct CompactCfg {
  static constexpr int CSEG = 4 * SPW;          // wave segments per block
  static constexpr int PFC = SPW >= 8 ? 1 : 4;  // chunks of 64 per segment held in registers
};

#ifndef DPZ_SL_PF  // planes read ahead per ripple-carry step (a divisor of 32)
#define DPZ_SL_PF 4
#endif
constexpr int SL_PF = DPZ_SL_PF;
static_assert(32 % SL_PF == 0, "the planes are read in whole steps");

// SL (dpz_topk_encode_sliced): no scattered counter / rewind; each wave ORs its segment's
// selected bits into an LDS row (R <= SL_RMAX, R a multiple of 32: the segment owns whole
// words), then writes every word of the row to selmask and adds it to the bit-sliced counter
// (planes[p * nwords + w], carry-propagated plane by plane) with coalesced accesses.
template <bool VEC, bool PLAIN, int SPW, bool SL>
__device__ __forceinline__ void sampled_compact_kernel_body(KeySrc s, int64_t n, int64_t k, int64_t W, int64_t R, int64_t CAP, TopkCtrl* ctrl, uint32_t* chist, const uint32_t* __restrict__ blkabove, const uint32_t* __restrict__ blcnt, const uint32_t* __restrict__ blkey, const uint32_t* __restrict__ blidx, const uint32_t* __restrict__ segcnt, const uint32_t* __restrict__ cidx, const uint32_t* __restrict__ ckey, const float* __restrict__ cval, const float* vals_src, int32_t* idx_out, float* val_out, int32_t* counter, float* rewind, int32_t* status_out, ReplaceJob pj, int64_t nrep_first, int val_h, uint32_t* selmask, uint32_t* planes, int64_t nwords, uint32_t* ghist, uint32_t sig, const uint32_t BID) {
  constexpr int CSEG = CompactCfg<SPW>::CSEG;
  constexpr int PFC = CompactCfg<SPW>::PFC;
  constexpr int SLW = SL ? (int)(SL_RMAX / 32) : 1;
  __shared__ uint32_t slrows[SL ? 4 : 1][SLW];
  __shared__ uint32_t wcnt[CSEG];
  __shared__ uint32_t subbase[NSUB + 1];
  __shared__ uint32_t flag, spec;
  __shared__ uint64_t wsum64[4];
  __shared__ ResolveLds RL;
  __shared__ __attribute__((aligned(16))) uint32_t bsk[BLDS];
  __shared__ __attribute__((aligned(16))) uint32_t bsi[BLDS];
  const int64_t CB_ = (W + CSEG - 1) / CSEG;
  const int64_t B = (W + 3) / 4;  // filter blocks (above counts)
  // co-scheduled replace decode: its blocks after compact's own, or (nrep_first > 0) before
  // them, dispatched first so their stores overlap the compact blocks' dependent prologue
  if (nrep_first > 0 ? (int64_t)BID < nrep_first : (int64_t)BID >= CB_) {
    replace_block(pj, nrep_first > 0 ? (int64_t)BID : (int64_t)BID - CB_);
    return;
  }
  const uint32_t blk = (uint32_t)((int64_t)BID - (nrep_first > 0 ? nrep_first : 0));
  STAMP_T0(0);
  const int t = threadIdx.x, wid = t >> 6, lane = t & 63;
  // select has read the window-histogram copies: leave them zero for the next call (a call with
  // a prior-round window has no sample launch to zero them, DPZ_TOPK_HINT)
  for (int64_t b = (int64_t)blk * 256 + t; b < (int64_t)GH_COPIES * GH_STRIDE; b += CB_ * 256)
    ghist[b] = 0u;
  const int64_t seg0 = (int64_t)blk * CSEG + wid * SPW;
  // every independent load first: control words, sub-list counts, above counts, own candidates
  const uint32_t status = ctrl->status;
  const uint32_t need = ctrl->need, lo = ctrl->lo, shift = ctrl->shift, bstar = ctrl->bstar;
  const uint32_t sc = t < NSUB ? blcnt[t] : 0u;
  // the first SPEC entries of every boundary sub-list, loaded with the counts (thread t: sub-list
  // t / SPEC, slot t % SPEC) instead of after them: when no sub-list holds more (the usual case,
  // ~k/1000 boundary entries over 16 sub-lists), the boundary set needs no dependent load
  constexpr uint32_t SPEC = 256 / NSUB;
  static_assert(NSUB * SPEC == 256 && SPEC <= SUBCAP, "one speculative entry per thread");
  const uint32_t sp_sub = (uint32_t)t / SPEC, sp_slot = (uint32_t)t % SPEC;
  const uint32_t spk = blkey[sp_sub * SUBCAP + sp_slot], spi = blidx[sp_sub * SUBCAP + sp_slot];
  static_assert(B_MAX <= 256 * 8, "above counts: 8 per thread");
  uint32_t abv_before = 0, abv_all = 0;
  {
    // blkabove holds B entries, zero-padded to a multiple of 8 by select (ws is 256-B aligned)
    const uint32_t fb0 = (uint32_t)t * 8u;
    uint4 v0 = make_uint4(0, 0, 0, 0), v1 = make_uint4(0, 0, 0, 0);
    if ((int64_t)fb0 < B) {
      v0 = reinterpret_cast<const uint4*>(blkabove)[2 * t];
      v1 = reinterpret_cast<const uint4*>(blkabove)[2 * t + 1];
    }
    const uint32_t v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    const uint32_t fbx = blk * (uint32_t)(CSEG / 4);  // first filter block of this block
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      abv_all += v[q];
      abv_before += fb0 + q < fbx ? v[q] : 0u;
    }
  }
  // candidate chunks of 64 kept in registers per segment (PFC chunks); chunk 0 is loaded without
  // waiting for the count (CAP >= 64; entries past it are ignored)
  uint32_t cnt[SPW], kk[SPW][PFC], ii[SPW][PFC];
  float vv[SPW][PFC];
#pragma unroll
  for (int u = 0; u < SPW; ++u) {
    const int64_t seg = seg0 + u;
    cnt[u] = seg < W ? segcnt[seg] : 0u;
#pragma unroll
    for (int c = 0; c < PFC; ++c) {
      kk[u][c] = 0u;
      ii[u][c] = 0u;
      vv[u][c] = 0.f;
    }
    kk[u][0] = seg < W ? ckey[seg * CAP + lane] : 0u;
    ii[u][0] = seg < W ? cidx[seg * CAP + lane] : 0u;
    if (cval && seg < W) vv[u][0] = cval[seg * CAP + lane];
  }
  if (blk == 0) {  // leave the sample histogram zeroed for the next call
    for (int b = t; b < CB; b += 256) chist[b] = 0;
  }
  if (status) {  // select reported a miss: the host runs the exact path
    if (blk == 0 && t == 0) {
      atomicOr(&ctrl->sticky, status);
      if (status_out) *status_out = (int32_t)status;
    }
    return;
  }
  // When the values are not carried from the filter (vals_src != x), every candidate of chunk 0
  // gathers its value now, while the threshold is resolved, not at write time.  (Reading the
  // counter words ahead the same way, for plain-store updates, measured ~1 us SLOWER than the
  // memory-side atomics at C2: it reads every candidate's line; PLAIN does it at dense alpha.)
  uint32_t cc[SPW][PFC];
#pragma unroll
  for (int u = 0; u < SPW; ++u)
#pragma unroll
    for (int c = 0; c < PFC; ++c) cc[u][c] = 0u;
#pragma unroll
  for (int u = 0; u < SPW; ++u) {
    const int64_t seg = seg0 + u;
    if (seg < W && cnt[u] != DENSE && (uint32_t)lane < cnt[u]) {
      if (!cval) vv[u][0] = vals_src[ii[u][0]];
      if (PLAIN && counter) cc[u][0] = (uint32_t)counter[ii[u][0]];
    }
  }
  if (t < 64) {
    uint32_t tot;
    const uint32_t ex = wave_excl_scan(sc, &tot);
    const bool over = __ballot(sc > (uint32_t)SUBCAP) != 0;
    const bool spec_ok = __ballot(sc > SPEC) == 0;
    if (t < NSUB) subbase[t] = ex;
    if (t == 0) {
      subbase[NSUB] = tot;
      flag = (over || tot > (uint32_t)BCAP || need == 0 || need > tot) ? 1u : 0u;
      spec = spec_ok ? 1u : 0u;
    }
  }
  __syncthreads();
  if (flag) {  // identical in every block
    if (blk == 0 && t == 0) {
      ctrl->status = 1;
      atomicOr(&ctrl->sticky, 1u);
      if (status_out) *status_out = 1;
    }
    return;
  }
  STAMP_T0(1);
  Bound bd{blkey, blidx, subbase, bsk, bsi, subbase[NSUB]};
  if (spec) {  // every boundary entry is in a speculative register (nb <= 256 <= BLDS)
    if (sp_slot < subbase[sp_sub + 1] - subbase[sp_sub]) {
      bsk[subbase[sp_sub] + sp_slot] = spk;
      bsi[subbase[sp_sub] + sp_slot] = spi;
    }
    __syncthreads();
  } else {
    bd.load();
  }
  uint32_t T, icut;
  block_resolve(bd, need, lo + (bstar << shift), shift, RL, &T, &icut);
  STAMP_T0(2);
  // selected boundary entries before this block / overall, plus the above counts
  const uint32_t bstart = (uint32_t)((int64_t)blk * CSEG * R);
  uint32_t sb_before = 0, sb_all = 0;
  bd.each([&](uint32_t kv, uint32_t iv) {
    const bool sel = kv > T || (kv == T && iv <= icut);
    sb_all += sel ? 1u : 0u;
    sb_before += (sel && iv < bstart) ? 1u : 0u;
  });
  const uint64_t tot2 = block_sum64(((uint64_t)(abv_all + sb_all) << 32) |
                                        (uint64_t)(abv_before + sb_before), wsum64);
  const uint32_t boff = (uint32_t)tot2, grand = (uint32_t)(tot2 >> 32);
  if (blk == 0 && t == 0) {
    ctrl->T = T;
    ctrl->icut = icut;
    if (grand != (uint32_t)k) {  // internal inconsistency
      ctrl->status = 2;
      atomicOr(&ctrl->sticky, 2u);
    } else if (T > 0u && T < 0x7F800000u) {
      // the next call with this signature may take its window from T (DPZ_TOPK_HINT)
      ctrl->hint_T = T;
      ctrl->hint_sig = sig;
    } else {
      // T == 0 (fewer than k nonzero keys) or a non-finite T gives no window: no prior, so a
      // hinted next call misses at once instead of filtering with a window it must reject
      ctrl->hint_sig = 0u;
    }
    if (status_out) *status_out = grand != (uint32_t)k ? 2 : 0;
  }
  if (grand != (uint32_t)k) return;  // identical in every block: nothing is written
  // chunks 1 .. PFC-1 of every segment with more than 64 candidates: all issued together
  if constexpr (PFC > 1) {
#pragma unroll
    for (int u = 0; u < SPW; ++u) {
      const int64_t seg = seg0 + u;
      if (seg < W && cnt[u] != DENSE && cnt[u] > 64u) {
#pragma unroll
        for (int c = 1; c < PFC; ++c) {
          const uint32_t j = c * 64u + lane;
          if (j < cnt[u]) {
            kk[u][c] = ckey[seg * CAP + j];
            ii[u][c] = cidx[seg * CAP + j];
            if (cval) vv[u][c] = cval[seg * CAP + j];
          }
        }
#pragma unroll
        for (int c = 1; c < PFC; ++c) {
          const uint32_t j = c * 64u + lane;
          if (j < cnt[u] && !cval) vv[u][c] = vals_src[ii[u][c]];
          if (PLAIN && counter && j < cnt[u]) cc[u][c] = (uint32_t)counter[ii[u][c]];
        }
      }
    }
  }
  auto is_sel = [&](uint32_t key, uint32_t idx) { return key > T || (key == T && idx <= icut); };
  // count pass (the first PFC chunks from registers), in-block offsets, write pass
#pragma unroll
  for (int u = 0; u < SPW; ++u) {
    const int64_t seg = seg0 + u;
    uint32_t mine = 0;
    if (seg < W && cnt[u] != DENSE) {
#pragma unroll
      for (int c = 0; c < PFC; ++c) {
        const uint32_t j = c * 64u + lane;
        mine += (uint32_t)__popcll(__ballot(j < cnt[u] && is_sel(kk[u][c], ii[u][c])));
      }
      // dense alpha: the chunks past the registers four at a time (keys in flight together;
      // the index only for a tie with T)
      for (uint32_t j0 = PFC * 64u; j0 < cnt[u]; j0 += 4 * 64u) {
        uint32_t kg[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const uint32_t j = j0 + g * 64u + lane;
          kg[g] = ckey[seg * CAP + (j < cnt[u] ? j : 0u)];
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const uint32_t j = j0 + g * 64u + lane;
          bool sel = false;
          if (j < cnt[u]) sel = kg[g] > T || (kg[g] == T && cidx[seg * CAP + j] <= icut);
          mine += (uint32_t)__popcll(__ballot(sel));
        }
      }
    } else if (seg < W) {
      mine = dense_count<VEC>(s, seg, R, n, lo, T, icut);
    }
    if (lane == 0) wcnt[wid * SPW + u] = mine;
  }
  __syncthreads();
  STAMP_T0(3);
  uint32_t run = boff;
  for (int w = 0; w < wid * SPW; ++w) run += wcnt[w];
  uint32_t* const slrow = SL ? slrows[wid] : nullptr;
#pragma unroll
  for (int u = 0; u < SPW; ++u) {
    const int64_t seg = seg0 + u;
    if (seg >= W) break;
    const int64_t segbeg = seg * R;
    const int segw = SL ? (int)((((segbeg + R < n) ? segbeg + R : n) - segbeg + 31) >> 5) : 0;
    if (SL) {
      for (int j = lane; j < segw; j += 64) slrow[j] = 0u;
      __builtin_amdgcn_wave_barrier();
    }
    if (cnt[u] != DENSE) {
      // pre: the value was read ahead (v valid); otherwise gathered here.  cw: the counter word
      // read ahead (PLAIN)
      auto emit = [&](bool sel, uint32_t idx, float v, bool pre, uint32_t cw) {
        const uint64_t m = __ballot(sel);
        if (sel) {
          const uint32_t pos = run + mbcnt64(m);
          if (pos < (uint64_t)k) {
            idx_out[pos] = (int32_t)idx;
            store_val(val_out, val_h, pos, (cval || pre) ? v : vals_src[idx]);
            if (SL) atomicOr(&slrow[(idx >> 5) - (uint32_t)(segbeg >> 5)], 1u << (idx & 31));
            if (counter) {
              if (PLAIN) counter[idx] = (int32_t)(cw + 1u);  // unique indices: no race
              else atomicAdd(&counter[idx], 1);  // non-returning: no round trip to wait on
            }
            if (rewind) rewind[idx] = 0.0f;
          }
        }
        run += (uint32_t)__popcll(m);
      };
#pragma unroll
      for (int c = 0; c < PFC; ++c) {
        const uint32_t j = c * 64u + lane;
        if (c * 64u < cnt[u])
          emit(j < cnt[u] && is_sel(kk[u][c], ii[u][c]), ii[u][c], vv[u][c], true, cc[u][c]);
      }
      for (uint32_t j0 = PFC * 64u; j0 < cnt[u]; j0 += 4 * 64u) {  // four chunks at a time
        uint32_t kg[4], ig[4];
        float vg[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const uint32_t j = j0 + g * 64u + lane;
          const uint32_t jc = seg * CAP + (j < cnt[u] ? j : 0u);
          kg[g] = ckey[jc];
          ig[g] = cidx[jc];
          vg[g] = cval ? cval[jc] : 0.f;
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const uint32_t j = j0 + g * 64u + lane;
          const bool sel = j < cnt[u] && is_sel(kg[g], ig[g]);
          const uint32_t cw = (PLAIN && counter && sel) ? (uint32_t)counter[ig[g]] : 0u;
          emit(sel, ig[g], vg[g], false, cw);
        }
      }
    } else {
      dense_write<VEC>(s, seg, R, n, k, lo, T, icut, run, vals_src, idx_out, val_out, counter,
                       rewind, val_h, slrow);
      run += wcnt[wid * SPW + u];
    }
    if (SL) {
      // this wave's LDS bit-ors precede the reads in program order (one wave: in order)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      for (int j = lane; j < segw; j += 64) {
        const uint32_t m = slrow[j];
        const int64_t w = (segbeg >> 5) + j;
        selmask[w] = m;
        uint32_t carry = planes ? m : 0u;
        // the ripple carry through the planes, SL_PF planes' words loaded together per step:
        // a wave's longest carry chain (~6-7 planes at 64 lanes) costs ceil(chain / SL_PF)
        // dependent round trips instead of one per plane
        for (int p = 0; p < 32 && carry != 0u; p += SL_PF) {
          uint32_t o[SL_PF];
#pragma unroll
          for (int q = 0; q < SL_PF; ++q) o[q] = planes[(int64_t)(p + q) * nwords + w];
#pragma unroll
          for (int q = 0; q < SL_PF; ++q) {
            if (carry != 0u) {
              planes[(int64_t)(p + q) * nwords + w] = o[q] ^ carry;
              carry &= o[q];
            }
          }
        }
      }
      __builtin_amdgcn_wave_barrier();  // the row is cleared for the next segment after this
    }
  }
  STAMP_T0(4);
}

template <bool VEC, bool PLAIN, int SPW, bool SL>
__global__ void __launch_bounds__(256, SPW >= 8 ? 1 : 4) sampled_compact_kernel(KeySrc s, int64_t n, int64_t k, int64_t W, int64_t R, int64_t CAP, TopkCtrl* ctrl, uint32_t* chist, const uint32_t* __restrict__ blkabove, const uint32_t* __restrict__ blcnt, const uint32_t* __restrict__ blkey, const uint32_t* __restrict__ blidx, const uint32_t* __restrict__ segcnt, const uint32_t* __restrict__ cidx, const uint32_t* __restrict__ ckey, const float* __restrict__ cval, const float* vals_src, int32_t* idx_out, float* val_out, int32_t* counter, float* rewind, int32_t* status_out, ReplaceJob pj, int64_t nrep_first, int val_h, uint32_t* selmask, uint32_t* planes, int64_t nwords, uint32_t* ghist, uint32_t sig) {
  sampled_compact_kernel_body<VEC, PLAIN, SPW, SL>(s, n, k, W, R, CAP, ctrl, chist, blkabove, blcnt, blkey, blidx, segcnt, cidx, ckey, cval, vals_src, idx_out, val_out, counter, rewind, status_out, pj, nrep_first, val_h, selmask, planes, nwords, ghist, sig, (uint32_t)blockIdx.x);
}

// Fractions of a co-scheduled replace job's chunks carried by sample / select / compact;
// DPZ_COSCHED="f0,f1,f2" overrides them in the diagnostic build (dpz_knobs.h).
// Defaults measured on MI355X, see DESIGN.md §3.6.
static void cosched_shares(double f[3]) {
  f[0] = 0.45; f[1] = 0.55; f[2] = 0.0;
  if (const char* e = DPZ_KNOB_STR(COSCHED)) {
    double v[3];
    if (sscanf(e, "%lf,%lf,%lf", &v[0], &v[1], &v[2]) == 3 && v[0] >= 0 && v[1] >= 0 &&
        v[2] >= 0) {
      const double t = v[0] + v[1] + v[2];
      if (t > 0)
        for (int i = 0; i < 3; ++i) f[i] = v[i] / t;
    }
  }
}

template <bool VEC>
static int run_sampled_t(const EncodeArgs& a, const WsLayout& L, int phases) {
  KeySrc s{a.x, a.x0, a.acc, a.acc_mode, 0};
  TopkCtrl* ctrl = reinterpret_cast<TopkCtrl*>(a.ws + L.ctrl);
  uint32_t* chist = reinterpret_cast<uint32_t*>(a.ws + L.chist);
  uint32_t* ghist = reinterpret_cast<uint32_t*>(a.ws + L.f_ghist);
  uint32_t* segcnt = reinterpret_cast<uint32_t*>(a.ws + L.f_segcnt);
  uint32_t* blkabove = reinterpret_cast<uint32_t*>(a.ws + L.f_blkabove);
  uint32_t* cidx = reinterpret_cast<uint32_t*>(a.ws + L.f_cidx);
  uint32_t* ckey = reinterpret_cast<uint32_t*>(a.ws + L.f_ckey);
  // candidate values carried from the filter when the payload values are x itself (PartialModel)
  float* cval = (a.vals_src == a.x) ? reinterpret_cast<float*>(a.ws + L.f_cval) : nullptr;
  uint32_t* blcnt = reinterpret_cast<uint32_t*>(a.ws + L.f_blcnt);
  uint32_t* blkey = reinterpret_cast<uint32_t*>(a.ws + L.f_blkey);
  uint32_t* blidx = reinterpret_cast<uint32_t*>(a.ws + L.f_blidx);
  const FastGeom& g = L.fg;
  const unsigned nb = (unsigned)g.B;
  const unsigned nsel = (unsigned)((g.W + SEL_SEGS - 1) / SEL_SEGS);
  // co-scheduled replace decode: its chunks are split over the four latency-bound launches
  // (sample, select, resolve, compact) and run in blocks appended after each launch's own
  ReplaceJob jb[3] = {};
  unsigned pb[3] = {0, 0, 0};
  // the sample's block size: 256 threads (64 blocks) or 1024 (16 blocks, fewer same-address
  // atomics per histogram bin); DPZ_SAMPLE_THREADS (diagnostic build) forces either
  // (1024-thread blocks measured no faster: 4.7-5.3 vs 4.6-5.4 us)
  const int smp_threads = DPZ_KNOB_INT(SAMPLE_THREADS, 256) == 1024 ? 1024 : 256;
  const int smp_blocks = SMP_NCHUNK / (4 * (smp_threads / 64));
  // a scatter job (dpz_topk_encode_replace over the tensor being encoded): the filter writes
  // out = x as it streams x, and the entries are scattered in blocks of the compact launch
  float* copy_out = (a.job && phases == 3 && a.job->scatter) ? a.job->out : nullptr;
  if (a.job && phases == 3) {
    const int64_t C = a.job->c1 - a.job->c0;
    double f[3];
    cosched_shares(f);
    if (copy_out) {
      // the scatter must follow the filter's copy: blocks appended to compact (default; the
      // latency-bound compact leaves most CU slots free: C2 one-node step 57.2 -> 55.6 us on
      // MI355X vs appended to select) or select (DPZ_SCATTER_AT=select, A/B diagnostics)
      // (DPZ_SCATTER_AT=split: half in each)
      const char* e = DPZ_KNOB_STR(SCATTER_AT);
      const bool at_select = e && e[0] == 's' && e[1] == 'e';
      const bool split = e && e[0] == 's' && e[1] == 'p';
      f[0] = 0.0;
      f[1] = split ? 0.5 : (at_select ? 1.0 : 0.0);
      f[2] = split ? 0.5 : (at_select ? 0.0 : 1.0);
    }
    const int per[3] = {smp_threads / 64, 16, 4};  // chunks per appended block (one per wave)
    int64_t c = a.job->c0;
    double acc_f = 0.0;
    for (int i = 0; i < 3; ++i) {
      acc_f += f[i];
      int64_t e = (i == 2) ? a.job->c1 : a.job->c0 + (int64_t)(acc_f * (double)C + 0.5);
      if (e > a.job->c1) e = a.job->c1;
      if (e < c) e = c;
      jb[i] = *a.job;
      jb[i].c0 = c;
      jb[i].c1 = e;
      pb[i] = (unsigned)((e - c + per[i] - 1) / per[i]);
      c = e;
    }
  }
  // The pipelined filter (PartialModel: aligned, no accumulation): depth 2 at 8 waves / SIMD
  // when the grid needs them (more than 4096 segments), else depth DPZ_FILTER_DEPTH (default
  // 4) at 4 waves / SIMD.  DPZ_FILTER_PIPE=0 selects the batched filter (A/B diagnostics).
  const int pipe = (int)DPZ_KNOB_INT(FILTER_PIPE, 1);
  const bool add_only = a.acc_mode == DPZ_ACC_ADD && !a.x0;
  const bool piped = VEC && (a.acc_mode == DPZ_ACC_NONE || add_only) && pipe > 0;
  // a prior-round window replaces the sample launch (pipelined filter only; a co-scheduled
  // decode with blocks in the sample launch keeps it — the fused one rides in compact only)
  const uint32_t hsig = (piped && (!a.job || pb[0] == 0)) ? a.hint_sig : 0u;
  const uint32_t sig = hint_signature(a.n, a.k, a.shared, a.acc_mode, a.x0 != nullptr);
  if (phases & 1) {
    if (!hsig)
      DPZ_TIMED(DPZ_KT_TOPK_SAMPLE, a.st,
                sampled_sample_kernel<<<smp_blocks + pb[0], smp_threads, 0, a.st>>>(
                    s, a.n, ctrl, chist, ghist, blcnt, jb[0], smp_blocks, a.val_h));
    uint32_t r_lo, r_hi;
    window_ranks(a.n, a.k, &r_lo, &r_hi);
    const int depth = (int)DPZ_KNOB_INT(FILTER_DEPTH, 4);
    if (piped) {
      const bool x0 = a.x0 != nullptr;
      // the fold base (dpz_topk_encode_foldbase) rides on the same copy slot
      const bool fbase = a.fbase && a.base_out && x0 && !copy_out;
      float* const cpo = fbase ? a.base_out : copy_out;
      FoldBase fbv{};
      if (fbase) fbv = *a.fbase;
      const int dsel = g.W > 4096 ? 2 : (depth >= 8 ? 8 : (depth >= 6 ? 6 : 4));
#define DPZ_PIPE(D_, O_)                                                                      \
  do {                                                                                        \
    if (add_only) DPZ_PIPE1(2, 0, D_, O_);                                                    \
    else if (fbase) DPZ_PIPE1(1, 2, D_, O_);                                                  \
    else if (x0 && copy_out) DPZ_PIPE1(1, 1, D_, O_);                                         \
    else if (x0) DPZ_PIPE1(1, 0, D_, O_);                                                     \
    else if (copy_out) DPZ_PIPE1(0, 1, D_, O_);                                               \
    else DPZ_PIPE1(0, 0, D_, O_);                                                             \
  } while (0)
#define DPZ_PIPE2(X0_, CP_, D_, O_, XNT_)                                                     \
  DPZ_TIMED(DPZ_KT_TOPK_FILTER, a.st, (sampled_filter_pipe_kernel<X0_, CP_, D_, O_, XNT_><<<nb, 256, 0, a.st>>>( \
      s, a.n, r_lo, r_hi, g.W, g.R, g.CAP, ctrl, chist, ghist, segcnt, cidx, ckey, cval, cpo, \
      fbv, hsig, blcnt, a.val_h)))
      // x with the default cache policy (DPZ_TOPK_KEEP_X) for the plugin's encode (CP 0) and the
      // fold-base encode (CP 2), whose callers read x again in the fold
#define DPZ_PIPE1(X0_, CP_, D_, O_)                                                           \
  do {                                                                                        \
    if ((CP_ == 0 || CP_ == 2) && X0_ == 1 && a.keep_x) DPZ_PIPE2(X0_, CP_, D_, O_, false);   \
    else DPZ_PIPE2(X0_, CP_, D_, O_, true);                                                   \
  } while (0)
      switch (dsel) {
        case 2: DPZ_PIPE(2, 8); break;
        case 8: DPZ_PIPE(8, 4); break;
        case 6: DPZ_PIPE(6, 4); break;
        default: DPZ_PIPE(4, 4); break;
      }
#undef DPZ_PIPE2
#undef DPZ_PIPE1
#undef DPZ_PIPE
    } else if (a.acc_mode == DPZ_ACC_NONE)
      DPZ_TIMED(DPZ_KT_TOPK_FILTER, a.st, sampled_filter_kernel<VEC, false, FG><<<nb, 256, 0, a.st>>>(
          s, a.n, r_lo, r_hi, g.W, g.R, g.CAP, ctrl, chist, ghist, segcnt, cidx, ckey, cval,
          copy_out));
    else
      DPZ_TIMED(DPZ_KT_TOPK_FILTER, a.st, sampled_filter_kernel<VEC, true, 3><<<nb, 256, 0, a.st>>>(
          s, a.n, r_lo, r_hi, g.W, g.R, g.CAP, ctrl, chist, ghist, segcnt, cidx, ckey, cval,
          copy_out));
  }
  if (!(phases & 2)) return DPZ_OK;
  s.rekey = 1;
  DPZ_TIMED(DPZ_KT_TOPK_SELECT, a.st, sampled_select_kernel<VEC><<<nsel + pb[1], 1024, 0, a.st>>>(
      s, a.n, a.k, g.W, g.B, g.R, g.CAP, ctrl, ghist, segcnt, cidx, ckey, blkabove, blcnt, blkey,
      blidx, jb[1]));
  float* rewind = (a.acc && a.acc_mode != DPZ_ACC_NONE && !a.selmask) ? a.acc : nullptr;
  // DPZ_COMPACT_ABLATE (diagnostic build only; results then differ from the reference): bit 0
  // drops the accumulator rewind, bit 1 the counter update — per-side-effect cost of compact
  const int ablate = (int)DPZ_KNOB_INT(COMPACT_ABLATE, 0);
  if (ablate & 1) rewind = nullptr;
  int32_t* const counter = ((ablate & 2) || a.selmask) ? nullptr : a.counter;
  // DPZ_COUNTER_PLAIN=0 / 1 forces the counter update form (diagnostic build, A/B)
  const bool plain = DPZ_KNOB_INT(COUNTER_PLAIN, a.k > a.n / 32 ? 1 : 0) != 0;
  // DPZ_SCATTER_FIRST=1: the decode's blocks dispatched ahead of compact's own (diagnostic, A/B)
  const int64_t nrep_first = DPZ_KNOB_INT(SCATTER_FIRST, 0) != 0 ? (int64_t)pb[2] : 0;
  // sparse alpha: 8 segments per wave, one compact block per CU; dense alpha: 2 segments per
  // wave with four chunks each in registers (DPZ_COMPACT_SPW=2 / 8 forces, diagnostic build)
  // (8 segments per wave, one block per CU, measured SLOWER at C2: 18.7 vs 12 us — the count and
  // write passes serialise four times the segments per wave, and the prologue does not get faster)
  const int spw = (int)DPZ_KNOB_INT(COMPACT_SPW, 2);
#define DPZ_COMPACT(PL_, SPW_, SL_)                                                               \
  DPZ_TIMED(DPZ_KT_TOPK_COMPACT, a.st,                                                            \
            (sampled_compact_kernel<VEC, PL_, SPW_, SL_><<<(unsigned)((g.W + 4 * SPW_ - 1) /       \
                                                                     (4 * SPW_)) + pb[2],         \
                                                           256, 0, a.st>>>(                       \
                s, a.n, a.k, g.W, g.R, g.CAP, ctrl, chist, blkabove, blcnt, blkey, blidx, segcnt, \
                cidx, ckey, cval, a.vals_src, a.idx_out, a.val_out, counter, rewind,              \
                a.status_out, jb[2], nrep_first, a.val_h, a.selmask, a.planes, mask_words(a.n),  \
                ghist, sig)))
  if (a.selmask && g.R <= SL_RMAX) {
    // sliced side effects (dpz_topk_encode_sliced) from per-wave LDS rows of the segment's words
    DPZ_COMPACT(false, 2, true);
  } else if (plain) {  // (sliced with longer segments: counter and rewind are null here, the
                       // caller builds the mask and the planes from idx_out)
    if (spw == 8) DPZ_COMPACT(true, 8, false);
    else DPZ_COMPACT(true, 2, false);
  } else {
    if (spw == 8) DPZ_COMPACT(false, 8, false);
    else DPZ_COMPACT(false, 2, false);
  }
#undef DPZ_COMPACT
  return DPZ_OK;
}

#ifdef DPZ_STAMPS
extern "C" int dpz_debug_filter_stamps(unsigned long long* host_out) {
  return (int)hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_fst), sizeof(g_fst));
}

extern "C" int dpz_debug_block_stamps(unsigned long long* host_out) {
  return (int)hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_bst), sizeof(g_bst));
}

extern "C" int dpz_debug_stamps(unsigned long long* host_out, int reset) {
  if (host_out) DPZ_HIP_TRY(hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_stamps), sizeof(g_stamps)));
  if (reset) {
    unsigned long long init[64];
    for (int i = 0; i < 64; ++i) init[i] = (i == 0 || i == 2 || i == 4 || i == 6 || i == 13) ? ~0ull : 0ull;
    DPZ_HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), init, sizeof(init)));
  }
  return 0;
}
#endif

// ---- the encodes of m nodes, one launch per phase (dpz_topk_encode_nodes) ----------------------
// A simulated gossip round encodes every node's model (reference: each node process runs
// sharing/PartialModel.py:164-255).  Node after node on a few streams, each encode is four
// dependent launches whose selection tail leaves the GPU idle; here every phase runs for all m
// nodes in ONE launch (grid = m x the per-node grid, block b -> node b / per-node blocks), so the
// tails of all nodes overlap each other and the filter streams all m models back to back.
struct EncNode {
  const float* x;
  const float* x0;
  int32_t* counter;
  int32_t* idx_out;
  float* val_out;
  char* ws;
  int32_t* status_out;
  uint64_t pad;
};
static_assert(sizeof(EncNode) == 64, "node table entry: 8 x 64-bit words (dpz_codec.h)");
struct WsOff {
  uint64_t ctrl, chist, ghist, segcnt, blkabove, cidx, ckey, cval, blcnt, blkey, blidx;
};

template <class T>
__device__ __forceinline__ T* wsp(char* ws, uint64_t off) {
  return reinterpret_cast<T*>(ws + off);
}

__global__ void __launch_bounds__(1024) nodes_sample_kernel(const EncNode* __restrict__ tab,
                                                            WsOff o, int64_t n, int nsb) {
  const uint32_t node = blockIdx.x / (uint32_t)nsb, bid = blockIdx.x % (uint32_t)nsb;
  const EncNode e = tab[node];
  KeySrc s{e.x, e.x0, nullptr, DPZ_ACC_NONE, 0};
  sampled_sample_kernel_body(s, n, wsp<TopkCtrl>(e.ws, o.ctrl), wsp<uint32_t>(e.ws, o.chist),
                             wsp<uint32_t>(e.ws, o.ghist), wsp<uint32_t>(e.ws, o.blcnt),
                             ReplaceJob{}, nsb, 0, bid);
}

template <int D, int OCC>
__global__ void __launch_bounds__(256, OCC) nodes_filter_kernel(
    const EncNode* __restrict__ tab, WsOff o, int64_t n, uint32_t r_lo, uint32_t r_hi, int64_t W,
    int64_t R, int64_t CAP, uint32_t nb, uint32_t hsig) {
  const uint32_t node = blockIdx.x / nb, bid = blockIdx.x % nb;
  const EncNode e = tab[node];
  KeySrc s{e.x, e.x0, nullptr, DPZ_ACC_NONE, 0};
  sampled_filter_pipe_kernel_body<1, 0, D, OCC, true>(
      s, n, r_lo, r_hi, W, R, CAP, wsp<TopkCtrl>(e.ws, o.ctrl), wsp<const uint32_t>(e.ws, o.chist),
      wsp<uint32_t>(e.ws, o.ghist), wsp<uint32_t>(e.ws, o.segcnt), wsp<uint32_t>(e.ws, o.cidx),
      wsp<uint32_t>(e.ws, o.ckey), wsp<float>(e.ws, o.cval), nullptr, FoldBase{}, hsig,
      wsp<uint32_t>(e.ws, o.blcnt), 0, bid);
}

__global__ void __launch_bounds__(1024) nodes_select_kernel(const EncNode* __restrict__ tab,
                                                            WsOff o, int64_t n, int64_t k,
                                                            int64_t W, int64_t B, int64_t R,
                                                            int64_t CAP, uint32_t nsel) {
  const uint32_t node = blockIdx.x / nsel, bid = blockIdx.x % nsel;
  const EncNode e = tab[node];
  KeySrc s{e.x, e.x0, nullptr, DPZ_ACC_NONE, 1};
  sampled_select_kernel_body<true>(
      s, n, k, W, B, R, CAP, wsp<TopkCtrl>(e.ws, o.ctrl), wsp<const uint32_t>(e.ws, o.ghist),
      wsp<const uint32_t>(e.ws, o.segcnt), wsp<const uint32_t>(e.ws, o.cidx),
      wsp<const uint32_t>(e.ws, o.ckey), wsp<uint32_t>(e.ws, o.blkabove),
      wsp<uint32_t>(e.ws, o.blcnt), wsp<uint32_t>(e.ws, o.blkey), wsp<uint32_t>(e.ws, o.blidx),
      ReplaceJob{}, bid);
}

#ifndef DPZ_NODES_NO_COUNTER  // ablation only (results then differ): no counter update
#define DPZ_NODES_NO_COUNTER 0
#endif
// SL (DPZ_TOPK_SLICED): the counter in bit-sliced form — the node table's counter word points at
// its planes and the last word at the selection mask, which compact writes (as
// dpz_topk_encode_sliced) instead of the scattered counter[idx] += 1 atomics
template <bool PLAIN, bool SL>
__global__ void __launch_bounds__(256, 4) nodes_compact_kernel(const EncNode* __restrict__ tab,
                                                               WsOff o, int64_t n, int64_t k,
                                                               int64_t W, int64_t R, int64_t CAP,
                                                               uint32_t ncb, int64_t nwords,
                                                               uint32_t sig) {
  const uint32_t node = blockIdx.x / ncb, bid = blockIdx.x % ncb;
  const EncNode e = tab[node];
  KeySrc s{e.x, e.x0, nullptr, DPZ_ACC_NONE, 1};
  int32_t* const counter = SL || DPZ_NODES_NO_COUNTER ? nullptr : e.counter;
  uint32_t* const selmask = SL ? reinterpret_cast<uint32_t*>(e.pad) : nullptr;
  uint32_t* const planes = SL ? reinterpret_cast<uint32_t*>(e.counter) : nullptr;
  sampled_compact_kernel_body<true, PLAIN, 2, SL>(
      s, n, k, W, R, CAP, wsp<TopkCtrl>(e.ws, o.ctrl), wsp<uint32_t>(e.ws, o.chist),
      wsp<const uint32_t>(e.ws, o.blkabove), wsp<const uint32_t>(e.ws, o.blcnt),
      wsp<const uint32_t>(e.ws, o.blkey), wsp<const uint32_t>(e.ws, o.blidx),
      wsp<const uint32_t>(e.ws, o.segcnt), wsp<const uint32_t>(e.ws, o.cidx),
      wsp<const uint32_t>(e.ws, o.ckey), wsp<const float>(e.ws, o.cval), e.x, e.idx_out,
      e.val_out, counter, nullptr, e.status_out, ReplaceJob{}, 0, 0, selmask, planes, nwords,
      wsp<uint32_t>(e.ws, o.ghist), sig, bid);
}

int topk_encode_nodes(int m, const void* table, int64_t n, int64_t k, size_t ws_bytes, int flags,
                      hipStream_t st) {
  if (m < 1 || !table || n <= 0 || n >= (int64_t(1) << 31) || k < 1 || k > n) return DPZ_ERR_ARG;
  if (flags & ~(DPZ_TOPK_HINT | DPZ_TOPK_SLICED)) return DPZ_ERR_ARG;
  if (!use_sampled(n, k)) return DPZ_ERR_UNSUPPORTED;
  const bool sl = (flags & DPZ_TOPK_SLICED) != 0;
  if (ws_bytes < ws_bytes_needed(n, k)) return DPZ_ERR_WORKSPACE;
  // the shared-GPU geometry (DPZ_TOPK_SHARED): many codecs run at once, and the smaller filter
  // grid per node leaves CU slots to the other nodes' kernels
  const WsLayout L = ws_layout(n, k, true);
  const FastGeom& g = L.fg;
  const WsOff o{L.ctrl, L.chist, L.f_ghist, L.f_segcnt, L.f_blkabove, L.f_cidx, L.f_ckey,
                L.f_cval, L.f_blcnt, L.f_blkey, L.f_blidx};
  const EncNode* tab = static_cast<const EncNode*>(table);
  const uint32_t sig = hint_signature(n, k, true, DPZ_ACC_NONE, true);
  const uint32_t hsig = (flags & DPZ_TOPK_HINT) ? sig : 0u;
  const int nsb = SMP_NCHUNK / 16;  // 256-thread sample blocks per node
  const uint32_t nb = (uint32_t)g.B, nsel = (uint32_t)((g.W + SEL_SEGS - 1) / SEL_SEGS);
  const uint32_t ncb = (uint32_t)((g.W + 7) / 8);
  if ((uint64_t)m * nb >= (1ull << 31) || (uint64_t)m * ncb >= (1ull << 31)) return DPZ_ERR_ARG;
  // a sliced compact builds a segment's mask words in one LDS row
  if (sl && (g.R > SL_RMAX || (g.R & 31) != 0)) return DPZ_ERR_UNSUPPORTED;
  if (!hsig)
    DPZ_TIMED(DPZ_KT_TOPK_SAMPLE, st,
              nodes_sample_kernel<<<(unsigned)(m * nsb), 256, 0, st>>>(tab, o, n, nsb));
  uint32_t r_lo, r_hi;
  window_ranks(n, k, &r_lo, &r_hi);
  if (g.W > 4096)
    DPZ_TIMED(DPZ_KT_TOPK_FILTER, st, (nodes_filter_kernel<2, 8><<<(unsigned)(m * nb), 256, 0, st>>>(
        tab, o, n, r_lo, r_hi, g.W, g.R, g.CAP, nb, hsig)));
  else
    DPZ_TIMED(DPZ_KT_TOPK_FILTER, st, (nodes_filter_kernel<4, 4><<<(unsigned)(m * nb), 256, 0, st>>>(
        tab, o, n, r_lo, r_hi, g.W, g.R, g.CAP, nb, hsig)));
  DPZ_TIMED(DPZ_KT_TOPK_SELECT, st, nodes_select_kernel<<<(unsigned)(m * nsel), 1024, 0, st>>>(
      tab, o, n, k, g.W, g.B, g.R, g.CAP, nsel));
  if (sl)
    DPZ_TIMED(DPZ_KT_TOPK_COMPACT, st, (nodes_compact_kernel<false, true><<<(unsigned)(m * ncb), 256, 0, st>>>(
        tab, o, n, k, g.W, g.R, g.CAP, ncb, mask_words(n), sig)));
  else if (k > n / 32)
    DPZ_TIMED(DPZ_KT_TOPK_COMPACT, st, (nodes_compact_kernel<true, false><<<(unsigned)(m * ncb), 256, 0, st>>>(
        tab, o, n, k, g.W, g.R, g.CAP, ncb, mask_words(n), sig)));
  else
    DPZ_TIMED(DPZ_KT_TOPK_COMPACT, st, (nodes_compact_kernel<false, false><<<(unsigned)(m * ncb), 256, 0, st>>>(
        tab, o, n, k, g.W, g.R, g.CAP, ncb, mask_words(n), sig)));
  return DPZ_OK;
}

bool fused_foldbase_ok(const EncodeArgs& a, bool vec) {
  // the pipelined filter's PartialModel configuration (run_sampled_t): aligned operands, no
  // accumulation, a change against x0; the whole encode in one call (no phase split)
  return vec && a.acc_mode == DPZ_ACC_NONE && a.x0 && aligned16(a.base_out) &&
         DPZ_KNOB_INT(FILTER_PIPE, 1) > 0 && use_sampled(a.n, a.k) && !a.job;
}

int run_sampled(const EncodeArgs& a, const WsLayout& L, bool vec, int phases) {
  return vec ? run_sampled_t<true>(a, L, phases) : run_sampled_t<false>(a, L, phases);
}

}  // namespace dpz
