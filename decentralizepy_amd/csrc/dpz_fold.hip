// Batched decode (replace) + Metro-Hastings weighted fold over a gossip round's payloads.
//
// Replaces (reference sacs-epfl/decentralizepy, src/decentralizepy/):
//   sharing/PartialModel.py:257-303  deserialized_model: T = cat(local); T[idx] = params
//   sharing/Sharing.py:156-190       _averaging: total = T_0*w_0; total += T_i*w_i; += (1-sum)*local
//   sharing/Sharing.py:200-229       _averaging_server: w = 1/n, no self term
//   sharing/JWINS/Wavelet.py:269-309 the same fold on wavelet coefficients
//
// Two launches per group of <= 16 payloads:
//  * fold_offsets_kernel: four payload entries per thread write, for every 4096-element output
//    tile that starts after the previous entry, the first entry index inside that tile
//    (start[p][t] = lower_bound(idx_p, t*4096)).  Coalesced over idx; replaces a dependent
//    binary search per tile.
//  * fold_kernel: persistent blocks walk 4096-element tiles (the next tile's entry ranges
//    prefetched).  Every payload's entries of the tile are loaded up front, flattened.  Then
//    - hit-chain path (no dense payload, <= FOLD_CAP entries in the tile): entries are pushed on
//      per-element hit chains in LDS in one pass; every element folds its base value alone
//      (packed fp32 pairs), and the tile's distinct hit elements, compacted to a list, are
//      folded exactly with their payload values (one thread each) and replace that result;
//    - phase path (dense payloads / dense alpha): per payload the block scatters the tile's hits
//      into an LDS value tile tagged with the payload number (the next payload's extra entries
//      prefetched meanwhile), and every thread folds its 8 elements:
//        t = (tag == p) ? hit : local;  total = (p == 0) ? t*w : total + t*w
//  * fold_group_kernel instead, for all-sparse groups of >= 8 payloads at moderate density
//    (JWINS alpha 0.03-0.1 x 16): every entry of the tile loaded at tile start, payloads folded
//    four at a time from their own LDS value slots (two barriers per four payloads).
//    All follow the reference's fp32 order exactly (library compiled with -ffp-contract=off).
// Algorithmic bytes: read local (4N) + write out (4N) + 8 bytes per payload entry.
#include <cstdlib>
#include <type_traits>

#include "dpz_common.h"
#include "dpz_replace.h"

namespace dpz {

#ifndef DPZ_FOLD_TS
#define DPZ_FOLD_TS 12
#endif
#ifndef DPZ_FOLD_THREADS
#define DPZ_FOLD_THREADS 512
#endif
constexpr int FOLD_TILE_SHIFT = DPZ_FOLD_TS;
constexpr int FOLD_TILE = 1 << FOLD_TILE_SHIFT;
constexpr int FOLD_MAXP = 16;  // payloads per launch (longer lists are chained)
constexpr int FOLD_THREADS = DPZ_FOLD_THREADS;
constexpr int FOLD_GROUPS = FOLD_TILE / (4 * FOLD_THREADS);  // float4 groups per thread
constexpr int FOLD_EQ = 4;  // payload entries per thread preloaded at tile start
constexpr int FOLD_POOL = 64;  // hit-chain path: elements hit by >= 3 payloads folded from LDS rows
constexpr int FOLD_NB = 4;  // phase path: next payload's extra entries per thread prefetched
// hit-chain path: per-element chain head (u32) + per-entry value and (next | payload << 16),
// the tile's local values and the distinct-hit list: 61 KB of LDS at 2816 entries (2 blocks of
// 512 threads per CU, as the registers allow)
constexpr int FOLD_CAP = FOLD_TILE / 16 * 11;
constexpr int FOLD_LDS_MASK = FOLD_TILE * 4 + FOLD_CAP * 8 + FOLD_TILE * 4 + FOLD_CAP * 2;
constexpr int FOLD_LDS_PHASE = FOLD_TILE * 4 + FOLD_TILE;
constexpr int FOLD_LDS_BYTES = FOLD_LDS_MASK > FOLD_LDS_PHASE ? FOLD_LDS_MASK : FOLD_LDS_PHASE;

struct FoldPayload {
  const int32_t* idx;  // nullptr: dense payload (vals has n entries)
  const float* val;
  int64_t k;
  float w;
};

struct FoldArgs {
  const float* local;
  float* out;
  float* out2;  // DPZ_FOLD_ALSO_LOCAL: the result also over local (in place), else nullptr
  const int32_t* starts;  // [np][ntiles + 1]
  int64_t n;
  int64_t ntiles;
  int np;
  int first;        // total starts from payload 0 (else continue from out)
  int add_self;     // add local * w_self at the end
  int replace_only; // out = t_0
  int zero_base;    // sparse payloads contribute 0 off their entries; first term = +0 + t0*w0
  int all_sparse;   // no dense payload in this group: the one-phase hit-chain path may run
  uint32_t dense_mask;  // bit p: payload p is dense (idx == nullptr)
  float w_self;
  FoldPayload p[FOLD_MAXP];
};

// grid (ceil((kmax+1)/256), np): thread j of payload p handles entry j (j == k: end sentinel).
// grid (ceil((kmax + 1) / (4 * 256)), np): thread g of payload p handles entries 4g .. 4g + 3
// (j == k: the end sentinel); the four indices come in one 16-byte load when aligned.
template <int SHIFT>
__global__ void __launch_bounds__(256) fold_offsets_kernel(FoldArgs a, int32_t* starts,
                                                           int64_t ntiles) {
  const int p = blockIdx.y;
  const FoldPayload& P = a.p[p];
  if (!P.idx) return;
  const int64_t j0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  const int64_t k = P.k;
  if (j0 > k) return;
  int32_t v[5];  // idx[j0 - 1 .. j0 + 3]
  v[0] = j0 == 0 ? 0 : P.idx[j0 - 1];
  if (j0 + 4 <= k && (reinterpret_cast<uintptr_t>(P.idx + j0) & 15u) == 0) {
    const int4 q = *reinterpret_cast<const int4*>(P.idx + j0);
    v[1] = q.x; v[2] = q.y; v[3] = q.z; v[4] = q.w;
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e + 1] = (j0 + e < k) ? P.idx[j0 + e] : 0;
  }
  int32_t* st = starts + (int64_t)p * (ntiles + 1);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int64_t j = j0 + e;
    if (j > k) break;
    int64_t tprev = j == 0 ? -1 : ((int64_t)v[e] >> SHIFT);
    int64_t tcur = j == k ? ntiles : ((int64_t)v[e + 1] >> SHIFT);
    // an invalid payload (negative / too large / unsorted indices) must not write out of bounds
    if (tprev < -1) tprev = -1;
    if (tprev > ntiles) tprev = ntiles;
    if (tcur > ntiles) tcur = ntiles;
    for (int64_t t = tprev + 1; t <= tcur; ++t) st[t] = (int32_t)j;
  }
}

// A payload pointer rebuilt from lane registers (readlane) or read back from an LDS table has lost
// its address space: loads through it compile to FLAT loads, which count on lgkmcnt as well as vmcnt, so every LDS wait
// of the fold would also wait for the window loads in flight.  Global loads count on vmcnt only.
template <class T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* as_global(const T* p) {
  return (const __attribute__((address_space(1))) T*)p;
}

// one payload term of the fold in the reference's fp32 order: the first term of a fresh total is
// t*w (+0 first with a zero base), later terms add; replace-only keeps the payload value
__device__ __forceinline__ void fold_term(float& acc, float tv, float w, bool first_term,
                                          int replace_only, int zero_base) {
  if (replace_only) {
    acc = tv;
  } else {
    const float term = tv * w;
    acc = first_term ? (zero_base ? 0.0f + term : term) : acc + term;
  }
}

#ifdef DPZ_STAMPS  // diagnostic build only: per (block, tile iteration) phase stamps
__device__ unsigned long long g_fold_st[6][8192];
#define FSTAMP(i)                                                    \
  do {                                                               \
    if (threadIdx.x == 0 && it_ < 16 && blockIdx.x < 512)            \
      g_fold_st[i][blockIdx.x * 16 + it_] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define FSTAMP(i) do {} while (0)
#endif

template <bool VEC>
__global__ void __launch_bounds__(FOLD_THREADS, 4) fold_kernel(FoldArgs a) {
  // phase path: hv (value tile) + htag (payload tag); hit-mask path: msk + epos + ev
  __shared__ __attribute__((aligned(16))) uint8_t lds_raw[FOLD_LDS_BYTES];
  float* hv = reinterpret_cast<float*>(lds_raw);
  uint8_t* htag = lds_raw + FOLD_TILE * sizeof(float);
  __shared__ int32_t rng[FOLD_MAXP][2];
  __shared__ int32_t pre[FOLD_MAXP + 1];  // flattened entry offset of each payload's tile range
  const int t = threadIdx.x;
  // payload pointer table in LDS: the entry loads below pick their payload per lane, and a
  // per-lane index into the kernel-argument array is a dependent global load per tile
  __shared__ const __attribute__((address_space(1))) int32_t* s_idx[FOLD_MAXP];  // as_global
  __shared__ const __attribute__((address_space(1))) float* s_val[FOLD_MAXP];
  __shared__ uint32_t s_nhit;
  __shared__ uint32_t s_pool_n;                // rows of s_pool taken in this tile
  __shared__ float s_pool[FOLD_POOL][FOLD_MAXP];  // payload values of elements hit >= 3 times
  __shared__ float s_w[FOLD_MAXP];
  if (t == 0) {
    for (int p = 0; p < a.np; ++p) {
      s_idx[p] = as_global(a.p[p].idx);
      s_val[p] = as_global(a.p[p].val);
      s_w[p] = a.p[p].w;
    }
  }
  // persistent blocks: tile, tile + gridDim.x, ...; the next tile's entry ranges are loaded
  // while the current tile is folded
  int32_t nr0 = 0, nr1 = 0;
  const bool rng_lane = t < a.np && !((a.dense_mask >> t) & 1u);
  if (rng_lane && (int64_t)blockIdx.x < a.ntiles) {
    const int32_t* st = a.starts + (int64_t)t * (a.ntiles + 1);
    nr0 = st[blockIdx.x];
    nr1 = st[blockIdx.x + 1];
  }
  float L[4 * FOLD_GROUPS];
  // local values of tile `tl` into L: issued early, consumed a phase later (loads stay in
  // flight across the plain barriers in between)
  auto load_local = [&](int64_t tl) {
    const int64_t lo_ = tl * FOLD_TILE;
    const int64_t hi_ = (lo_ + FOLD_TILE < a.n) ? lo_ + FOLD_TILE : a.n;
#pragma unroll
    for (int q = 0; q < FOLD_GROUPS; ++q) {
      const int64_t i0 = lo_ + q * 4 * FOLD_THREADS + t * 4;
      if (VEC && i0 + 3 < hi_) {
        float4 v = *reinterpret_cast<const float4*>(a.local + i0);
        L[q * 4 + 0] = v.x; L[q * 4 + 1] = v.y; L[q * 4 + 2] = v.z; L[q * 4 + 3] = v.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) L[q * 4 + e] = i0 + e < hi_ ? a.local[i0 + e] : 0.0f;
      }
    }
  };
  if ((int64_t)blockIdx.x < a.ntiles) load_local(blockIdx.x);
  int it_ = -1;
  (void)it_;
  for (int64_t tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
  ++it_;
  FSTAMP(0);
  const int64_t tlo = tile * FOLD_TILE;
  const int64_t thi = (tlo + FOLD_TILE < a.n) ? tlo + FOLD_TILE : a.n;
  if (t < 64) {
    // entry ranges and their flattened offsets (a wave scan; pre[u] = etot for u >= np)
    const int32_t c = (t < a.np && nr1 > nr0) ? nr1 - nr0 : 0;
    if (t < a.np) {
      rng[t][0] = nr0;
      rng[t][1] = nr1;
    }
    int32_t incl = c;
#pragma unroll
    for (int d = 1; d < FOLD_MAXP; d <<= 1) {
      const int32_t v = __shfl_up(incl, d, 64);
      if (t >= d) incl += v;
    }
    if (t < FOLD_MAXP) pre[t + 1] = incl;
    if (t == 0) pre[0] = 0;
  }
  if (rng_lane && tile + gridDim.x < a.ntiles) {
    const int32_t* st = a.starts + (int64_t)t * (a.ntiles + 1);
    nr0 = st[tile + gridDim.x];
    nr1 = st[tile + gridDim.x + 1];
  }

  // this thread's elements: q-th group = tlo + q*1024 + 4t .. +3; L (the local values) was
  // loaded ahead (prologue, or behind the previous tile's hit fold)
  float acc[4 * FOLD_GROUPS];
  if (!a.first) {
#pragma unroll
    for (int q = 0; q < FOLD_GROUPS; ++q) {
      const int64_t i0 = tlo + q * 4 * FOLD_THREADS + t * 4;
      if (VEC && i0 + 3 < thi) {
        float4 o = *reinterpret_cast<const float4*>(a.out + i0);
        acc[q * 4 + 0] = o.x; acc[q * 4 + 1] = o.y; acc[q * 4 + 2] = o.z; acc[q * 4 + 3] = o.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[q * 4 + e] = i0 + e < thi ? a.out[i0 + e] : 0.0f;
      }
    }
  }
  bool l_ahead = false;  // L already holds the next tile's values

  __syncthreads();  // rng / pre visible
  FSTAMP(1);
  // every payload's entries of this tile (flattened, the first FOLD_EQ * FOLD_THREADS of them)
  // are loaded before any is used: one memory latency per tile instead of one per payload
  int ep[FOLD_EQ];
  int32_t ei[FOLD_EQ];
  float evl[FOLD_EQ];
  const int32_t etot = pre[a.np];
#pragma unroll
  for (int q = 0; q < FOLD_EQ; ++q) {
    const int32_t j = t + q * FOLD_THREADS;
    ep[q] = -1;
    ei[q] = 0;
    evl[q] = 0.0f;
    if (j < etot) {
      // payload of flattened entry j: binary search over pre[0..15] (pre[u] = etot > j for
      // u >= np), four dependent LDS reads instead of a read per payload
      int p = 0;
#pragma unroll
      for (int s = FOLD_MAXP / 2; s >= 1; s >>= 1) p += pre[p + s] <= j ? s : 0;
      const int64_t src = (int64_t)rng[p][0] + (j - pre[p]);
      ep[q] = p;
      ei[q] = s_idx[p][src];
      evl[q] = s_val[p][src];
    }
  }

  if (a.all_sparse && etot <= FOLD_CAP) {
    // Hit-chain path.  The fold is VALU-bound when every element runs the per-payload select
    // (16 payloads x 8 elements x ~6 instructions per thread), so it is split:
    //  A) every element folds its base value alone (no hits): 2 flops per payload term, packed;
    //  B) the tile's hit elements (~15 % at 16 payloads x 1 %), compacted to a list, are folded
    //     exactly with their payload values by one thread each and overwrite A's result.
    // Entries are pushed on per-element hit chains (head[pos] -> j -> ...) in one scatter phase.
    uint32_t* head = reinterpret_cast<uint32_t*>(lds_raw);
    uint32_t* meta = head + FOLD_TILE;                       // next (low 16) | payload << 16
    float* ev = reinterpret_cast<float*>(meta + FOLD_CAP);
    float* lv = ev + FOLD_CAP;                               // the tile's local values
    uint16_t* hitl = reinterpret_cast<uint16_t*>(lv + FOLD_TILE);  // distinct hit elements
    for (int j = t * 4; j < FOLD_TILE; j += 4 * FOLD_THREADS)
      *reinterpret_cast<uint4*>(&head[j]) = make_uint4(~0u, ~0u, ~0u, ~0u);
#pragma unroll
    for (int q = 0; q < FOLD_GROUPS; ++q)
      *reinterpret_cast<float4*>(&lv[q * 4 * FOLD_THREADS + t * 4]) =
          make_float4(L[q * 4 + 0], L[q * 4 + 1], L[q * 4 + 2], L[q * 4 + 3]);
    if (t == 0) {
      s_nhit = 0;
      s_pool_n = 0;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < FOLD_EQ; ++q) {
      if (ep[q] >= 0) {
        const int32_t j = t + q * FOLD_THREADS;
        const int64_t pos = (int64_t)ei[q] - tlo;
        ev[j] = evl[q];
        if (pos >= 0 && pos < FOLD_TILE) {  // guards against an unsorted caller array
          const uint32_t old = atomicExch(&head[pos], (uint32_t)j);
          meta[j] = (old & 0xFFFFu) | ((uint32_t)ep[q] << 16);
          if (old == ~0u) hitl[atomicAdd(&s_nhit, 1u)] = (uint16_t)pos;
        }
      }
    }
    for (int32_t j = FOLD_EQ * FOLD_THREADS + t; j < etot; j += FOLD_THREADS) {
      // payload of flattened entry j: binary search over pre[0..15] (pre[u] = etot > j for
      // u >= np), four dependent LDS reads instead of a read per payload
      int p = 0;
#pragma unroll
      for (int s = FOLD_MAXP / 2; s >= 1; s >>= 1) p += pre[p + s] <= j ? s : 0;
      const int64_t src = (int64_t)rng[p][0] + (j - pre[p]);
      const int64_t pos = (int64_t)s_idx[p][src] - tlo;
      ev[j] = s_val[p][src];
      if (pos >= 0 && pos < FOLD_TILE) {
        const uint32_t old = atomicExch(&head[pos], (uint32_t)j);
        meta[j] = (old & 0xFFFFu) | ((uint32_t)p << 16);
        if (old == ~0u) hitl[atomicAdd(&s_nhit, 1u)] = (uint16_t)pos;
      }
    }
    __syncthreads();
    FSTAMP(2);
    // A) base fold of this thread's elements; remember which of them carry hits
    uint32_t hitbits = 0;
#pragma unroll
    for (int q = 0; q < FOLD_GROUPS; ++q) {
      const uint4 h4 = *reinterpret_cast<const uint4*>(&head[q * 4 * FOLD_THREADS + t * 4]);
      hitbits |= ((h4.x != ~0u) ? 1u : 0u) << (4 * q);
      hitbits |= ((h4.y != ~0u) ? 1u : 0u) << (4 * q + 1);
      hitbits |= ((h4.z != ~0u) ? 1u : 0u) << (4 * q + 2);
      hitbits |= ((h4.w != ~0u) ? 1u : 0u) << (4 * q + 3);
    }
    {
      typedef float f2 __attribute__((ext_vector_type(2)));
      f2 b2[2 * FOLD_GROUPS], a2[2 * FOLD_GROUPS];
#pragma unroll
      for (int h = 0; h < 2 * FOLD_GROUPS; ++h) {
        b2[h] = a.zero_base ? f2{0.0f, 0.0f} : f2{L[2 * h], L[2 * h + 1]};
        a2[h] = f2{acc[2 * h], acc[2 * h + 1]};
      }
      if (a.replace_only) {
#pragma unroll
        for (int h = 0; h < 2 * FOLD_GROUPS; ++h) a2[h] = b2[h];
      } else {
        // weights from LDS (uniform reads); an unrolled loop over scalar weights spilled SGPRs
        // into VGPR lanes and cost occupancy
        int p0 = 0;
        if (a.first) {
          const float w = s_w[0];
          const f2 w2 = {w, w};
#pragma unroll
          for (int h = 0; h < 2 * FOLD_GROUPS; ++h) {
            const f2 term = b2[h] * w2;
            a2[h] = a.zero_base ? f2{0.0f, 0.0f} + term : term;
          }
          p0 = 1;
        }
        for (int p = p0; p < a.np; ++p) {
          const float w = s_w[p];
          const f2 w2 = {w, w};
#pragma unroll
          for (int h = 0; h < 2 * FOLD_GROUPS; ++h) a2[h] = a2[h] + b2[h] * w2;
        }
      }
#pragma unroll
      for (int h = 0; h < 2 * FOLD_GROUPS; ++h) {
        acc[2 * h] = a2[h].x;
        acc[2 * h + 1] = a2[h].y;
      }
    }
    // L is dead from here on (B and add_self read the LDS copy lv): the next tile's local
    // values load behind the hit fold and the stores
    if (tile + gridDim.x < a.ntiles) {
      load_local(tile + gridDim.x);
      l_ahead = true;
    }
    __syncthreads();  // every owner has read its hit flags before B overwrites head[]
    FSTAMP(3);
    // B) exact fold of the hit elements, two per thread with their chain walks interleaved
    //    (the walks are dependent LDS reads: one latency for both); the result replaces
    //    head[pos].  The usual one or two hits of an element fold branch-free; an element with
    //    three or more (rare) is refolded by the general chain walk.
    const uint32_t nhit = s_nhit;
    float wr[FOLD_MAXP];
#pragma unroll
    for (int p = 0; p < FOLD_MAXP; ++p) wr[p] = s_w[p];
    for (uint32_t s0 = t; s0 < nhit; s0 += 2 * FOLD_THREADS) {
      const uint32_t s1 = s0 + FOLD_THREADS;
      const bool two = s1 < nhit;
      int pos[2];
      pos[0] = hitl[s0];
      pos[1] = two ? hitl[s1] : pos[0];
      float bb[2], av[2], v1[2], v2[2];
      uint32_t p1[2], p2[2], more[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        bb[h] = a.zero_base ? 0.0f : lv[pos[h]];
        av[h] = a.first ? 0.0f : a.out[tlo + pos[h]];
        const uint32_t c1 = head[pos[h]] & 0xFFFFu;
        const uint32_t m1 = meta[c1];
        p1[h] = m1 >> 16;
        v1[h] = ev[c1];
        const uint32_t c2 = m1 & 0xFFFFu;
        const uint32_t m2 = meta[c2 != 0xFFFFu ? c2 : c1];
        p2[h] = c2 != 0xFFFFu ? (m2 >> 16) : 0xFFFFu;
        v2[h] = ev[c2 != 0xFFFFu ? c2 : c1];
        more[h] = c2 != 0xFFFFu ? (m2 & 0xFFFFu) : 0xFFFFu;
      }
#pragma unroll
      for (int p = 0; p < FOLD_MAXP; ++p) {
        if (p >= a.np) break;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float tv = ((uint32_t)p == p1[h]) ? v1[h] : (((uint32_t)p == p2[h]) ? v2[h] : bb[h]);
          fold_term(av[h], tv, wr[p], a.first && p == 0, a.replace_only, a.zero_base);
        }
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (more[h] != 0xFFFFu) {  // three or more hits (rare): walk the chain once into a row
          float acc = a.first ? 0.0f : a.out[tlo + pos[h]];
          const uint32_t row = atomicAdd(&s_pool_n, 1u);
          if (row < FOLD_POOL) {
            uint32_t mask = 0;
            for (uint32_t c = head[pos[h]] & 0xFFFFu; c != 0xFFFFu;) {
              const uint32_t m = meta[c];
              s_pool[row][m >> 16] = ev[c];
              mask |= 1u << (m >> 16);
              c = m & 0xFFFFu;
            }
            for (int p = 0; p < a.np; ++p) {
              const float tv = ((mask >> p) & 1u) ? s_pool[row][p] : bb[h];
              fold_term(acc, tv, wr[p], a.first && p == 0, a.replace_only, a.zero_base);
            }
          } else {  // the pool is full: a walk per payload
            for (int p = 0; p < a.np; ++p) {
              float tv = bb[h];
              for (uint32_t c = head[pos[h]] & 0xFFFFu; c != 0xFFFFu;) {
                const uint32_t m = meta[c];
                if ((m >> 16) == (uint32_t)p) {
                  tv = ev[c];
                  break;
                }
                c = m & 0xFFFFu;
              }
              fold_term(acc, tv, wr[p], a.first && p == 0, a.replace_only, a.zero_base);
            }
          }
          av[h] = acc;
        }
      }
      // every hit element's chain head is read above before any result overwrites it: each
      // element belongs to exactly one (thread, h), and only its own head[pos] is written
      head[pos[0]] = __float_as_uint(av[0]);
      if (two) head[pos[1]] = __float_as_uint(av[1]);
    }
    __syncthreads();
    FSTAMP(4);
    if (hitbits) {
#pragma unroll
      for (int q = 0; q < FOLD_GROUPS; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if ((hitbits >> (4 * q + e)) & 1u)
            acc[q * 4 + e] = __uint_as_float(head[q * 4 * FOLD_THREADS + t * 4 + e]);
    }
  } else {
  for (int j = t * 4; j < FOLD_TILE; j += 4 * FOLD_THREADS) *reinterpret_cast<uint32_t*>(&htag[j]) = 0xFFFFFFFFu;
  // entries of a payload past the preloaded ones (dense ranges, e.g. JWINS alpha 0.1-0.4):
  // the next payload's first FOLD_NB per thread are loaded while the current payload folds
  int32_t nbi[FOLD_NB];
  float nbv[FOLD_NB];
  auto prefetch = [&](int pp) {
#pragma unroll
    for (int u = 0; u < FOLD_NB; ++u) nbi[u] = -1;
    if (pp < a.np && !((a.dense_mask >> pp) & 1u)) {
      const int64_t first = (int64_t)FOLD_EQ * FOLD_THREADS - pre[pp];
      const int64_t j0 = rng[pp][0] + (first > 0 ? first : 0) + t;
      const int64_t e = rng[pp][1];
#pragma unroll
      for (int u = 0; u < FOLD_NB; ++u) {
        const int64_t j = j0 + (int64_t)u * FOLD_THREADS;
        if (j < e) {
          nbi[u] = s_idx[pp][j];
          nbv[u] = s_val[pp][j];
        }
      }
    }
  };
  prefetch(0);
  for (int p = 0; p < a.np; ++p) {
    const FoldPayload& P = a.p[p];
    __syncthreads();  // previous payload's reads of hv/htag done
    if (P.idx) {
#pragma unroll
      for (int q = 0; q < FOLD_EQ; ++q) {
        if (ep[q] == p) {
          const int64_t pos = (int64_t)ei[q] - tlo;
          if (pos >= 0 && pos < FOLD_TILE) {  // guards against an unsorted caller array
            hv[pos] = evl[q];
            htag[pos] = (uint8_t)p;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < FOLD_NB; ++u) {
        const int64_t pos = (int64_t)nbi[u] - tlo;
        if (pos >= 0 && pos < FOLD_TILE) {
          hv[pos] = nbv[u];
          htag[pos] = (uint8_t)p;
        }
      }
      // entries past the preloaded and prefetched ones: loaded here
      const int64_t b = rng[p][0], e = rng[p][1];
      const int64_t first = (int64_t)FOLD_EQ * FOLD_THREADS - pre[p];  // relative to b
      for (int64_t j = b + (first > 0 ? first : 0) + (int64_t)FOLD_NB * FOLD_THREADS + t; j < e;
           j += FOLD_THREADS) {
        const int64_t pos = (int64_t)P.idx[j] - tlo;
        if (pos >= 0 && pos < FOLD_TILE) {
          hv[pos] = P.val[j];
          htag[pos] = (uint8_t)p;
        }
      }
    }
    __syncthreads();
    prefetch(p + 1);
    const float w = P.w;
#pragma unroll
    for (int q = 0; q < FOLD_GROUPS; ++q) {
      const int j0 = q * 4 * FOLD_THREADS + t * 4;
      const int64_t i0 = tlo + j0;
      float tv[4];
      if (P.idx) {
        const float4 h4 = *reinterpret_cast<const float4*>(&hv[j0]);
        const uint32_t g4 = *reinterpret_cast<const uint32_t*>(&htag[j0]);
        const float hh[4] = {h4.x, h4.y, h4.z, h4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e)
          tv[e] = (((g4 >> (8 * e)) & 0xFFu) == (uint32_t)p) ? hh[e]
                                                               : (a.zero_base ? 0.0f : L[q * 4 + e]);
      } else {
        if (VEC && i0 + 3 < thi) {
          float4 v = *reinterpret_cast<const float4*>(P.val + i0);
          tv[0] = v.x; tv[1] = v.y; tv[2] = v.z; tv[3] = v.w;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) tv[e] = (i0 + e < thi) ? P.val[i0 + e] : 0.0f;
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (a.replace_only) {
          acc[q * 4 + e] = tv[e];
        } else {
          const float term = tv[e] * w;
          acc[q * 4 + e] = (a.first && p == 0) ? (a.zero_base ? 0.0f + term : term)
                                               : acc[q * 4 + e] + term;
        }
      }
    }
  }
  }  // phase path
  if (a.add_self) {
    if (l_ahead) {  // hit-chain path: this tile's local values from the LDS copy
      const float* lv = reinterpret_cast<const float*>(lds_raw) + FOLD_TILE + 2 * FOLD_CAP;
#pragma unroll
      for (int q = 0; q < FOLD_GROUPS; ++q) {
        const float4 v = *reinterpret_cast<const float4*>(&lv[q * 4 * FOLD_THREADS + t * 4]);
        acc[q * 4 + 0] = acc[q * 4 + 0] + v.x * a.w_self;
        acc[q * 4 + 1] = acc[q * 4 + 1] + v.y * a.w_self;
        acc[q * 4 + 2] = acc[q * 4 + 2] + v.z * a.w_self;
        acc[q * 4 + 3] = acc[q * 4 + 3] + v.w * a.w_self;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4 * FOLD_GROUPS; ++e) acc[e] = acc[e] + L[e] * a.w_self;
    }
  }
#pragma unroll
  for (int q = 0; q < FOLD_GROUPS; ++q) {
    const int64_t i0 = tlo + q * 4 * FOLD_THREADS + t * 4;
    if (VEC && i0 + 3 < thi) {
      const float4 r4 = make_float4(acc[q * 4 + 0], acc[q * 4 + 1], acc[q * 4 + 2], acc[q * 4 + 3]);
      *reinterpret_cast<float4*>(a.out + i0) = r4;
      // in place over local: every local read of this tile happened before (registers / LDS)
      if (a.out2) *reinterpret_cast<float4*>(a.out2 + i0) = r4;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (i0 + e < thi) {
          a.out[i0 + e] = acc[q * 4 + e];
          if (a.out2) a.out2[i0 + e] = acc[q * 4 + e];
        }
    }
  }
  if (!l_ahead && tile + gridDim.x < a.ntiles) load_local(tile + gridDim.x);
  __syncthreads();  // the next tile reuses rng / pre / the LDS tile
  FSTAMP(5);
  }  // tile loop
}

// ------------------------------------------------------------------------------------------------
// Slotted fold for dense all-sparse groups (JWINS alpha 0.1-0.4: thousands of entries per tile).
// The phase path pays a global load latency per payload (the next payload's entries arrive while
// only a short fold runs) and two barriers per payload.  Here every entry of the tile (up to
// FG_CAP per round) is loaded at tile start, into registers, and the payloads are folded
// FG_SLOTS at a time: each payload of a phase scatters into its own LDS value tile with a hit bit,
// then every thread folds its 8 elements over the phase's payloads in the reference's order
//   t = hit ? value : local;  total = (p == 0) ? t*w : total + t*w
// Hit flags are one byte per element (bit s: slot s hit), so the entries of a payload, sorted and
// spread over consecutive lanes, rarely collide in an LDS atomic; each thread clears its own
// elements' flags right after folding them, so a phase costs two barriers and no global round
// trip.
constexpr int FG_SLOTS = 4;                    // payloads per phase
constexpr int FG_CAP = 6144;                   // entries held per round (>= one payload's 4096)
constexpr int FG_EPT = FG_CAP / FOLD_THREADS;  // per thread
#ifndef DPZ_FG_HALVES
#define DPZ_FG_HALVES 2
#endif
constexpr int FG_HALVES = DPZ_FG_HALVES;  // entry load batches per round (register pressure)
static_assert(FG_CAP >= FOLD_TILE && FOLD_TILE <= 65536, "a round holds one payload's tile");
static_assert(FG_SLOTS <= 8, "slot flags are the bits of one byte per element");
#ifndef DPZ_FOLD_GROUP_MIN
#define DPZ_FOLD_GROUP_MIN 1536
#endif
constexpr int64_t FOLD_GROUP_MIN = DPZ_FOLD_GROUP_MIN;  // average entries per tile

template <bool VEC>
__global__ void __launch_bounds__(FOLD_THREADS, 4) fold_group_kernel(FoldArgs a) {
  __shared__ __attribute__((aligned(16))) float hv[FG_SLOTS][FOLD_TILE];
  __shared__ uint32_t hf[FOLD_TILE / 4];  // hit flags: byte e of word w = element 4w + e
  __shared__ int32_t rng[FOLD_MAXP][2];
  __shared__ int32_t pre[FOLD_MAXP + 1];
  __shared__ const __attribute__((address_space(1))) int32_t* s_idx[FOLD_MAXP];  // as_global
  __shared__ const __attribute__((address_space(1))) float* s_val[FOLD_MAXP];
  __shared__ float s_w[FOLD_MAXP];
  const int t = threadIdx.x;
  if (t == 0) {
    for (int p = 0; p < a.np; ++p) {
      s_idx[p] = as_global(a.p[p].idx);
      s_val[p] = as_global(a.p[p].val);
      s_w[p] = a.p[p].w;
    }
  }
#pragma unroll
  for (int q = 0; q < FOLD_GROUPS; ++q) hf[q * FOLD_THREADS + t] = 0;
  int32_t nr0 = 0, nr1 = 0;
  const bool rng_lane = t < a.np;
  if (rng_lane && (int64_t)blockIdx.x < a.ntiles) {
    const int32_t* st = a.starts + (int64_t)t * (a.ntiles + 1);
    nr0 = st[blockIdx.x];
    nr1 = st[blockIdx.x + 1];
  }
  float L[4 * FOLD_GROUPS];
  auto load_local = [&](int64_t tl) {
    const int64_t lo_ = tl * FOLD_TILE;
    const int64_t hi_ = (lo_ + FOLD_TILE < a.n) ? lo_ + FOLD_TILE : a.n;
#pragma unroll
    for (int q = 0; q < FOLD_GROUPS; ++q) {
      const int64_t i0 = lo_ + q * 4 * FOLD_THREADS + t * 4;
      if (VEC && i0 + 3 < hi_) {
        float4 v = *reinterpret_cast<const float4*>(a.local + i0);
        L[q * 4 + 0] = v.x; L[q * 4 + 1] = v.y; L[q * 4 + 2] = v.z; L[q * 4 + 3] = v.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) L[q * 4 + e] = i0 + e < hi_ ? a.local[i0 + e] : 0.0f;
      }
    }
  };
  if ((int64_t)blockIdx.x < a.ntiles) load_local(blockIdx.x);
  for (int64_t tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
    const int64_t tlo = tile * FOLD_TILE;
    const int64_t thi = (tlo + FOLD_TILE < a.n) ? tlo + FOLD_TILE : a.n;
    if (t < 64) {
      const int32_t c = (t < a.np && nr1 > nr0) ? nr1 - nr0 : 0;
      if (t < a.np) {
        rng[t][0] = nr0;
        rng[t][1] = nr1;
      }
      int32_t incl = c;
#pragma unroll
      for (int d = 1; d < FOLD_MAXP; d <<= 1) {
        const int32_t v = __shfl_up(incl, d, 64);
        if (t >= d) incl += v;
      }
      if (t < FOLD_MAXP) pre[t + 1] = incl;
      if (t == 0) pre[0] = 0;
    }
    if (rng_lane && tile + gridDim.x < a.ntiles) {
      const int32_t* st = a.starts + (int64_t)t * (a.ntiles + 1);
      nr0 = st[tile + gridDim.x];
      nr1 = st[tile + gridDim.x + 1];
    }
    typedef float f2v __attribute__((ext_vector_type(2)));
    f2v acc2[2 * FOLD_GROUPS];  // this thread's 8 running totals as packed pairs
    float base[4 * FOLD_GROUPS];  // a payload's value off its entries: local, or 0 (zero base)
#pragma unroll
    for (int e = 0; e < 4 * FOLD_GROUPS; ++e) base[e] = a.zero_base ? 0.0f : L[e];
#pragma unroll
    for (int h = 0; h < 2 * FOLD_GROUPS; ++h) acc2[h] = f2v{0.0f, 0.0f};
    if (!a.first) {
#pragma unroll
      for (int q = 0; q < FOLD_GROUPS; ++q) {
        const int64_t i0 = tlo + q * 4 * FOLD_THREADS + t * 4;
        float o[4];
        if (VEC && i0 + 3 < thi) {
          const float4 v = *reinterpret_cast<const float4*>(a.out + i0);
          o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = i0 + e < thi ? a.out[i0 + e] : 0.0f;
        }
        acc2[2 * q] = f2v{o[0], o[1]};
        acc2[2 * q + 1] = f2v{o[2], o[3]};
      }
    }
    __syncthreads();  // rng / pre visible; the previous tile's last phase is done
    for (int pa = 0; pa < a.np;) {
      // the round: payloads [pa, pb) whose entries of this tile fit FG_CAP (at least one)
      int pb = pa + 1;
      while (pb < a.np && pre[pb + 1] - pre[pa] <= FG_CAP) ++pb;
      const int32_t j0 = pre[pa], jn = pre[pb] - pre[pa];
      // entry u of this thread: ei = (position in the tile | payload << 16) or ~0 (absent /
      // outside the tile: an invalid payload cannot write out of bounds), ev = its value.
      // Loaded in FG_HALVES batches (fewer address registers live at once).
      uint32_t ei[FG_EPT];
      float ev[FG_EPT];
#pragma unroll
      for (int h = 0; h < FG_HALVES; ++h) {
        constexpr int HU = FG_EPT / FG_HALVES;
#pragma unroll
        for (int u = h * HU; u < (h + 1) * HU; ++u) {
          const int32_t j = t + u * FOLD_THREADS;
          ei[u] = 0;
          ev[u] = 0.0f;
          if (j < jn) {
            const int32_t jj = j0 + j;
            int p = 0;
#pragma unroll
            for (int s = FOLD_MAXP / 2; s >= 1; s >>= 1) p += pre[p + s] <= jj ? s : 0;
            const int64_t src = (int64_t)rng[p][0] + (jj - pre[p]);
            ei[u] = (uint32_t)s_idx[p][src];
            ev[u] = s_val[p][src];
          }
        }
#pragma unroll
        for (int u = h * HU; u < (h + 1) * HU; ++u) {
          // the entry's payload again (4 LDS reads): cheaper than holding it in registers
          uint32_t p = 0;
          {
            const int32_t jj = j0 + t + u * FOLD_THREADS;
#pragma unroll
            for (int s = FOLD_MAXP / 2; s >= 1; s >>= 1) p += pre[p + s] <= jj ? s : 0;
          }
          const int64_t pos = (int64_t)(int32_t)ei[u] - tlo;
          const bool in = t + u * FOLD_THREADS < jn && pos >= 0 && pos < FOLD_TILE;
          ei[u] = in ? ((uint32_t)pos | (p << 16)) : ~0u;
        }
      }
      for (int pbase = pa; pbase < pb; pbase += FG_SLOTS) {
        const int ns = (pb - pbase) < FG_SLOTS ? (pb - pbase) : FG_SLOTS;
        // scatter this phase's payloads into their slots
#pragma unroll
        for (int u = 0; u < FG_EPT; ++u) {
          const uint32_t s = (ei[u] >> 16) - (uint32_t)pbase;  // ~0 entries: s is huge
          if (s < (uint32_t)ns) {
            const uint32_t pos = ei[u] & 0xFFFFu;
            hv[s][pos] = ev[u];
            atomicOr(&hf[pos >> 2], (1u << s) << (8u * (pos & 3u)));
          }
        }
        __syncthreads();
        // fold the phase's payloads (this thread's own elements: flag word q * 512 + t)
        uint32_t fw[FOLD_GROUPS];
#pragma unroll
        for (int q = 0; q < FOLD_GROUPS; ++q) {
          fw[q] = hf[q * FOLD_THREADS + t];
          hf[q * FOLD_THREADS + t] = 0;  // read: cleared for the next phase (no one else reads it)
        }
        // packed fp32 pairs (v_pk_mul / v_pk_add: two elements per instruction, no FMA); the
        // first term of a fresh total (payload 0) is peeled off the loop
        for (int s = 0; s < ns; ++s) {
          const int p = pbase + s;
          const float w = s_w[p];
          const f2v w2 = {w, w};
          const bool first_term = a.first && p == 0;
#pragma unroll
          for (int q = 0; q < FOLD_GROUPS; ++q) {
            const int jt = q * 4 * FOLD_THREADS + t * 4;
            const uint32_t f = fw[q] >> s;  // bit 8e: element e hit by slot s
            const float4 h4 = *reinterpret_cast<const float4*>(&hv[s][jt]);
            const f2v t01 = {(f & 0x1u) ? h4.x : base[q * 4 + 0], (f & 0x100u) ? h4.y : base[q * 4 + 1]};
            const f2v t23 = {(f & 0x10000u) ? h4.z : base[q * 4 + 2], (f & 0x1000000u) ? h4.w : base[q * 4 + 3]};
            if (first_term) {
              const f2v z = {0.0f, 0.0f};
              acc2[2 * q] = a.zero_base ? z + t01 * w2 : t01 * w2;
              acc2[2 * q + 1] = a.zero_base ? z + t23 * w2 : t23 * w2;
            } else {
              acc2[2 * q] = acc2[2 * q] + t01 * w2;
              acc2[2 * q + 1] = acc2[2 * q + 1] + t23 * w2;
            }
          }
        }
        __syncthreads();  // slots and flags free for the next phase
      }
      pa = pb;
    }
    float acc[4 * FOLD_GROUPS];
#pragma unroll
    for (int h = 0; h < 2 * FOLD_GROUPS; ++h) {
      acc[2 * h] = acc2[h].x;
      acc[2 * h + 1] = acc2[h].y;
    }
    if (a.add_self) {
#pragma unroll
      for (int e = 0; e < 4 * FOLD_GROUPS; ++e) acc[e] = acc[e] + L[e] * a.w_self;
    }
#pragma unroll
    for (int q = 0; q < FOLD_GROUPS; ++q) {
      const int64_t i0 = tlo + q * 4 * FOLD_THREADS + t * 4;
      if (VEC && i0 + 3 < thi) {
        const float4 r4 =
            make_float4(acc[q * 4 + 0], acc[q * 4 + 1], acc[q * 4 + 2], acc[q * 4 + 3]);
        *reinterpret_cast<float4*>(a.out + i0) = r4;
        if (a.out2) *reinterpret_cast<float4*>(a.out2 + i0) = r4;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (i0 + e < thi) {
            a.out[i0 + e] = acc[q * 4 + e];
            if (a.out2) a.out2[i0 + e] = acc[q * 4 + e];
          }
      }
    }
    if (tile + gridDim.x < a.ntiles) load_local(tile + gridDim.x);
    // no barrier here: every read of rng / pre / the slots of this tile happened before the
    // last phase's barrier (a group with no payload has no phase: np == 0 never reaches here)
  }  // tile loop
}

// ---- the walk fold: one wave per contiguous element range, payload cursors, no barriers -----
// Every other fold kernel needs the tile-offsets pre-pass (fold_offsets_kernel reads every
// payload index once more: 35-100 us of 25 M x 16 payloads at JWINS alphas) and block barriers
// per tile or per payload.  Here each wave owns a contiguous run of tiles of TE = 64 * EPL
// elements and walks every payload's sorted entries with a cursor:
//  * start: a 64-ary search (64 probes per step, one wave-wide load) finds each payload's first
//    entry of the wave's range: <= 6 dependent steps for any k, all payloads' probes in flight;
//  * per tile: a 64-entry window per payload (idx, val; one coalesced load each) is already in
//    registers; the entries inside the tile are its leading lanes (sorted), their count advances
//    the cursor, and the NEXT tile's windows, local values and dense payload values are issued
//    before this tile is folded;
//  * payload by payload, in the reference's order, the window's lanes write their values with a
//    (tile, payload) tag into the wave's own LDS row, and every lane folds its EPL elements
//      t = (tag == mine) ? value : local;  total = t_0*w_0 (+0 first with a zero base);
//      total += t_p*w_p;  total += w_self * local
//    (no block barrier: the row is the wave's own, LDS ops of one wave run in order).
// A window whose 64 entries all fall inside the tile (dense tiles) is followed by synchronous
// extra windows (correct, slower); EPL is chosen so a tile holds ~52 entries or fewer per
// payload on average (launch_walk).  Invalid payloads (unsorted / out of range) cannot write out
// of bounds.
constexpr int FW_WAVES = 4;  // waves per block (256 threads)
// fold_walk_kernel's register bound (blocks per CU = waves per SIMD): the walk hides its window
// loads by occupancy (measured on MI355X, 3 payloads x alpha 0.4 at 128-element tiles: 125 -> 111
// us at 8 waves / SIMD).  The 4-group kernel is left unbounded: bounding it to 5 waves at
// 512-element tiles measured slower (16 x 0.1: 233 vs 222 us, profiles/r03_s2_fold_occ_ab.json).
#define FW_MINB_1(EPL) ((EPL) >= 16 ? 4 : ((EPL) >= 8 ? 5 : ((EPL) >= 4 ? 7 : 8)))

template <int EPL>
struct FwV {
  float v[EPL];
};

// A lane's EPL elements of a tile: contiguous for EPL <= 4; for EPL = 4C > 4, chunk c holds the
// lane's 4 elements at 256 c + 4 lane (every float4 wave-instruction reads 1 KB contiguous).
template <int EPL>
__device__ __forceinline__ int fw_elem(int lane, int e) {
  return EPL <= 4 ? lane * EPL + e : 256 * (e >> 2) + 4 * lane + (e & 3);
}

// Loads are branch-free (addresses clamped into [0, n); results past n are never stored), so
// the compiler counts them and waits only for the tile it folds, never for the next tile's loads
// in flight (a load under a branch makes it wait for everything: vmcnt(0)).  VEC kernels run
// when the operands are 16-byte aligned and n >= 1024: a vector group reaching past n is clamped
// to the last whole aligned group, and the ragged last tile reloads its values element-wise
// (sym2 level-4 coefficient arrays, M = 25,000,009 at C3, are not a multiple of 4).
template <bool VEC, int EPL>
__device__ __forceinline__ FwV<EPL> fw_load(const float* p, int64_t tlo, int lane, int64_t n) {
  FwV<EPL> r;
  if constexpr (VEC && EPL >= 4) {
    const int64_t last = (n & ~int64_t(3)) - 4;  // the last whole float4 group inside [0, n)
#pragma unroll
    for (int c = 0; c < EPL / 4; ++c) {
      const int64_t i0 = tlo + fw_elem<EPL>(lane, 4 * c);
      const int64_t q = i0 + 4 <= n ? i0 : last;
      const float4 v = *reinterpret_cast<const float4*>(p + q);
      r.v[4 * c] = v.x; r.v[4 * c + 1] = v.y; r.v[4 * c + 2] = v.z; r.v[4 * c + 3] = v.w;
    }
    return r;
  } else if constexpr (VEC && EPL == 2) {
    const int64_t i0 = tlo + 2 * lane;
    const int64_t q = i0 + 2 <= n ? i0 : (n & ~int64_t(1)) - 2;
    const float2 v = *reinterpret_cast<const float2*>(p + q);
    r.v[0] = v.x; r.v[1] = v.y;
    return r;
  }
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const int64_t i = tlo + fw_elem<EPL>(lane, e);
    r.v[e] = p[i < n ? i : n - 1];
  }
  return r;
}

// GUARD: the ragged last tile (elements past n are not stored).  NTS: non-temporal stores — the
// few-payload walk's output is a model that no later kernel of the step re-reads (same-box A/B on
// MI355X: C2 product path 72.0 -> 65.1 us, 64 MiB 91.0 -> 80.6 us, C4 round 5.72 -> 5.49 ms);
// the 16-payload JWINS fold keeps plain stores (its output feeds the IDWT right after)
template <bool VEC, int EPL, bool GUARD, bool NTS = false>
__device__ __forceinline__ void fw_store(float* p, int64_t tlo, int lane, int64_t n,
                                         const float (&r)[EPL]) {
  if constexpr (VEC && EPL >= 4) {
#pragma unroll
    for (int c = 0; c < EPL / 4; ++c) {
      const int64_t i0 = tlo + fw_elem<EPL>(lane, 4 * c);
      if (!GUARD || i0 + 4 <= n) {
        typedef float v4f __attribute__((ext_vector_type(4)));
        const v4f v = {r[4 * c], r[4 * c + 1], r[4 * c + 2], r[4 * c + 3]};
        if (NTS) __builtin_nontemporal_store(v, reinterpret_cast<v4f*>(p + i0));
        else *reinterpret_cast<v4f*>(p + i0) = v;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (i0 + e < n) p[i0 + e] = r[4 * c + e];
      }
    }
    return;
  } else if constexpr (VEC && EPL == 2) {
    const int64_t i0 = tlo + 2 * lane;
    if (!GUARD || i0 + 2 <= n) {
      *reinterpret_cast<float2*>(p + i0) = make_float2(r[0], r[1]);
    } else if (i0 < n) {
      p[i0] = r[0];
    }
    return;
  }
#pragma unroll
  for (int e = 0; e < EPL; ++e) {
    const int64_t i = tlo + fw_elem<EPL>(lane, e);
    if (!GUARD || i < n) p[i] = r[e];
  }
}

// the leading lanes whose index lies below `hi` (a sorted window): 0..64
__device__ __forceinline__ int fw_lead(bool in) {
  const uint64_t b = __ballot(in);
  return ~b == 0 ? 64 : (int)__builtin_ctzll(~b);
}

__device__ __forceinline__ int32_t fw_uni(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// lower_bound(idx_p, e0) of every payload p < np (np <= NSX) as lane p's value: 64-ary searches
// (one wave-wide probe load per step) run in LOCK STEP over the payloads, so each round's np probe
// loads are in flight together and a wave's start costs ~log64(k) dependent round trips, not np
// times that (16 payloads at k = 2.5 M: 4 rounds instead of 64 dependent loads).  Probe loads are
// branch-free (an idle payload re-reads a valid word: entry 0 of `dflt`) so the compiler waits once
// per round.  idx_of(p) / k_of(p) take compile-time p.
template <int NSX, class IdxOf, class KOf, class E0Of>
__device__ __forceinline__ int32_t fw_lower_bounds_t(int np, E0Of e0_of, int lane, IdxOf idx_of,
                                                     KOf k_of, const int32_t* dflt) {
  int32_t slo[NSX], shi[NSX];
#pragma unroll
  for (int p = 0; p < NSX; ++p) {
    slo[p] = 0;
    shi[p] = p < np ? k_of(p) : 0;
  }
  for (;;) {
    int32_t xv[NSX], st[NSX];
    bool act = false;
#pragma unroll
    for (int p = 0; p < NSX; ++p) {
      const bool on = shi[p] > slo[p];
      act |= on;
      const int32_t len = shi[p] - slo[p];
      st[p] = on ? (len <= 64 ? 1 : (len + 63) / 64) : 0;
      const int64_t q = (int64_t)slo[p] + (int64_t)lane * st[p];
      const bool ok = on && q < shi[p];
      const auto* ip = as_global(on ? idx_of(p) : dflt);
      xv[p] = ip[ok ? q : (on ? (int64_t)slo[p] : 0)];
    }
    if (!act) break;
#pragma unroll
    for (int p = 0; p < NSX; ++p) {
      if (st[p] == 0) continue;  // uniform
      const int64_t q = (int64_t)slo[p] + (int64_t)lane * st[p];
      const int32_t c = (int32_t)__popcll(__ballot(q < shi[p] && xv[p] < e0_of(p)));  // a prefix
      if (st[p] == 1) {
        slo[p] += c;
        shi[p] = slo[p];
      } else {
        const int32_t nlo = c > 0 ? slo[p] + (c - 1) * st[p] + 1 : slo[p];
        const int64_t nhi = (int64_t)slo[p] + (int64_t)c * st[p];
        shi[p] = nhi < shi[p] ? (int32_t)nhi : shi[p];
        slo[p] = nlo;
      }
    }
  }
  int32_t cur = 0;
#pragma unroll
  for (int p = 0; p < NSX; ++p) cur = lane == p ? slo[p] : cur;
  return cur;
}

// every search of the same target e0
template <int NSX, class IdxOf, class KOf>
__device__ __forceinline__ int32_t fw_lower_bounds(int np, int32_t e0, int lane, IdxOf idx_of,
                                                   KOf k_of, const int32_t* dflt) {
  return fw_lower_bounds_t<NSX>(np, [e0](int) { return e0; }, lane, idx_of, k_of, dflt);
}

// Walk-kernel start, compile-time switches (A/B variants: tools/diag/build_variant.sh):
// *_LOCKSTEP 1: the payloads' cursor searches in lock step (fw_lower_bounds); 0: one payload after
// the other.  *_L_FIRST 1: the first tile's local values issued before the search.  WALK4: the
// 1..4-payload kernel (a node's few neighbours: C4 rounds, the plugins), WALKG: the 5..16-payload
// groups kernel (C3).  Measured on MI355X (same box, tools/diag/c4_round_ab.py, 96-node C4 round
// on 3 streams): the fold leg 3.33 ms with lock step + local first, 3.14 sequential + local
// first, 3.42 lock step + local after, 3.00 sequential + local after — under three concurrent
// codecs the lock-step probes (and locals issued ahead of them) delay every wave's first window.
// The 16-payload groups kernel (C3 shape, tools/diag/fold_time.py) is no faster with them either
// (alpha 0.02: 128.7 vs 122.1 us, 0.1: 171.1 vs 170.2, 0.2: 261.4 vs 255.2), so both kernels
// search one payload after the other; fw_lower_bounds serves the patch decode.
// DPZ_MERGE_HIT2 1 (A/B variant, round 6): the merge fold's hit elements two per lane at a time
// (two independent chains).  Measured on MI355X (tools/diag/merge_keep_ab.sh with lib_keep =
// this switch, profiles/r06_merge_hit2_ab.jsonl): C3 16 x 0.01 105.1-105.6 -> 110.4-111.1 us,
// 16 x 0.005 88 -> 106-107 — the second chain's loads and selects cost more than the overlap
// gains at 4 waves per SIMD; off.
#ifndef DPZ_MERGE_HIT2
#define DPZ_MERGE_HIT2 0
#endif
#ifndef DPZ_WALK4_LOCKSTEP
#define DPZ_WALK4_LOCKSTEP 0
#endif
#ifndef DPZ_WALK4_L_FIRST
#define DPZ_WALK4_L_FIRST 0
#endif
#ifndef DPZ_WALKG_LOCKSTEP
#define DPZ_WALKG_LOCKSTEP 0
#endif
#ifndef DPZ_WALKG_L_FIRST
#define DPZ_WALKG_L_FIRST 0
#endif
template <int NSX, bool LOCK, class IdxOf, class KOf>
__device__ __forceinline__ int32_t fw_start_cursors(int np, int32_t e0, int lane, IdxOf idx_of,
                                                    KOf k_of, const int32_t* dflt) {
  if (LOCK) return fw_lower_bounds<NSX>(np, e0, lane, idx_of, k_of, dflt);
  int32_t curv = 0;
#pragma unroll
  for (int p = 0; p < NSX; ++p) {
    if (p >= np) break;
    const int32_t* ip = idx_of(p);
    int32_t lo = 0, hi = k_of(p);
    while (hi > lo) {
      const int32_t len = hi - lo;
      const int32_t stride = len <= 64 ? 1 : (len + 63) / 64;
      const int64_t q = (int64_t)lo + (int64_t)lane * stride;
      const bool ok = q < hi;
      const int32_t x = ip[ok ? q : lo];
      const int32_t c = (int32_t)__popcll(__ballot(ok && x < e0));  // a prefix
      if (stride == 1) {
        lo += c;
        break;
      }
      const int32_t nlo = c > 0 ? lo + (c - 1) * stride + 1 : lo;
      const int64_t nhi = (int64_t)lo + (int64_t)c * stride;
      hi = nhi < hi ? (int32_t)nhi : hi;
      lo = nlo;
    }
    curv = lane == p ? lo : curv;
  }
  return curv;
}

// Sparse payloads only (dense ones take the classic kernels), a fresh total (a.first),
// n < 2^31 - 1024 (walk_ok), np <= NS.  NS payload slots, all compile-time: every slot's window
// of the NEXT tile is issued at the start of this tile (branch-free loads), so the loads are in
// flight while all of this tile's payloads fold.  NS = 4: the payloads' pointers, sizes, weights
// and cursors in scalar registers (a generic path holds them one per lane and reads them back
// with readlane; measured slower than fold_walk_groups_kernel at 16 payloads, which is used there).
// One wave's run of tiles [t0, t1) of one fold (fold_walk_kernel; fold_walk_batch_kernel runs
// several folds' runs back to back).  wv / wt: the wave's LDS row; seq: the wave's tile sequence
// number, carried across runs so a stale tag of an earlier run never matches.
template <bool VEC, int EPL, int NS, class FA>
__device__ __forceinline__ void fold_walk_run(const FA& a, int64_t t0, int64_t t1, float* wv,
                                              uint32_t* wt, int lane, uint32_t& seq) {
  constexpr bool ONE = NS <= 4;
  constexpr int TE = 64 * EPL;
  const int64_t n = a.n;
  const int np = a.np;
  const int lp = lane < np && lane < FOLD_MAXP ? lane : 0;
  const int32_t kl = lane < np ? (int32_t)a.p[lp].k : 0;
  const uint64_t ipl = ONE ? 0 : reinterpret_cast<uint64_t>(a.p[lp].idx);
  const uint64_t vpl = ONE ? 0 : reinterpret_cast<uint64_t>(a.p[lp].val);
  const float wl = ONE ? 0.0f : a.p[lp].w;
  auto rl64 = [](uint64_t v, int p) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, p);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), p);
    return ((uint64_t)hi << 32) | lo;
  };
  auto P_idx = [&](int p) {
    return ONE ? a.p[p].idx : reinterpret_cast<const int32_t*>(rl64(ipl, p));
  };
  auto P_val = [&](int p) {
    return ONE ? a.p[p].val : reinterpret_cast<const float*>(rl64(vpl, p));
  };
  auto P_k = [&](int p) { return ONE ? (int32_t)a.p[p].k : fw_uni(__builtin_amdgcn_readlane(kl, p)); };
  auto P_w = [&](int p) {
    return ONE ? a.p[p].w : __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wl), p));
  };
  // the first tile's local values are issued before the cursor search (independent of it)
  FwV<EPL> L, Ln;
  if (DPZ_WALK4_L_FIRST) L = fw_load<VEC, EPL>(a.local, t0 * TE, lane, n);
  // ---- start cursors: lower_bound(idx_p, t0 * TE) ----
  // lane p: payload p's cursor (the next window's first entry)
  int32_t curv = fw_start_cursors<NS, DPZ_WALK4_LOCKSTEP != 0>(
      np, (int32_t)(t0 * TE), lane, [&](int p) { return P_idx(p); },
      [&](int p) { return P_k(p); }, reinterpret_cast<const int32_t*>(a.local));
  if (!DPZ_WALK4_L_FIRST) L = fw_load<VEC, EPL>(a.local, t0 * TE, lane, n);
  int32_t cs[ONE ? NS : 1];
  if constexpr (ONE) {
#pragma unroll
    for (int p = 0; p < NS; ++p) cs[p] = fw_uni(__builtin_amdgcn_readlane(curv, p));
  }
  auto cur_of = [&](int p) {
    if constexpr (ONE) return cs[p];
    else return fw_uni(__builtin_amdgcn_readlane(curv, p));
  };
  auto set_cur = [&](int p, int32_t v) {
    if constexpr (ONE) cs[p] = fw_uni(v);
    else curv = lane == p ? v : curv;
  };
  // ---- one 64-entry window per slot: (idx, val) at cur + lane, branch-free loads of raw values
  // (lanes past k read entry 0 and are masked when the window is used) ----
  int32_t wi[NS], wn[NS];
  float wvv[NS], wvn[NS];
  auto load_window = [&](int p, int32_t& ix, float& vx, int32_t at) {
    const bool live = p < np;
    const int pc = live ? p : 0;
    const int32_t j = (live ? at : 0) + lane;
    const int32_t kp = P_k(pc);
    const int32_t k = live ? kp : 0;
    const int32_t jc = j < k ? j : 0;
    // an empty payload's arrays may be null: read a valid address instead (masked at use)
    const bool has = kp > 0;
    ix = (has ? P_idx(pc) : reinterpret_cast<const int32_t*>(a.local))[jc];
    vx = (has ? P_val(pc) : a.local)[jc];
  };
#pragma unroll
  for (int p = 0; p < NS; ++p) load_window(p, wi[p], wvv[p], cur_of(p));
  auto tile_body = [&](int64_t tile, auto guard) {
    constexpr bool GUARD = decltype(guard)::value;
    const int64_t tlo = tile * TE;
    const int32_t tlo32 = (int32_t)tlo, thi32 = tlo32 + TE;
    // the run's last tile issues no windows past it: they re-request this tile's entries (L2)
    const bool more = tile + 1 < t1;
    // the ragged last tile: its vector groups past the last whole one were clamped on load
    if constexpr (GUARD && VEC) L = fw_load<false, EPL>(a.local, tlo, lane, n);
    // every slot: this tile's window start and entry count (the leading lanes below thi); the
    // cursors move to the next tile's windows, which are issued now with the next local values
    int32_t c0[NS], cnt[NS];
#pragma unroll
    for (int p = 0; p < NS; ++p) {
      const bool live = p < np;
      c0[p] = live ? cur_of(p) : 0;
      const int32_t k = live ? P_k(p) : 0;
      cnt[p] = fw_lead(c0[p] + lane < k && wi[p] < thi32);
      if (live) set_cur(p, c0[p] + cnt[p]);
    }
#pragma unroll
    for (int p = 0; p < NS; ++p) load_window(p, wn[p], wvn[p], more ? cur_of(p) : c0[p]);
    // the next tile's local values; the run's last tile re-requests its own lines instead (L2
    // hits) — a load of the tile past the run fetched 1 / tpw more model bytes from HBM
    // (64 MiB, 3 payloads: 4 tiles per wave, PMC 97 MB fetched against 71 MB)
    Ln = fw_load<VEC, EPL>(a.local, tile + 1 < t1 ? tlo + TE : tlo, lane, n);
    float acc[EPL], base[EPL];
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      base[e] = a.zero_base ? 0.0f : L.v[e];
      acc[e] = 0.0f;
    }
#pragma unroll
    for (int p = 0; p < NS; ++p) {
      if (p >= np) break;
      const float w = P_w(p);
      const uint32_t tag = (seq << 4) | (uint32_t)p;
      {
        const uint32_t pos = (uint32_t)(wi[p] - tlo32);  // < TE: inside the tile
        if (lane < cnt[p] && pos < (uint32_t)TE) {
          wv[pos] = wvv[p];
          wt[pos] = tag;
        }
      }
      if (cnt[p] == 64) {  // a dense tile: this payload's further windows, synchronously
        const int32_t k = P_k(p);
        const int32_t* pi = P_idx(p);
        const float* pv = P_val(p);
        int32_t c = 64;
        for (int32_t j0 = c0[p] + 64;; j0 += 64) {
          const int32_t j = j0 + lane;
          const int32_t iv = j < k ? pi[j] : INT32_MAX;
          const int cc = fw_lead(iv < thi32);
          const uint32_t pos = (uint32_t)(iv - tlo32);
          if (lane < cc && pos < (uint32_t)TE) {
            wv[pos] = pv[j];
            wt[pos] = tag;
          }
          c += cc;
          if (cc < 64) break;
        }
        set_cur(p, c0[p] + c);
        load_window(p, wn[p], wvn[p], more ? cur_of(p) : c0[p]);  // this payload's next window moved
      }
      // the row is this wave's own and one wave's LDS instructions execute in order, so the
      // lanes' writes above are seen by the reads below with no wait; the scheduling barriers
      // only keep the compiler from moving LDS accesses across (no memory fence: a fence would
      // also wait for the next tile's loads in flight)
      __builtin_amdgcn_wave_barrier();
      uint32_t tg[EPL];
      float hv[EPL];
      if constexpr (EPL >= 4) {
#pragma unroll
        for (int c = 0; c < EPL / 4; ++c) {
          const int o = fw_elem<EPL>(lane, 4 * c);
          const uint4 t4 = *reinterpret_cast<const uint4*>(&wt[o]);
          const float4 h4 = *reinterpret_cast<const float4*>(&wv[o]);
          tg[4 * c] = t4.x; tg[4 * c + 1] = t4.y; tg[4 * c + 2] = t4.z; tg[4 * c + 3] = t4.w;
          hv[4 * c] = h4.x; hv[4 * c + 1] = h4.y; hv[4 * c + 2] = h4.z; hv[4 * c + 3] = h4.w;
        }
      } else {
#pragma unroll
        for (int e = 0; e < EPL; ++e) {
          tg[e] = wt[lane * EPL + e];
          hv[e] = wv[lane * EPL + e];
        }
      }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int e = 0; e < EPL; ++e) {
        const float tv = tg[e] == tag ? hv[e] : base[e];
        const float term = tv * w;
        acc[e] = p == 0 ? (a.zero_base ? 0.0f + term : term) : acc[e] + term;
      }
    }
    if (a.add_self) {
#pragma unroll
      for (int e = 0; e < EPL; ++e) acc[e] = acc[e] + L.v[e] * a.w_self;
    }
    fw_store<VEC, EPL, GUARD, true>(a.out, tlo, lane, n, acc);
    if (a.out2) fw_store<VEC, EPL, GUARD, true>(a.out2, tlo, lane, n, acc);
#pragma unroll
    for (int p = 0; p < NS; ++p) {
      wi[p] = wn[p];
      wvv[p] = wvn[p];
    }
    L = Ln;
    ++seq;
  };
  const int64_t tfull = n / TE;  // tiles wholly inside [0, n)
  const int64_t tf = t1 < tfull ? t1 : (tfull > t0 ? tfull : t0);
  for (int64_t tile = t0; tile < tf; ++tile) tile_body(tile, std::false_type{});
  if (tf < t1) tile_body(tf, std::true_type{});  // the global last tile, ragged
}

template <bool VEC, int EPL, int NS>
__global__ void __launch_bounds__(256, FW_MINB_1(EPL)) fold_walk_kernel(FoldArgs a, int64_t tpw) {
  constexpr int TE = 64 * EPL;
  __shared__ float s_val[FW_WAVES][TE];
  __shared__ uint32_t s_tag[FW_WAVES][TE];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float* wv = s_val[wid];
  uint32_t* wt = s_tag[wid];
#pragma unroll
  for (int e = 0; e < EPL; ++e) wt[lane + 64 * e] = 0xFFFFFFFFu;
  const int64_t ntl = (a.n + TE - 1) / TE;
  const int64_t gw = (int64_t)blockIdx.x * FW_WAVES + wid;
  const int64_t t0 = gw * tpw;
  const int64_t t1 = (t0 + tpw < ntl) ? t0 + tpw : ntl;
  if (t0 >= t1) return;  // no block barrier anywhere: a wave may leave alone
  uint32_t seq = 0;
  fold_walk_run<VEC, EPL, NS>(a, t0, t1, wv, wt, lane, seq);
}

// A node's plain Metro-Hastings walk fold of <= 4 sparse payloads (fold_walk_batch_kernel's
// kernel-argument table entry) and the view fold_walk_run reads it through.
struct FoldNode {
  const float* local;
  float* out;
  float* out2;
  int np;
  float w_self;
  FoldPayload p[4];
};
constexpr int FW_BATCH = 22;  // nodes per launch: the table stays within the 4 KB of arguments
struct FoldNodeBatch {
  FoldNode nd[FW_BATCH];
  int64_t n;
  int m;
  int add_self;
  // dpz_decode_average_batch_guarded: int32 words (the round's encode status words) that must
  // all be 0, or the launch writes nothing (nullptr: no guard)
  const int32_t* guard;
  int64_t guard_n;
};
static_assert(sizeof(FoldNodeBatch) <= 3584, "kernel arguments");
struct FoldNodeView {
  const float* local;
  float* out;
  float* out2;
  int64_t n;
  int np;
  int add_self;
  int zero_base;
  float w_self;
  const FoldPayload* p;
};

// ONE launch for the folds of up to FW_BATCH nodes of a gossip round (dpz_decode_average_batch:
// every node's fold a plain Metro-Hastings walk of <= 4 sparse payloads over the same n): the
// folds' tiles form one range [0, m * ntl) that the persistent grid's waves split into contiguous
// runs, a run crossing a node boundary continuing in the next node's fold.  One launch instead of
// m: the folds' start-up latencies (cursor searches, first windows) overlap and no launch drains
// alone (a full-GPU persistent grid per node serialises on a few streams).
template <bool VEC, int EPL>
__global__ void __launch_bounds__(256, FW_MINB_1(EPL)) fold_walk_batch_kernel(FoldNodeBatch b,
                                                                              int64_t tpw) {
  constexpr int TE = 64 * EPL;
  const int64_t ntl = (b.n + TE - 1) / TE;
  const int64_t m = b.m;
  __shared__ float s_val[FW_WAVES][TE];
  __shared__ uint32_t s_tag[FW_WAVES][TE];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float* wv = s_val[wid];
  uint32_t* wt = s_tag[wid];
#pragma unroll
  for (int e = 0; e < EPL; ++e) wt[lane + 64 * e] = 0xFFFFFFFFu;
  const int64_t gw = (int64_t)blockIdx.x * FW_WAVES + fw_uni(wid);
  if (b.guard) {  // a missed encode: no fold of this launch writes (the host re-runs the round)
    bool bad = false;
    for (int64_t i = lane; i < b.guard_n; i += 64) bad |= b.guard[i] != 0;
    if (__ballot(bad) != 0) return;  // every wave reads the same final words
  }
  int64_t g = gw * tpw;
  const int64_t gend = m * ntl;
  const int64_t g1 = g + tpw < gend ? g + tpw : gend;
  uint32_t seq = 0;
  while (g < g1) {
    const int64_t node = g / ntl;
    const int64_t lt0 = g - node * ntl;
    const int64_t lt1 = lt0 + (g1 - g) < ntl ? lt0 + (g1 - g) : ntl;
    const FoldNode& nd = b.nd[node];
    const FoldNodeView v{nd.local, nd.out, nd.out2, b.n, nd.np, b.add_self, 0, nd.w_self, nd.p};
    fold_walk_run<VEC, EPL, 4>(v, lt0, lt1, wv, wt, lane, seq);
    g += lt1 - lt0;
  }
}

constexpr int FW_G = 4;  // payloads per group: the windows of one group are in registers

// 5..16 sparse payloads (fold_walk_kernel's conditions otherwise).  The payloads are walked in
// groups of FW_G: the windows of the
// group being folded and of the next group (of this tile, or group 0 of the next tile) are in
// registers, so every window load is in flight while the group before it folds, with 16
// registers of windows whatever the payload count.  Cursors live one per lane (lane p: payload
// p) in one register.
template <bool VEC, int EPL, bool ONE, int DIST, bool W2>
__global__ void __launch_bounds__(256) fold_walk_groups_kernel(FoldArgs a, int64_t tpw) {
  constexpr int TE = 64 * EPL;
  __shared__ float s_val[FW_WAVES][TE];
  // tags (tile sequence << 4 | payload): 16-bit under DPZ_TAG16 (the sequence wraps every 4095
  // tiles, the row is cleared then), so a lane's read-back of 4 tags is one 8-byte LDS read
#ifdef DPZ_TAG16
  using tag_t = uint16_t;
  constexpr uint32_t SEQ_WRAP = 4095u;
#else
  using tag_t = uint32_t;
  constexpr uint32_t SEQ_WRAP = 0x0FFFFFFFu;
#endif
  __shared__ tag_t s_tag[FW_WAVES][TE];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float* wv = s_val[wid];
  tag_t* wt = s_tag[wid];
#pragma unroll
  for (int e = 0; e < EPL; ++e) wt[lane + 64 * e] = (tag_t)~0u;
  const int64_t n = a.n;
  const int64_t ntl = (n + TE - 1) / TE;
  const int64_t gw = (int64_t)blockIdx.x * FW_WAVES + wid;
  const int64_t t0 = gw * tpw;
  const int64_t t1 = (t0 + tpw < ntl) ? t0 + tpw : ntl;
  if (t0 >= t1) return;  // no block barrier anywhere: a wave may leave alone
  const int np = a.np;
  // ONE (np <= FW_G): one group, its payload numbers compile-time constants, so their
  // pointers / sizes / weights and cursors stay in scalar registers; otherwise the group loop is
  // dynamic and the cursors live one per lane (lane p: payload p) in one register
  const int ng = ONE ? 1 : (np + FW_G - 1) / FW_G;
  // CT: every payload number in the loop is a compile-time constant (ONE; DIST 3, whose four
  // groups are unrolled): the cursors in scalar registers (no readlane / writelane round trips)
  constexpr bool CT = ONE || DIST == 3;
  const int lp = lane < np && lane < FOLD_MAXP ? lane : 0;
  const int32_t kl = lane < np ? (int32_t)a.p[lp].k : 0;
  // !ONE: payload p's pointers and weight held by lane p, read back with readlane (no scalar
  // loads of the kernel arguments with a run-time payload number inside the loop)
  const uint64_t ipl = reinterpret_cast<uint64_t>(a.p[lp].idx);
  const uint64_t vpl = reinterpret_cast<uint64_t>(a.p[lp].val);
  const float wl = a.p[lp].w;
  auto rl64 = [](uint64_t v, int p) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, p);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), p);
    return ((uint64_t)hi << 32) | lo;
  };
  auto P_idx = [&](int p) {
    return ONE ? a.p[p].idx : reinterpret_cast<const int32_t*>(rl64(ipl, p));
  };
  auto P_val = [&](int p) {
    return ONE ? a.p[p].val : reinterpret_cast<const float*>(rl64(vpl, p));
  };
  auto P_k = [&](int p) { return ONE ? (int32_t)a.p[p].k : fw_uni(__builtin_amdgcn_readlane(kl, p)); };
  auto P_w = [&](int p) {
    return ONE ? a.p[p].w : __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wl), p));
  };
  static_assert(DIST == 1 || (DIST == 3 && !ONE), "DIST 3: four groups");
  int32_t cs[FOLD_MAXP];  // CT: the cursors (scalar registers)
  // the first tile's local values are issued before the cursor search (independent of it)
  FwV<EPL> L, Ln;
  if (DPZ_WALKG_L_FIRST) L = fw_load<VEC, EPL>(a.local, t0 * TE, lane, n);
  // ---- start cursors: lower_bound(idx_p, t0 * TE), every payload in lock step ----
  int32_t curv = fw_start_cursors<FOLD_MAXP, DPZ_WALKG_LOCKSTEP != 0>(
      np, (int32_t)(t0 * TE), lane,
      [&](int p) { return reinterpret_cast<const int32_t*>(rl64(ipl, p)); },
      [&](int p) { return fw_uni(__builtin_amdgcn_readlane(kl, p)); },
      reinterpret_cast<const int32_t*>(a.local));
  if (!DPZ_WALKG_L_FIRST) L = fw_load<VEC, EPL>(a.local, t0 * TE, lane, n);
  if (CT) {
#pragma unroll
    for (int q = 0; q < (ONE ? FW_G : FOLD_MAXP); ++q) cs[q] = fw_uni(__builtin_amdgcn_readlane(curv, q));
  }
  auto cur_of = [&](int p) {
    return CT ? cs[ONE ? (p & (FW_G - 1)) : p] : fw_uni(__builtin_amdgcn_readlane(curv, p));
  };
  auto set_cur = [&](int p, int32_t v) {
    if (CT) cs[ONE ? (p & (FW_G - 1)) : p] = fw_uni(v);
    else curv = lane == p ? v : curv;
  };
  // ---- the windows of one group: (idx, val) at cur + lane, branch-free loads of raw values
  // (lanes past k read entry 0 and are masked when the window is used) ----
  // W2: 128-entry windows (entries cur + lane and cur + 64 + lane), so a tile of ~50 entries per
  // payload on average rarely overflows into the synchronous path (whose loads, the youngest in
  // flight, make the wave wait for every window load issued ahead: vmcnt(0))
  constexpr int NSL = DIST == 3 ? FW_G : 2;
  constexpr int NW2 = W2 ? NSL : 1;
  int32_t WI[NSL][FW_G], WI2[NW2][FW_G];
  float WV[NSL][FW_G], WV2[NW2][FW_G];
  auto load_group = [&](int g, int sl) {
#pragma unroll
    for (int q = 0; q < FW_G; ++q) {
      const int p = g * FW_G + q;
      const bool live = p < np;
      const int pc = live ? p : 0;
      const int32_t j = (live ? cur_of(pc) : 0) + lane;
      const int32_t kp = P_k(pc);
      const int32_t k = live ? kp : 0;
      const int32_t jc = j < k ? j : 0;
      // an empty payload's arrays may be null: read a valid address instead (masked at use)
      const bool has = kp > 0;
      const auto* ip = as_global(has ? P_idx(pc) : reinterpret_cast<const int32_t*>(a.local));
      const auto* vp = as_global(has ? P_val(pc) : a.local);
      WI[sl][q] = ip[jc];
      WV[sl][q] = vp[jc];
      if constexpr (W2) {
        const int32_t jc2 = j + 64 < k ? j + 64 : 0;
        WI2[sl][q] = ip[jc2];
        WV2[sl][q] = vp[jc2];
      }
    }
  };
  // DIST 1: the windows of the group being folded and of the next one (wi, wn);
  // DIST 3 (four groups, 13..16 payloads): all four groups' windows in registers, each group's
  // issued three groups ahead (into the slot the group before it just freed), so three groups'
  // loads are in flight while one folds
  if constexpr (DIST == 3) {
    load_group(0, 0);
    load_group(1, 1);
    load_group(2, 2);
  } else {
    load_group(0, 0);
  }
  uint32_t seq = 0;
  auto tile_body = [&](int64_t tile, auto guard) {
    constexpr bool GUARD = decltype(guard)::value;
    const int64_t tlo = tile * TE;
    const int32_t tlo32 = (int32_t)tlo, thi32 = tlo32 + TE;
    // the ragged last tile: its vector groups past the last whole one were clamped on load
    if constexpr (GUARD && VEC) L = fw_load<false, EPL>(a.local, tlo, lane, n);
    // the next tile's local values; the run's last tile re-requests its own lines instead (L2
    // hits) — a load of the tile past the run fetched 1 / tpw more model bytes from HBM
    // (64 MiB, 3 payloads: 4 tiles per wave, PMC 97 MB fetched against 71 MB)
    Ln = fw_load<VEC, EPL>(a.local, tile + 1 < t1 ? tlo + TE : tlo, lane, n);
    float acc[EPL], base[EPL];
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
      base[e] = a.zero_base ? 0.0f : L.v[e];
      acc[e] = 0.0f;
    }
    // one group: its windows (wi, wvv) are in registers; `issue` starts a later group's loads
    // once this group's cursors have advanced
    auto fold_group = [&](int g, int sl, auto issue) {
      const int32_t (&wi)[FW_G] = WI[sl];
      const float (&wvv)[FW_G] = WV[sl];
      // this group's window starts; the entries of the tile are the leading lanes below thi
      int32_t c0[FW_G], cnt[FW_G];
#pragma unroll
      for (int q = 0; q < FW_G; ++q) {
        const int p = g * FW_G + q;
        const bool live = p < np;
        c0[q] = live ? cur_of(p) : 0;
        const int32_t k = live ? P_k(p) : 0;
        cnt[q] = fw_lead(c0[q] + lane < k && wi[q] < thi32);
        if (W2 && cnt[q] == 64) cnt[q] += fw_lead(c0[q] + 64 + lane < k && WI2[W2 ? sl : 0][q] < thi32);
        // the next tile's window start of this payload (a full window is finished in its phase)
        if (live) set_cur(p, c0[q] + cnt[q]);
      }
      issue();
#pragma unroll
      for (int q = 0; q < FW_G; ++q) {
        const int p = g * FW_G + q;
        if (p >= np) break;
        const float w = P_w(p);
        const uint32_t tag = (seq << 4) | (uint32_t)p;
        {
          const uint32_t pos = (uint32_t)(wi[q] - tlo32);  // < TE: inside the tile
          if (lane < cnt[q] && pos < (uint32_t)TE) {
            wv[pos] = wvv[q];
            wt[pos] = (tag_t)tag;
          }
          if constexpr (W2) {
            const uint32_t pos2 = (uint32_t)(WI2[sl][q] - tlo32);
            if (lane + 64 < cnt[q] && pos2 < (uint32_t)TE) {
              wv[pos2] = WV2[sl][q];
              wt[pos2] = (tag_t)tag;
            }
          }
        }
        constexpr int WN = W2 ? 128 : 64;
        if (cnt[q] == WN) {  // a dense tile: this payload's further windows, synchronously
          const int32_t k = P_k(p);
          const int32_t* pi = P_idx(p);
          const float* pv = P_val(p);
          int32_t c = WN;
          for (int32_t j0 = c0[q] + WN;; j0 += 64) {
            const int32_t j = j0 + lane;
            const int32_t iv = j < k ? as_global(pi)[j] : INT32_MAX;
            const int cc = fw_lead(iv < thi32);
            const uint32_t pos = (uint32_t)(iv - tlo32);
            if (lane < cc && pos < (uint32_t)TE) {
              wv[pos] = as_global(pv)[j];
              wt[pos] = (tag_t)tag;
            }
            c += cc;
            if (cc < 64) break;
          }
          set_cur(p, c0[q] + c);
          // the next tile's window of this group moved (DIST 1, one group: already issued)
          if (DIST == 1 && ng == 1) load_group(0, 1);
        }
        // the row is this wave's own and one wave's LDS instructions execute in order, so the
        // lanes' writes above are seen by the reads below with no wait; the scheduling barriers
        // only keep the compiler from moving LDS accesses across (no memory fence: a fence
        // would also wait for the next windows in flight)
        __builtin_amdgcn_wave_barrier();
        uint32_t tg[EPL];
        float hv[EPL], tv[EPL];
        if constexpr (EPL >= 4) {
#pragma unroll
          for (int c = 0; c < EPL / 4; ++c) {
            const int o = fw_elem<EPL>(lane, 4 * c);
            if constexpr (sizeof(tag_t) == 2) {
              const uint2 t2 = *reinterpret_cast<const uint2*>(&wt[o]);
              tg[4 * c] = t2.x & 0xFFFFu; tg[4 * c + 1] = t2.x >> 16;
              tg[4 * c + 2] = t2.y & 0xFFFFu; tg[4 * c + 3] = t2.y >> 16;
            } else {
              const uint4 t4 = *reinterpret_cast<const uint4*>(&wt[o]);
              tg[4 * c] = t4.x; tg[4 * c + 1] = t4.y; tg[4 * c + 2] = t4.z; tg[4 * c + 3] = t4.w;
            }
            const float4 h4 = *reinterpret_cast<const float4*>(&wv[o]);
            hv[4 * c] = h4.x; hv[4 * c + 1] = h4.y; hv[4 * c + 2] = h4.z; hv[4 * c + 3] = h4.w;
          }
        } else {
#pragma unroll
          for (int e = 0; e < EPL; ++e) {
            tg[e] = wt[lane * EPL + e];
            hv[e] = wv[lane * EPL + e];
          }
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int e = 0; e < EPL; ++e) {
          tv[e] = tg[e] == tag ? hv[e] : base[e];
          const float term = tv[e] * w;
          acc[e] = p == 0 ? (a.zero_base ? 0.0f + term : term) : acc[e] + term;
        }
      }
    };
    if constexpr (DIST == 3) {
      // group g of this tile issues group g + 3: group 3 of this tile (g = 0), else group g - 1
      // of the next tile, into the slot group g - 1 freed
#pragma unroll
      for (int g = 0; g < FW_G; ++g) {
        fold_group(g, g, [&] {
          const int s3 = (g + 3) & (FW_G - 1);
          load_group(s3, s3);
        });
      }
    } else {
      for (int gg = 0; gg < ng; ++gg) {
        const int g = ONE ? 0 : gg;
        // the next group's windows (this tile's next group, or group 0 of the next tile)
        fold_group(g, 0, [&] { load_group(g + 1 < ng ? g + 1 : 0, 1); });
#pragma unroll
        for (int q = 0; q < FW_G; ++q) {
          WI[0][q] = WI[1][q];
          WV[0][q] = WV[1][q];
          if constexpr (W2) {
            WI2[0][q] = WI2[W2 ? 1 : 0][q];
            WV2[0][q] = WV2[W2 ? 1 : 0][q];
          }
        }
      }
    }
    if (a.add_self) {
#pragma unroll
      for (int e = 0; e < EPL; ++e) acc[e] = acc[e] + L.v[e] * a.w_self;
    }
    fw_store<VEC, EPL, GUARD>(a.out, tlo, lane, n, acc);
    if (a.out2) fw_store<VEC, EPL, GUARD>(a.out2, tlo, lane, n, acc);
    L = Ln;
    if (++seq == SEQ_WRAP) {  // tags restart: no stale tag of this row may match a new one
      seq = 0;
#pragma unroll
      for (int e = 0; e < EPL; ++e) wt[lane + 64 * e] = (tag_t)~0u;
    }
  };
  const int64_t tfull = n / TE;  // tiles wholly inside [0, n)
  const int64_t tf = t1 < tfull ? t1 : (tfull > t0 ? tfull : t0);
  for (int64_t tile = t0; tile < tf; ++tile) tile_body(tile, std::false_type{});
  if (tf < t1) tile_body(tf, std::true_type{});  // the global last tile, ragged
}

// blocks of the persistent fold grid: what the CUs hold at once (occupancy API)
template <bool VEC>
static unsigned fold_grid(int64_t ntiles, bool group = false) {
  static int slots[2] = {0, 0};
  int& sl = slots[group ? 1 : 0];
  if (sl == 0) {
    int dev = 0, cus = 256, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    const hipError_t e =
        group ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fold_group_kernel<VEC>, FOLD_THREADS, 0)
              : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fold_kernel<VEC>, FOLD_THREADS, 0);
    if (e != hipSuccess || per < 1) per = 1;
    sl = cus * per;
  }
  const int slots_now = sl;
  // DPZ_FOLD_BLOCKS=N caps the grid at N blocks (diagnostic build; 0 = the occupancy slots)
  const int64_t cap = DPZ_KNOB_INT(FOLD_BLOCKS, 0);
  const int64_t g = cap > 0 ? cap : slots_now;
  return (unsigned)(ntiles < g ? (ntiles > 0 ? ntiles : 1) : g);
}

static inline int64_t fold_ntiles(int64_t n) { return (n + FOLD_TILE - 1) / FOLD_TILE; }

// The walk fold's launch: EPL from the densest payload (~32 entries per payload per tile on
// average at dens <= 0.125: 256-element tiles; denser payloads 128-element tiles); a
// persistent grid of what the CUs hold, each wave a contiguous run of tiles.
template <bool VEC, int EPL, int NS, int DIST = 1, bool W2 = false>
static int launch_walk_t(const FoldArgs& fa, bool w2, hipStream_t st) {
  // 13..16 payloads (four groups): the groups kernel with windows issued three groups ahead
  // (DPZ_FOLD_DIST=1: one group ahead, A/B); w2: 128-entry windows
  if constexpr (NS > 4 && DIST == 1 && !W2) {
    const bool d3 = DPZ_KNOB_INT(FOLD_DIST, 3) != 1;
    if (d3 && (fa.np + FW_G - 1) / FW_G == FW_G)
      return w2 ? launch_walk_t<VEC, EPL, NS, 3, true>(fa, w2, st)
                : launch_walk_t<VEC, EPL, NS, 3, false>(fa, w2, st);
    if (w2) return launch_walk_t<VEC, EPL, NS, 1, true>(fa, w2, st);
  }
  static int per = 0, cus = 0;
  if (per == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    const void* kf = NS <= 4 ? reinterpret_cast<const void*>(fold_walk_kernel<VEC, EPL, 4>)
                             : reinterpret_cast<const void*>(fold_walk_groups_kernel<VEC, EPL, false, DIST, W2>);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kf, 256, 0) !=
            hipSuccess || per < 1)
      per = 1;
  }
  constexpr int TE = 64 * EPL;
  const int64_t ntl = (fa.n + TE - 1) / TE;
  int64_t blocks = (int64_t)cus * per;
  // DPZ_WALK_BLOCKS=N: the walk grid at N blocks (diagnostic build, A/B)
  if (DPZ_KNOB_INT(WALK_BLOCKS, 0) > 0) blocks = DPZ_KNOB_INT(WALK_BLOCKS, 0);
  const int64_t need = (ntl + FW_WAVES - 1) / FW_WAVES;
  if (blocks > need) blocks = need;
  if (blocks < 1) blocks = 1;
  const int64_t tpw = (ntl + blocks * FW_WAVES - 1) / (blocks * FW_WAVES);
  if constexpr (NS <= 4) {
    DPZ_TIMED(DPZ_KT_FOLD, st, fold_walk_kernel<VEC, EPL, NS><<<(unsigned)blocks, 256, 0, st>>>(fa, tpw));
  } else {
    DPZ_TIMED(DPZ_KT_FOLD, st,
              (fold_walk_groups_kernel<VEC, EPL, false, DIST, W2><<<(unsigned)blocks, 256, 0, st>>>(fa, tpw)));
  }
  return DPZ_OK;
}

static bool walk_ok(const FoldArgs& fa) {
  return !fa.replace_only && fa.first && fa.all_sparse && fa.np > 0 &&
         fa.n < (int64_t(1) << 31) - 1024;
}

template <int NS>
static int launch_walk_o(const FoldArgs& fa, bool vec, int epl, bool w2, hipStream_t st) {
  if (vec) {
    switch (epl) {
      case 16: return launch_walk_t<true, 16, NS>(fa, w2, st);
      case 8: return launch_walk_t<true, 8, NS>(fa, w2, st);
      case 4: return launch_walk_t<true, 4, NS>(fa, w2, st);
      default: return launch_walk_t<true, 2, NS>(fa, w2, st);
    }
  }
  switch (epl) {
    case 16: return launch_walk_t<false, 16, NS>(fa, w2, st);
    case 8: return launch_walk_t<false, 8, NS>(fa, w2, st);
    case 4: return launch_walk_t<false, 4, NS>(fa, w2, st);
    default: return launch_walk_t<false, 2, NS>(fa, w2, st);
  }
}

// The largest tile that holds about one window per payload on average (the densest payload,
// `dens`): fewer tiles mean fewer window loads and LDS passes per element, and an overflowing
// window is re-read synchronously.  Measured on MI355X (M = 25 M, profiles/r03_s3_walk_win_sweep.txt):
//   <= 4 payloads / 5..12: 64-entry windows, ~52 entries per tile or fewer (16 x 0.1 at
//     512-element tiles 215 us, 1024: 283, 256: 287; 3 x 0.1: 64 / 72 / 77 us);
//   13..16 payloads: 64-entry windows up to dens 0.055 (1024-element tiles), then 128-entry
//     windows: 1024-element tiles to 0.105, 512 to 0.21 (16 x 0.15: 297 -> 247 us, 16 x 0.2:
//     309 -> 266 us against 64-entry windows at 256-element tiles).
static int launch_walk(const FoldArgs& fa, bool vec, double dens, hipStream_t st) {
  const bool four = (fa.np + FW_G - 1) / FW_G == FW_G;
  int e = dens <= 0.055 ? 16 : (dens <= 0.105 ? 8 : (dens <= 0.21 ? 4 : 2));
  bool w2 = false;
  if (four && dens > 0.055 && dens <= 0.21) {
    w2 = true;
    e = dens <= 0.105 ? 16 : 8;
  }
  {  // forced tile / window sizes (diagnostic build)
    const int v = (int)DPZ_KNOB_INT(FOLD_WALK_EPL, 0);
    if (v == 16 || v == 8 || v == 4 || v == 2) e = v;
    if (DPZ_KNOB_STR(FOLD_WIN)) w2 = DPZ_KNOB_INT(FOLD_WIN, 64) == 128;
  }
  return fa.np <= 4 ? launch_walk_o<4>(fa, vec, e, false, st) : launch_walk_o<16>(fa, vec, e, w2, st);
}

// Replace-only decode of ONE sparse payload (reference PartialModel.py:257-303, T[idx] = params):
// one 256-thread block per chunk of RP_E payload entries (dpz_replace.h).
// Standalone replace: one wave per chunk of RP_E entries (~1,600 elements at 1 %), a grid of
// many short blocks (measured on MI355X: shorter than persistent waves walking the chunks with
// the next chunk's entries prefetched, and than 64-entry chunks per 256-thread block).
__global__ void __launch_bounds__(256) replace_kernel(ReplaceJob j) { replace_block(j, blockIdx.x); }

int launch_replace(const ReplaceJob& j, hipStream_t st) {
  if (j.c1 > j.c0)
    DPZ_TIMED(DPZ_KT_FOLD, st, replace_kernel<<<(unsigned)((j.c1 - j.c0 + 3) / 4), 256, 0, st>>>(j));
  return DPZ_OK;
}

// ---- the fold base on its own (dpz_topk_encode_foldbase off the pipelined filter) -------------
template <bool VEC>
__global__ void __launch_bounds__(256) fold_base_kernel(const float* __restrict__ x, int64_t n,
                                                        FoldBase fb, float* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  if (VEC) {
    const int64_t n4 = n >> 2;
    for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < n4; g += stride) {
      const float4 v = reinterpret_cast<const float4*>(x)[g];
      reinterpret_cast<float4*>(out)[g] = make_float4(fb.of(v.x), fb.of(v.y), fb.of(v.z), fb.of(v.w));
    }
    for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
      out[i] = fb.of(x[i]);
  } else {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) out[i] = fb.of(x[i]);
  }
}

int launch_fold_base(const float* x, int64_t n, const FoldBase& fb, float* out, hipStream_t st) {
  if (n <= 0) return DPZ_OK;
  const int64_t groups = (n + 3) / 4;
  unsigned nb = (unsigned)((groups + 255) / 256);
  if (nb > 4096) nb = 4096;
  if (aligned16(x) && aligned16(out))
    DPZ_TIMED(DPZ_KT_FOLD, st, fold_base_kernel<true><<<nb, 256, 0, st>>>(x, n, fb, out));
  else
    DPZ_TIMED(DPZ_KT_FOLD, st, fold_base_kernel<false><<<nb, 256, 0, st>>>(x, n, fb, out));
  return DPZ_OK;
}

// ---- DPZ_FOLD_BASE_READY: rewrite only the elements the payloads hit --------------------------
// out already holds the fold of every element's local value alone (FoldBase::of, written by the
// encoder's filter); an element hit by one or more payloads is folded here exactly, in the
// reference's order (payload terms in payload order, then the self term).  Block b owns the
// 4096-element tile b: its payload runs come from fold_offsets_kernel's tile starts (one coalesced
// pre-pass over the payload indices, so a block's chain is starts -> entries -> local gather ->
// store), staged in LDS, and each entry whose element no EARLIER payload hits (an LDS binary
// search per earlier run) folds that element: the local value gathered once, the later payloads'
// values by LDS binary search.  A tile whose runs exceed the LDS stage is processed in halves,
// the sub-ranges' runs found by lock-step searches (adversarially clustered payloads; always
// terminates: one element holds <= 16 entries).  Bytes: the payload entries, a local gather and
// an out write per hit element.
constexpr int PT_CAP = 1024;  // entries staged per pass (8 KB of LDS: 8 blocks per CU)
constexpr int PT_EPT = PT_CAP / 256;

__device__ __forceinline__ int pt_find(const int32_t* sidx, int b, int e, int32_t key) {
  // position of key in the sorted LDS run [b, e), or -1
  while (b < e) {
    const int m = (b + e) >> 1;
    const int32_t v = sidx[m];
    if (v < key) b = m + 1;
    else if (v > key) e = m;
    else return m;
  }
  return -1;
}

__global__ void __launch_bounds__(256) fold_patch_kernel(FoldArgs a, int64_t range) {
  // range == FOLD_TILE: the first pass takes its runs from a.starts (fold_offsets_kernel)
  __shared__ int32_t s_idx[PT_CAP];
  __shared__ float s_val[PT_CAP];
  __shared__ int32_t s_rlo[FOLD_MAXP], s_rhi[FOLD_MAXP], s_off[FOLD_MAXP + 1];
  const int t = threadIdx.x, wid = t >> 6, lane = t & 63;
  const int np = a.np;
  const int64_t n = a.n;
  const int64_t b_lo = (int64_t)blockIdx.x * range;
  const int64_t b_hi = b_lo + range < n ? b_lo + range : n;
  int64_t cur = b_lo, len = b_hi - b_lo;
  bool from_starts = a.starts != nullptr;
  while (cur < b_hi) {
    const int64_t s_end = cur + len < b_hi ? cur + len : b_hi;
    if (from_starts) {  // the whole tile: runs from the pre-pass
      if (t < np) {
        const int32_t* st = a.starts + (int64_t)t * (a.ntiles + 1);
        s_rlo[t] = st[blockIdx.x];
        s_rhi[t] = st[blockIdx.x + 1];
      }
    } else {
    // runs of [cur, s_end): wave w searches payloads w, w + 4, w + 8, w + 12, both ends, in lock
    // step (virtual search q: payload w + 4 (q & 3), target q < 4 ? cur : s_end)
      const int32_t lo32 = (int32_t)cur, hi32 = (int32_t)s_end;
      const int32_t r = fw_lower_bounds_t<8>(
          8, [&](int q) { return q < 4 ? lo32 : hi32; }, lane,
          [&](int q) { return a.p[wid + 4 * (q & 3)].idx; },
          [&](int q) {
            const int pp = wid + 4 * (q & 3);
            return pp < np ? (int32_t)a.p[pp].k : 0;
          },
          reinterpret_cast<const int32_t*>(a.local));
      if (lane < 8) {
        const int pp = wid + 4 * (lane & 3);
        if (pp < np) {
          if (lane < 4) s_rlo[pp] = r;
          else s_rhi[pp] = r;
        }
      }
    }
    from_starts = false;
    __syncthreads();
    if (t == 0) {
      int32_t o = 0;
      for (int p = 0; p < np; ++p) {
        s_off[p] = o;
        o += s_rhi[p] > s_rlo[p] ? s_rhi[p] - s_rlo[p] : 0;
      }
      s_off[np] = o;
    }
    __syncthreads();
    const int total = s_off[np];
    if (total > PT_CAP) {  // uniform: halve the range and search again
      len = (s_end - cur + 1) / 2;
      __syncthreads();
      continue;
    }
    // stage the runs (payload-major, each run sorted)
    for (int j = t; j < total; j += 256) {
      int p = 0;
      while (p + 1 < np && j >= s_off[p + 1]) ++p;
      const int64_t src = (int64_t)s_rlo[p] + (j - s_off[p]);
      s_idx[j] = as_global(a.p[p].idx)[src];
      s_val[j] = as_global(a.p[p].val)[src];
    }
    __syncthreads();
    // owners: entry j of payload p folds its element iff no earlier payload's run holds it; the
    // local values of every owned element are gathered before any later-payload search
    int32_t ee[PT_EPT];
    int pj[PT_EPT];
    float xv[PT_EPT];
#pragma unroll
    for (int i = 0; i < PT_EPT; ++i) {
      const int j = t + 256 * i;
      ee[i] = -1;
      pj[i] = 0;
      if (j < total) {
        int p = 0;
        while (p + 1 < np && j >= s_off[p + 1]) ++p;
        const int32_t e = s_idx[j];
        bool own = e >= cur && e < s_end;  // an invalid (unsorted) payload cannot write outside
        for (int q = 0; q < p && own; ++q) own = pt_find(s_idx, s_off[q], s_off[q + 1], e) < 0;
        if (own) {
          ee[i] = e;
          pj[i] = p;
        }
      }
      xv[i] = a.local[ee[i] >= 0 ? ee[i] : 0];
    }
#pragma unroll
    for (int i = 0; i < PT_EPT; ++i) {
      if (ee[i] < 0) continue;
      const int j = t + 256 * i;
      const int p = pj[i];
      const float x = xv[i];
      float acc = 0.0f;
      for (int q = 0; q < np; ++q) {
        float v = x;
        if (q == p) {
          v = s_val[j];
        } else if (q > p) {
          const int pos = pt_find(s_idx, s_off[q], s_off[q + 1], ee[i]);
          if (pos >= 0) v = s_val[pos];
        }
        const float term = v * a.p[q].w;
        acc = q == 0 ? term : acc + term;
      }
      acc = acc + x * a.w_self;
      a.out[ee[i]] = acc;
    }
    __syncthreads();  // the stage is reused by the next sub-range
    cur = s_end;
    len = b_hi - cur;
  }
}

// One payload: its indices are unique, so every hit element is hit once and each entry folds its
// element alone (out[e] = v·w + x[e]·w_self, the reference's order) — no tile runs, no pre-pass.
// Four entries per thread, strided by the block so the idx / val loads stay coalesced; the local
// gathers of all four are issued before any store.
__global__ void __launch_bounds__(256) fold_patch1_kernel(const int32_t* __restrict__ idx,
                                                          const float* __restrict__ val, int64_t k,
                                                          const float* __restrict__ local,
                                                          float* __restrict__ out, int64_t n,
                                                          float w, float w_self) {
  const int64_t j0 = (int64_t)blockIdx.x * 1024 + threadIdx.x;
  int32_t e[4];
  float v[4], xv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t j = j0 + 256 * i;
    e[i] = j < k ? idx[j] : -1;
    v[i] = j < k ? val[j] : 0.0f;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (e[i] >= n) e[i] = -1;  // an invalid payload cannot write outside
    xv[i] = local[e[i] >= 0 ? e[i] : 0];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (e[i] < 0) continue;
    const float acc = v[i] * w;
    out[e[i]] = acc + xv[i] * w_self;
  }
}

static int launch_fold_patch(FoldArgs fa, int32_t* starts, hipStream_t st) {
  int64_t etot = 0, kmax = 0;
  for (int i = 0; i < fa.np; ++i) {
    etot += fa.p[i].k;
    if (fa.p[i].k > kmax) kmax = fa.p[i].k;
  }
  if (etot == 0) return DPZ_OK;
  if (fa.np == 1) {
    DPZ_TIMED(DPZ_KT_FOLD, st,
              fold_patch1_kernel<<<(unsigned)((kmax + 1023) / 1024), 256, 0, st>>>(
                  fa.p[0].idx, fa.p[0].val, kmax, fa.local, fa.out, fa.n, fa.p[0].w, fa.w_self));
    return DPZ_OK;
  }
  fa.ntiles = fold_ntiles(fa.n);
  dim3 og((unsigned)((kmax + 1 + 1023) / 1024), (unsigned)fa.np);
  DPZ_TIMED(DPZ_KT_FOLD_OFFSETS, st,
            fold_offsets_kernel<FOLD_TILE_SHIFT><<<og, 256, 0, st>>>(fa, starts, fa.ntiles));
  fa.starts = starts;
  DPZ_TIMED(DPZ_KT_FOLD, st, fold_patch_kernel<<<(unsigned)fa.ntiles, 256, 0, st>>>(fa, FOLD_TILE));
  return DPZ_OK;
}

template <bool VEC, int EPL>
static int launch_walk_batch_t(const FoldNodeBatch& b, hipStream_t st) {
  static int per = 0, cus = 0;
  if (per == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per, reinterpret_cast<const void*>(fold_walk_batch_kernel<VEC, EPL>), 256, 0) !=
            hipSuccess || per < 1)
      per = 1;
  }
  constexpr int TE = 64 * EPL;
  const int64_t tiles = (int64_t)b.m * ((b.n + TE - 1) / TE);
  int64_t blocks = (int64_t)cus * per;
  const int64_t need = (tiles + FW_WAVES - 1) / FW_WAVES;
  if (blocks > need) blocks = need;
  if (blocks < 1) blocks = 1;
  const int64_t tpw = (tiles + blocks * FW_WAVES - 1) / (blocks * FW_WAVES);
  DPZ_TIMED(DPZ_KT_FOLD, st, (fold_walk_batch_kernel<VEC, EPL><<<(unsigned)blocks, 256, 0, st>>>(b, tpw)));
  return DPZ_OK;
}

// dpz_decode_average_batch's one-launch path: every node's fold a plain Metro-Hastings walk (1..4
// sparse payloads, a fresh total, DPZ_FOLD_SELF / DPZ_FOLD_ALSO_LOCAL only) over 16-byte aligned
// rows of the same n.  Returns 1 (nothing enqueued) when the batch does not qualify.
int fold_batch_walk(int m, const float* const* local, float* const* out, int64_t n,
                    const int* n_payloads, const int32_t* const* idx, const float* const* vals,
                    const int64_t* k, const float* w, const float* w_self, int flags,
                    hipStream_t st, const int32_t* guard, int64_t guard_n) {
  if (DPZ_KNOB_INT(FOLD_BATCH, 1) == 0) return 1;  // diagnostic build: per-node launches (A/B)
  // (every array this path reads is checked here: a null one falls through to the per-node
  // validation, which returns DPZ_ERR_ARG)
  if (m < 2 || (flags & ~(DPZ_FOLD_SELF | DPZ_FOLD_ALSO_LOCAL)) || !w || !idx || !vals || !k ||
      !n_payloads || !local || !out)
    return 1;
  if (n < 1024 || n >= (int64_t(1) << 31) - 1024) return 1;
  double dens = 0.0;
  int64_t off = 0;
  for (int j = 0; j < m; ++j) {
    const int np = n_payloads[j];
    if (np < 1 || np > 4 || !local[j] || !out[j] || local[j] == out[j]) return 1;
    if (((reinterpret_cast<uintptr_t>(local[j]) | reinterpret_cast<uintptr_t>(out[j])) & 15u) != 0)
      return 1;
    for (int i = 0; i < np; ++i) {
      const int64_t kk = k[off + i];
      if (!idx[off + i] || !vals[off + i] || kk < 1 || kk > n) return 1;  // sparse, non-empty
      if ((double)kk / (double)n > dens) dens = (double)kk / (double)n;
    }
    off += np;
  }
  // the walk's tile size for the densest payload (launch_walk, <= 4 payloads)
  const int e = dens <= 0.055 ? 16 : (dens <= 0.105 ? 8 : (dens <= 0.21 ? 4 : 2));
  off = 0;
  for (int j0 = 0; j0 < m; j0 += FW_BATCH) {
    FoldNodeBatch b{};
    b.n = n;
    b.m = (m - j0) < FW_BATCH ? (m - j0) : FW_BATCH;
    b.add_self = (flags & DPZ_FOLD_SELF) ? 1 : 0;
    b.guard = guard;
    b.guard_n = guard ? guard_n : 0;
    for (int j = 0; j < b.m; ++j) {
      FoldNode& nd = b.nd[j];
      const int jj = j0 + j;
      nd.local = local[jj];
      nd.out = out[jj];
      nd.out2 = (flags & DPZ_FOLD_ALSO_LOCAL) ? const_cast<float*>(local[jj]) : nullptr;
      nd.np = n_payloads[jj];
      nd.w_self = w_self ? w_self[jj] : 0.0f;
      for (int i = 0; i < nd.np; ++i) {
        nd.p[i].idx = idx[off + i];
        nd.p[i].val = vals[off + i];
        nd.p[i].k = k[off + i];
        nd.p[i].w = w[off + i];
      }
      off += nd.np;
    }
    int rc;
    switch (e) {
      case 16: rc = launch_walk_batch_t<true, 16>(b, st); break;
      case 8: rc = launch_walk_batch_t<true, 8>(b, st); break;
      case 4: rc = launch_walk_batch_t<true, 4>(b, st); break;
      default: rc = launch_walk_batch_t<true, 2>(b, st); break;
    }
    if (rc != DPZ_OK) return rc;
  }
  return DPZ_OK;
}

}  // namespace dpz

using namespace dpz;

#ifdef DPZ_STAMPS
extern "C" int dpz_debug_fold_stamps(unsigned long long* host_out, int reset) {
  if (host_out) DPZ_HIP_TRY(hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_fold_st), sizeof(g_fold_st)));
  if (reset) {
    static unsigned long long zero[6][8192];
    DPZ_HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_fold_st), zero, sizeof(zero)));
  }
  return 0;
}
#endif

// ---- merge fold: a group of sparse payloads merged per tile through an LDS hit mask ------------
// (round 6; the JWINS receive, 16 payloads at alpha 0.01: reference Wavelet.py:269-309)
// A persistent block walks a contiguous run of TE-element tiles.  Wave w holds the 64-entry
// windows of payloads w, w + 4, w + 8, w + 12 (the next tile's windows and local values are
// issued one tile ahead, so the stream's loads are in flight while a tile is merged).  Per tile:
//   1. every payload's entries in the tile (the leading window lanes below the tile's end) set
//      bit p of their element's 16-bit word in an LDS mask; meanwhile every element folds its
//      local value alone (the no-hit base; the elements advance through the terms together);
//   2. each wave numbers its own elements' bits (a wave scan): every hit element gets a run of
//      value slots in the wave's region, in payload order (the rank of bit p among its bits);
//   3. every entry writes its value to its slot;
//   4. each wave lists its own hit elements (ballots) and its lanes fold them exactly — term p
//      = (bit p ? slot value : local) * w_p in payload order, then the self term (the
//      reference's fp32 order) — over the base.
// Three block barriers per tile.  Every element's local value and output are read / written
// once, every payload entry read once (extra windows of a payload denser than 64 entries per
// tile are re-read from L2).  A tile whose entries exceed a wave's value slots (1 per element;
// adversarial clustering) folds payload by payload instead.  Weights all equal (EQW: a regular
// graph's Metro-Hastings weights): the base is one product and np - 1 additions of it, the same
// bits as the general order.
constexpr int FM_THREADS = 256;
constexpr int FM_WAVES = FM_THREADS / 64;
constexpr int FM_SLOTS = FOLD_MAXP / FM_WAVES;  // payload slots per wave: payload wid + 4 j

template <int EPT>
struct FmCfg {
  static constexpr int TE = FM_THREADS * EPT;  // elements per tile (= value slots per tile)
  static_assert(EPT % 4 == 0 && TE <= 65535, "float4 chunks, u16 slot offsets");
};

// element e of thread t (chunk e / 4 at (e / 4) * 4 * FM_THREADS + 4 t + e % 4: float4-coalesced)
__device__ __forceinline__ int fm_elem(int t, int e) {
  return (e >> 2) * (4 * FM_THREADS) + 4 * t + (e & 3);
}

// Branch-free (the compiler then waits only for the registers it uses, never for the next
// tile's loads in flight): a float4 group reaching past n reads the last whole group instead; the
// global last tile, if ragged, is reloaded element-wise by fm_load_tail before use.
template <int EPT>
__device__ __forceinline__ void fm_load(const float* __restrict__ p, int64_t tlo, int64_t n, int t,
                                        float (&v)[EPT]) {
  const int64_t last = (n & ~int64_t(3)) - 4;
#pragma unroll
  for (int c = 0; c < EPT / 4; ++c) {
    const int64_t i0 = tlo + fm_elem(t, 4 * c);
    const float4 q = *reinterpret_cast<const float4*>(p + (i0 + 4 <= n ? i0 : last));
    v[4 * c] = q.x; v[4 * c + 1] = q.y; v[4 * c + 2] = q.z; v[4 * c + 3] = q.w;
  }
}

template <int EPT>
__device__ __forceinline__ void fm_load_tail(const float* __restrict__ p, int64_t tlo, int64_t n,
                                             int t, float (&v)[EPT]) {
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    const int64_t i = tlo + fm_elem(t, e);
    v[e] = p[i < n ? i : n - 1];
  }
}

template <int EPT>
__device__ __forceinline__ void fm_store(float* __restrict__ p, int64_t tlo, int64_t n, int t,
                                         const float (&v)[EPT]) {
  constexpr int TE = FmCfg<EPT>::TE;
  typedef float v4f __attribute__((ext_vector_type(4)));
  if (tlo + TE <= n) {
#pragma unroll
    for (int c = 0; c < EPT / 4; ++c) {
      const v4f q = {v[4 * c], v[4 * c + 1], v[4 * c + 2], v[4 * c + 3]};
      __builtin_nontemporal_store(q, reinterpret_cast<v4f*>(p + tlo + fm_elem(t, 4 * c)));
    }
  } else {
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
      const int64_t i = tlo + fm_elem(t, e);
      if (i < n) p[i] = v[e];
    }
  }
}

template <int EPT, bool EQW>
__global__ void __launch_bounds__(FM_THREADS) __attribute__((amdgpu_waves_per_eu(EPT <= 8 ? 4 : 2, 8))) fold_merge_kernel(FoldArgs a, int64_t tpb, int abl) {
  using C = FmCfg<EPT>;
  constexpr int TE = C::TE;
  constexpr int WE = 64 * EPT;     // elements of one wave (its value slots: WE, 1 per element)
  // element e's payload bits: the 16-bit half (e & 1) of word e / 2 (np <= 16)
  __shared__ __attribute__((aligned(16))) uint32_t s_mask[2][TE / 2];
  __shared__ __attribute__((aligned(16))) uint16_t s_pre[TE];
  __shared__ __attribute__((aligned(16))) float s_x[TE];
  __shared__ float s_val[TE];
  __shared__ uint16_t s_list[TE];
  __shared__ uint32_t s_over[2];
  const int t = threadIdx.x, lane = t & 63;
  const int wid = __builtin_amdgcn_readfirstlane(t >> 6);
  const int64_t n = a.n;
  const int np = a.np;
  const int64_t ntl = (n + TE - 1) / TE;
  const int64_t t0 = (int64_t)blockIdx.x * tpb;
  const int64_t t1 = t0 + tpb < ntl ? t0 + tpb : ntl;
  if (t0 >= t1) return;  // uniform over the block
  // payload parameters: lane p holds payload p's, read back per slot / per chain step (readlane)
  const int lp = lane < np ? lane : 0;
  const uint64_t ipl = reinterpret_cast<uint64_t>(a.p[lp].k > 0 ? a.p[lp].idx
                                                                : reinterpret_cast<const int32_t*>(a.local));
  const uint64_t vpl = reinterpret_cast<uint64_t>(a.p[lp].k > 0 ? a.p[lp].val : a.local);
  const int32_t kl = lane < np ? (int32_t)a.p[lp].k : 0;
  const float wl = a.p[lp].w;
  auto rl64 = [](uint64_t v, int p) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, p);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), p);
    return ((uint64_t)hi << 32) | lo;
  };
  auto W = [&](int p) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wl), p)); };
  const int32_t* sidx[FM_SLOTS];
  const float* sval[FM_SLOTS];
  int32_t sk[FM_SLOTS];
#pragma unroll
  for (int j = 0; j < FM_SLOTS; ++j) {
    const int p = wid + FM_WAVES * j;
    const bool live = p < np;
    sidx[j] = reinterpret_cast<const int32_t*>(rl64(ipl, live ? p : 0));
    sval[j] = reinterpret_cast<const float*>(rl64(vpl, live ? p : 0));
    sk[j] = live ? fw_uni(__builtin_amdgcn_readlane(kl, p)) : 0;
  }
  const int nsl = np > wid ? (np - wid + FM_WAVES - 1) / FM_WAVES : 0;  // this wave's live slots
  for (int i = t; i < TE; i += FM_THREADS) (&s_mask[0][0])[i] = 0u;
  if (t < 2) s_over[t] = 0u;
  // start cursors: lower_bound(idx_p, t0 * TE) of this wave's payloads (lane j: slot j)
  const int32_t curv = fw_start_cursors<FM_SLOTS, false>(
      nsl, (int32_t)(t0 * TE), lane, [&](int j) { return sidx[j]; }, [&](int j) { return sk[j]; },
      reinterpret_cast<const int32_t*>(a.local));
  int32_t cs[FM_SLOTS];
#pragma unroll
  for (int j = 0; j < FM_SLOTS; ++j) cs[j] = fw_uni(__builtin_amdgcn_readlane(curv, j));
  int32_t wi[FM_SLOTS], wn[FM_SLOTS];
  float wv[FM_SLOTS], wvn[FM_SLOTS];
  auto load_window = [&](int j, int32_t c, int32_t& ix, float& vx) {
    const int32_t q = c + lane;
    const bool ok = q < sk[j];
    const int32_t qq = ok ? q : 0;
    ix = as_global(sidx[j])[qq];
    vx = as_global(sval[j])[qq];
    ix = ok ? ix : INT32_MAX;
  };
#pragma unroll
  for (int j = 0; j < FM_SLOTS; ++j) load_window(j, cs[j], wi[j], wv[j]);
  float L[EPT], Ln[EPT];
  fm_load<EPT>(a.local, t0 * TE, n, t, L);
  const float w0 = W(0);
  uint32_t buf = 0;
  const int zb = a.zero_base;
  __syncthreads();  // masks zeroed
  for (int64_t tile = t0; tile < t1; ++tile) {
    const int64_t tlo = tile * TE;
    const int32_t tlo32 = (int32_t)tlo, thi32 = tlo32 + TE;
    uint32_t* const mask = s_mask[buf];
    if (tlo + TE > n) fm_load_tail<EPT>(a.local, tlo, n, t, L);  // the ragged last tile
    // 1. mask bits of every payload's entries in the tile; the next tile's windows issued
    int32_t c0[FM_SLOTS], cfirst[FM_SLOTS];
#pragma unroll
    for (int j = 0; j < FM_SLOTS; ++j) {
      c0[j] = cs[j];
      cfirst[j] = 0;
      if (j >= nsl) continue;  // uniform
      const int p = wid + FM_WAVES * j;
      int32_t c = fw_lead(wi[j] < thi32);
      cfirst[j] = c;
      if (!(abl & 4)) {
        const uint32_t pos = (uint32_t)(wi[j] - tlo32);
        if (lane < c && pos < (uint32_t)TE) atomicOr(&mask[pos >> 1], 1u << (p + 16 * (pos & 1u)));
      }
      if (c == 64) {  // a payload denser than one window per tile: its further windows now
        for (int32_t q0 = cs[j] + 64;; q0 += 64) {
          const int32_t q = q0 + lane;
          const int32_t iv = q < sk[j] ? as_global(sidx[j])[q] : INT32_MAX;
          const int cc = fw_lead(iv < thi32);
          const uint32_t pos = (uint32_t)(iv - tlo32);
          if (lane < cc && pos < (uint32_t)TE) atomicOr(&mask[pos >> 1], 1u << (p + 16 * (pos & 1u)));
          c += cc;
          if (cc < 64) break;
        }
      }
      cs[j] = cs[j] + c;
    }
#pragma unroll
    for (int j = 0; j < FM_SLOTS; ++j) load_window(j, cs[j], wn[j], wvn[j]);
    fm_load<EPT>(a.local, tile + 1 < t1 ? tlo + TE : tlo, n, t, Ln);  // (the run's last: L2)
    // the base: every element's fold of its local value alone (the no-hit value); the elements
    // advance through the terms together (independent adds, one loop for all), while other
    // waves still set mask bits
    float base[EPT];
    if (abl & 8) {
#pragma unroll
      for (int e = 0; e < EPT; ++e) base[e] = L[e];
    } else {
      float tw[EPT];
#pragma unroll
      for (int e = 0; e < EPT; ++e) {
        tw[e] = (zb ? 0.0f : L[e]) * w0;
        base[e] = zb ? 0.0f + tw[e] : tw[e];
      }
      for (int p = 1; p < np; ++p) {
        if (EQW) {
#pragma unroll
          for (int e = 0; e < EPT; ++e) base[e] = base[e] + tw[e];
        } else {
          const float w = W(p);
#pragma unroll
          for (int e = 0; e < EPT; ++e) base[e] = base[e] + (zb ? 0.0f : L[e]) * w;
        }
      }
      if (a.add_self) {
#pragma unroll
        for (int e = 0; e < EPT; ++e) base[e] = base[e] + L[e] * a.w_self;
      }
    }
    __syncthreads();  // B1: the tile's mask is complete; the previous tile is done everywhere
    // 2. per-element value runs: each wave numbers its own elements' entries (slots of the
    // wave's region, in payload order per element); the local values staged for the hit folds
    uint32_t m[EPT];
#pragma unroll
    for (int c = 0; c < EPT / 4; ++c) {
      const uint2 q = *reinterpret_cast<const uint2*>(&mask[fm_elem(t, 4 * c) >> 1]);
      m[4 * c] = q.x & 0xFFFFu; m[4 * c + 1] = q.x >> 16;
      m[4 * c + 2] = q.y & 0xFFFFu; m[4 * c + 3] = q.y >> 16;
      *reinterpret_cast<float4*>(&s_x[fm_elem(t, 4 * c)]) =
          make_float4(L[4 * c], L[4 * c + 1], L[4 * c + 2], L[4 * c + 3]);
    }
    uint32_t mine = 0;
#pragma unroll
    for (int e = 0; e < EPT; ++e) mine += (uint32_t)__popc(m[e]);
    uint32_t wtot = 0;
    uint32_t run = (abl & 16) ? 0u : wave_excl_scan(mine, &wtot) + (uint32_t)(wid * WE);
    if (wtot > (uint32_t)WE && lane == 0) s_over[buf] = 1u;  // (uniform read after B3)
#pragma unroll
    for (int c = 0; c < EPT / 4; ++c) {
      uint32_t pr[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        pr[e] = run < 65535u ? run : 65535u;
        run += (uint32_t)__popc(m[4 * c + e]);
      }
      *reinterpret_cast<uint2*>(&s_pre[fm_elem(t, 4 * c)]) =
          make_uint2(pr[0] | (pr[1] << 16), pr[2] | (pr[3] << 16));
    }
    __syncthreads();  // B3: every element's slot run known
    const bool over = s_over[buf] != 0u;  // uniform
    if (!over) {
      // 3. values into their slots (slot = the run start + the rank of bit p among the bits)
      if (!(abl & 2)) {
#pragma unroll
        for (int j = 0; j < FM_SLOTS; ++j) {
          if (j >= nsl) continue;
          const int p = wid + FM_WAVES * j;
          const uint32_t below = (1u << p) - 1u;
          auto place = [&](int32_t iv, float vv, bool in) {
            const uint32_t pos = (uint32_t)(iv - tlo32);
            if (in && pos < (uint32_t)TE) {
              const uint32_t mm = (mask[pos >> 1] >> (16 * (pos & 1u))) & 0xFFFFu;
              const uint32_t slot = (uint32_t)s_pre[pos] + (uint32_t)__popc(mm & below);
              if (slot < (uint32_t)TE) s_val[slot] = vv;
            }
          };
          place(wi[j], wv[j], lane < cfirst[j]);
          if (cfirst[j] == 64) {
            for (int32_t q0 = c0[j] + 64;; q0 += 64) {
              const int32_t q = q0 + lane;
              const bool ok = q < sk[j];
              const int32_t iv = ok ? as_global(sidx[j])[q] : INT32_MAX;
              const float vv = as_global(sval[j])[ok ? q : 0];
              const int cc = fw_lead(iv < thi32);
              place(iv, vv, lane < cc);
              if (cc < 64) break;
            }
          }
        }
      }
      __syncthreads();  // B4: every value in its slot
      // 4. the wave's own hit elements, listed (ballot order) and folded exactly by its lanes
      // (reference order: the payload terms, then the self term); results over the staged
      // local values, then over the base
      if (!(abl & 1)) {
        uint16_t* const wl_ = s_list + wid * WE;
        uint32_t nh = 0;
#pragma unroll
        for (int e = 0; e < EPT; ++e) {
          const uint64_t b = __ballot(m[e] != 0u);
          if (m[e])
            wl_[nh + __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32),
                                               __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u))] =
                (uint16_t)fm_elem(t, e);
          nh += (uint32_t)__popcll(b);
        }
        __builtin_amdgcn_wave_barrier();
#if DPZ_MERGE_HIT2
        // two hit elements per lane at a time (i and i + 64): two independent dependent chains
        // interleave; the one-to-three-hit fold runs for both unconditionally and the rare
        // element with four or more hits is redone payload by payload afterwards
        auto fast = [&](uint32_t mm, uint32_t sl, float tb) -> float {
          const int p0 = __ffs((int)mm) - 1;
          const uint32_t mm1 = mm & (mm - 1u);
          const int p1 = mm1 ? __ffs((int)mm1) - 1 : 32;
          const uint32_t mm2 = mm1 & (mm1 - 1u);
          const int p2 = mm2 ? __ffs((int)mm2) - 1 : 32;
          const float v0 = s_val[sl < (uint32_t)TE ? sl : 0u];
          const float v1 = s_val[sl + 1u < (uint32_t)TE ? sl + 1u : 0u];
          const float v2 = s_val[sl + 2u < (uint32_t)TE ? sl + 2u : 0u];
          float acc = 0.0f;
          if (EQW) {
            const float xw = tb * w0, v0w = v0 * w0, v1w = v1 * w0, v2w = v2 * w0;
#pragma unroll
            for (int p = 0; p < FOLD_MAXP; ++p) {
              if (p >= np) break;
              const float term = p == p0 ? v0w : (p == p1 ? v1w : (p == p2 ? v2w : xw));
              acc = p == 0 ? (zb ? 0.0f + term : term) : acc + term;
            }
          } else {
#pragma unroll
            for (int p = 0; p < FOLD_MAXP; ++p) {
              if (p >= np) break;
              const float tv = p == p0 ? v0 : (p == p1 ? v1 : (p == p2 ? v2 : tb));
              const float term = tv * W(p);
              acc = p == 0 ? (zb ? 0.0f + term : term) : acc + term;
            }
          }
          return acc;
        };
        auto slow = [&](uint32_t mm, uint32_t sl, float tb) -> float {
          uint32_t s2 = sl;
          float acc = 0.0f;
          for (int p = 0; p < np; ++p) {
            float tv = tb;
            if ((mm >> p) & 1u) {
              tv = s_val[s2 < (uint32_t)TE ? s2 : 0u];
              ++s2;
            }
            const float term = tv * W(p);
            acc = p == 0 ? (zb ? 0.0f + term : term) : acc + term;
          }
          return acc;
        };
        for (uint32_t i = (uint32_t)lane; i < nh; i += 128) {
          const uint32_t i2 = i + 64u < nh ? i + 64u : i;
          const uint32_t pa = wl_[i], pb = wl_[i2];
          const uint32_t ma = (mask[pa >> 1] >> (16 * (pa & 1u))) & 0xFFFFu;
          const uint32_t mb = (mask[pb >> 1] >> (16 * (pb & 1u))) & 0xFFFFu;
          const uint32_t sa = s_pre[pa], sb = s_pre[pb];
          const float xa = s_x[pa], xb = s_x[pb];
          float acca = fast(ma, sa, zb ? 0.0f : xa);
          float accb = fast(mb, sb, zb ? 0.0f : xb);
          if (__popc(ma) > 3) acca = slow(ma, sa, zb ? 0.0f : xa);
          if (__popc(mb) > 3) accb = slow(mb, sb, zb ? 0.0f : xb);
          if (a.add_self) {
            acca = acca + xa * a.w_self;
            accb = accb + xb * a.w_self;
          }
          s_x[pb] = accb;  // (i2 == i: the same value twice)
          s_x[pa] = acca;
        }
#else
        for (uint32_t i = (uint32_t)lane; i < nh; i += 64) {
          const uint32_t pos = wl_[i];
          const uint32_t mm = (mask[pos >> 1] >> (16 * (pos & 1u))) & 0xFFFFu;
          const uint32_t sl = s_pre[pos];
          const float xv = s_x[pos];
          const float tb = zb ? 0.0f : xv;
          const int p0 = __ffs((int)mm) - 1;
          const uint32_t mm1 = mm & (mm - 1u);
          const int p1 = mm1 ? __ffs((int)mm1) - 1 : 32;
          const uint32_t mm2 = mm1 & (mm1 - 1u);
          const int p2 = mm2 ? __ffs((int)mm2) - 1 : 32;
          float acc;
          if (abl & 32) {  // (timing ablation: the chain skipped, its loads kept)
            acc = s_val[sl < (uint32_t)TE ? sl : 0u] + tb + (float)p0 + (float)p1 + (float)p2;
          } else if ((mm2 & (mm2 - 1u)) == 0u) {  // one to three payloads hit it (all but ~1e-4)
            const float v0 = s_val[sl < (uint32_t)TE ? sl : 0u];
            const float v1 = s_val[sl + 1u < (uint32_t)TE ? sl + 1u : 0u];
            const float v2 = s_val[sl + 2u < (uint32_t)TE ? sl + 2u : 0u];
            acc = 0.0f;
            if (EQW) {  // every product once (equal weights: the same bits as w_p each term)
              const float xw = tb * w0, v0w = v0 * w0, v1w = v1 * w0, v2w = v2 * w0;
#pragma unroll
              for (int p = 0; p < FOLD_MAXP; ++p) {
                if (p >= np) break;
                const float term = p == p0 ? v0w : (p == p1 ? v1w : (p == p2 ? v2w : xw));
                acc = p == 0 ? (zb ? 0.0f + term : term) : acc + term;
              }
            } else {
#pragma unroll
              for (int p = 0; p < FOLD_MAXP; ++p) {
                if (p >= np) break;
                const float tv = p == p0 ? v0 : (p == p1 ? v1 : (p == p2 ? v2 : tb));
                const float term = tv * W(p);
                acc = p == 0 ? (zb ? 0.0f + term : term) : acc + term;
              }
            }
          } else {  // four or more (adversarial overlap): payload by payload from the slots
            uint32_t s2 = sl;
            acc = 0.0f;
            for (int p = 0; p < np; ++p) {
              float tv = tb;
              if ((mm >> p) & 1u) {
                tv = s_val[s2 < (uint32_t)TE ? s2 : 0u];
                ++s2;
              }
              const float term = tv * W(p);
              acc = p == 0 ? (zb ? 0.0f + term : term) : acc + term;
            }
          }
          if (a.add_self) acc = acc + xv * a.w_self;
          s_x[pos] = acc;
        }
#endif
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int c = 0; c < EPT / 4; ++c) {
          const float4 q = *reinterpret_cast<const float4*>(&s_x[fm_elem(t, 4 * c)]);
          const float h[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (m[4 * c + e]) base[4 * c + e] = h[e];
        }
      }
    } else {
      // more entries than a wave's value slots: payload by payload, an LDS value tile tagged
      // with p + 1 (adversarially clustered payloads)
      uint16_t* const tag = s_pre;  // (the runs are not used on this path)
      float* const vt = s_val;
#pragma unroll
      for (int e = 0; e < EPT; ++e) {
        base[e] = 0.0f;
        tag[fm_elem(t, e)] = 0;
      }
      __syncthreads();
      for (int p = 0; p < np; ++p) {
        if ((p & (FM_WAVES - 1)) == wid) {
          const int j = p / FM_WAVES;
          for (int32_t q0 = c0[j];; q0 += 64) {
            const int32_t q = q0 + lane;
            const bool ok = q < sk[j];
            const int32_t iv = ok ? as_global(sidx[j])[q] : INT32_MAX;
            const float vv = as_global(sval[j])[ok ? q : 0];
            const int cc = fw_lead(iv < thi32);
            const uint32_t pos = (uint32_t)(iv - tlo32);
            if (lane < cc && pos < (uint32_t)TE) {
              vt[pos] = vv;
              tag[pos] = (uint16_t)(p + 1);
            }
            if (cc < 64) break;
          }
        }
        __syncthreads();
        const float w = W(p);
#pragma unroll
        for (int e = 0; e < EPT; ++e) {
          const int el = fm_elem(t, e);
          const float tb = zb ? 0.0f : L[e];
          const float tv = tag[el] == (uint16_t)(p + 1) ? vt[el] : tb;
          const float term = tv * w;
          base[e] = p == 0 ? (zb ? 0.0f + term : term) : base[e] + term;
        }
        __syncthreads();
      }
      if (a.add_self) {
#pragma unroll
        for (int e = 0; e < EPT; ++e) base[e] = base[e] + L[e] * a.w_self;
      }
    }
    fm_store<EPT>(a.out, tlo, n, t, base);
    if (a.out2) fm_store<EPT>(a.out2, tlo, n, t, base);
    // this buffer's mask words and overflow flag back to zero (the next tile uses the other pair)
#pragma unroll
    for (int c = 0; c < EPT / 4; ++c)
      *reinterpret_cast<uint2*>(&mask[fm_elem(t, 4 * c) >> 1]) = make_uint2(0u, 0u);
    if (t == 0) s_over[buf] = 0u;
    buf ^= 1u;
#pragma unroll
    for (int j = 0; j < FM_SLOTS; ++j) {
      wi[j] = wn[j];
      wv[j] = wvn[j];
    }
#pragma unroll
    for (int e = 0; e < EPT; ++e) L[e] = Ln[e];
  }
}

// The merge fold's launch: a persistent grid of what the CUs hold, each block a contiguous run.
template <int EPT, bool EQW>
static int launch_merge_t(const FoldArgs& fa, hipStream_t st) {
  static int per = 0, cus = 0;
  if (per == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per, reinterpret_cast<const void*>(fold_merge_kernel<EPT, EQW>), FM_THREADS, 0) !=
            hipSuccess || per < 1)
      per = 1;
  }
  constexpr int TE = FmCfg<EPT>::TE;
  const int64_t ntl = (fa.n + TE - 1) / TE;
  int64_t blocks = (int64_t)cus * per;
  if (DPZ_KNOB_INT(MERGE_BLOCKS, 0) > 0) blocks = DPZ_KNOB_INT(MERGE_BLOCKS, 0);
  if (blocks > ntl) blocks = ntl;
  if (blocks < 1) blocks = 1;
  const int64_t tpb = (ntl + blocks - 1) / blocks;
  blocks = (ntl + tpb - 1) / tpb;
  // DPZ_MERGE_ABL (diagnostic build, timing only: results then differ) skips phases: 1 the hit
  // folds, 2 the value placement, 4 the mask bits, 8 the base, 16 the scan
  const int abl = (int)DPZ_KNOB_INT(MERGE_ABL, 0);
  DPZ_TIMED(DPZ_KT_FOLD, st, (fold_merge_kernel<EPT, EQW><<<(unsigned)blocks, FM_THREADS, 0, st>>>(fa, tpb, abl)));
  return DPZ_OK;
}

static bool merge_ok(const FoldArgs& fa) {
  if (fa.replace_only || !fa.first || !fa.all_sparse || fa.np < 1 || fa.np > FOLD_MAXP) return false;
  if (fa.n < 1024 || fa.n >= (int64_t(1) << 31) - 8192) return false;
  return aligned16(fa.local) && aligned16(fa.out) && (!fa.out2 || aligned16(fa.out2));
}

// elements per thread by the group's average entries per element (value slots hold 2 per element)
static int launch_merge(const FoldArgs& fa, double avg_per_elem, hipStream_t st) {
  bool eqw = true;
  for (int i = 1; i < fa.np; ++i) eqw = eqw && fa.p[i].w == fa.p[0].w;
  int ept = (int)DPZ_KNOB_INT(MERGE_EPT, 8);
  if (ept != 4 && ept != 8 && ept != 16) ept = 8;
  (void)avg_per_elem;
  switch (ept) {
    case 4: return eqw ? launch_merge_t<4, true>(fa, st) : launch_merge_t<4, false>(fa, st);
    case 16: return eqw ? launch_merge_t<16, true>(fa, st) : launch_merge_t<16, false>(fa, st);
    default: return eqw ? launch_merge_t<8, true>(fa, st) : launch_merge_t<8, false>(fa, st);
  }
}

extern "C" size_t dpz_decode_workspace_bytes(int64_t n, int n_payloads) {
  const int64_t np = n_payloads < FOLD_MAXP ? (n_payloads > 0 ? n_payloads : 1) : FOLD_MAXP;
  return (size_t)np * (size_t)(fold_ntiles(n > 0 ? n : 1) + 1) * sizeof(int32_t);
}

extern "C" int dpz_decode_average(const float* local, int64_t n, int n_payloads,
                                  const int32_t* const* idx, const float* const* vals,
                                  const int64_t* k, const float* w, float w_self, int flags,
                                  float* out, void* ws, size_t ws_bytes, dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (n < 0 || n_payloads < 0) return DPZ_ERR_ARG;
  if (n == 0) return DPZ_OK;
  if (!local || !out || local == out) return DPZ_ERR_ARG;
  const bool replace_only = (flags & DPZ_FOLD_REPLACE_ONLY) != 0;
  const bool add_only = (flags & DPZ_FOLD_ADD_ONLY) != 0;
  const bool zero_base = (flags & DPZ_FOLD_ZERO_BASE) != 0;
  if ((replace_only || add_only) && n_payloads != 1) return DPZ_ERR_ARG;
  const bool also_local = (flags & DPZ_FOLD_ALSO_LOCAL) != 0;
  if (also_local && (replace_only || add_only)) return DPZ_ERR_ARG;
  float* const out2 = also_local ? const_cast<float*>(local) : nullptr;
  if (replace_only && add_only) return DPZ_ERR_ARG;
  if (n_payloads > 0 && (!vals || !k || (!replace_only && !add_only && !w))) return DPZ_ERR_ARG;
  // payload i is dense (a full model) iff idx[i] == NULL and k[i] == n
  auto is_dense = [&](int i) { return (!idx || !idx[i]) && k[i] == n; };
  for (int i = 0; i < n_payloads; ++i) {
    if (k[i] < 0 || k[i] > n) return DPZ_ERR_ARG;
    if (!vals[i] && k[i] > 0) return DPZ_ERR_ARG;
    if (!is_dense(i) && k[i] > 0 && (!idx || !idx[i])) return DPZ_ERR_ARG;
  }
  if (!ws || ws_bytes < dpz_decode_workspace_bytes(n, n_payloads)) return DPZ_ERR_WORKSPACE;
  if (flags & DPZ_FOLD_BASE_READY) {
    // out holds the no-hit base of exactly this fold (dpz_topk_encode_foldbase over local with
    // these weights): only the plain Metro-Hastings form of one group of sparse payloads
    if (flags & ~(DPZ_FOLD_BASE_READY | DPZ_FOLD_SELF)) return DPZ_ERR_ARG;
    if (!(flags & DPZ_FOLD_SELF) || n_payloads < 1 || n_payloads > FOLD_MAXP) return DPZ_ERR_ARG;
    if (n >= (int64_t(1) << 31) - 1024) return DPZ_ERR_UNSUPPORTED;
    FoldArgs fa{};
    fa.local = local; fa.out = out; fa.n = n; fa.np = n_payloads; fa.w_self = w_self;
    for (int i = 0; i < n_payloads; ++i) {
      if (is_dense(i)) return DPZ_ERR_ARG;
      fa.p[i].idx = (idx && idx[i]) ? idx[i] : reinterpret_cast<const int32_t*>(local);
      fa.p[i].val = vals[i] ? vals[i] : local;
      fa.p[i].k = k[i];
      fa.p[i].w = w[i];
    }
    return launch_fold_patch(fa, static_cast<int32_t*>(ws), st);
  }
  bool vec = ((reinterpret_cast<uintptr_t>(local) | reinterpret_cast<uintptr_t>(out)) & 15u) == 0;
  for (int i = 0; i < n_payloads; ++i)
    if (is_dense(i) && (reinterpret_cast<uintptr_t>(vals[i]) & 15u)) vec = false;
  const int64_t ntiles = fold_ntiles(n);
  int32_t* starts = static_cast<int32_t*>(ws);
  if (n_payloads == 0) {
    // no payloads: out = w_self * local (self term only) or zeros
    FoldArgs fa{};
    fa.local = local; fa.out = out; fa.out2 = out2; fa.starts = starts; fa.n = n; fa.ntiles = ntiles;
    fa.np = 0; fa.first = 0;
    fa.add_self = (flags & DPZ_FOLD_SELF) ? 1 : 0; fa.w_self = w_self;
    if (!(flags & DPZ_FOLD_ACCUMULATE)) DPZ_HIP_TRY(hipMemsetAsync(out, 0, n * sizeof(float), st));
    if (vec) DPZ_TIMED(DPZ_KT_FOLD, st, fold_kernel<true><<<fold_grid<true>(ntiles), FOLD_THREADS, 0, st>>>(fa));
    else DPZ_TIMED(DPZ_KT_FOLD, st, fold_kernel<false><<<fold_grid<false>(ntiles), FOLD_THREADS, 0, st>>>(fa));
    return DPZ_OK;
  }
  // one sparse payload, replace only: single-kernel range-partitioned copy + scatter
  if (replace_only && !is_dense(0) && k[0] > 0 && vec) {
    const int64_t nc = replace_chunks(k[0]);
    return launch_replace(ReplaceJob{local, idx[0], vals[0], k[0], n, out, 0, nc, 0}, st);
  }
  if (add_only) {
    // out = local + T_0: the range-partitioned chunk kernel in add mode (k = 0: one virtual
    // chunk list over [0, n) with no entries is not possible, so k = 0 and dense payloads take
    // the fold path below with weight 1 and the self term)
    if (!is_dense(0) && k[0] > 0 && vec) {
      const int64_t nc = replace_chunks(k[0]);
      return launch_replace(ReplaceJob{local, idx[0], vals[0], k[0], n, out, 0, nc, 1}, st);
    }
  }
  for (int base = 0; base < n_payloads; base += FOLD_MAXP) {
    FoldArgs fa{};
    fa.local = local; fa.out = out; fa.out2 = out2; fa.starts = starts; fa.n = n; fa.ntiles = ntiles;
    fa.np = (n_payloads - base) < FOLD_MAXP ? (n_payloads - base) : FOLD_MAXP;
    fa.first = (base == 0 && !(flags & DPZ_FOLD_ACCUMULATE)) ? 1 : 0;
    fa.add_self = (base + fa.np == n_payloads && ((flags & DPZ_FOLD_SELF) || add_only)) ? 1 : 0;
    // over local only with the last group: the earlier groups' launches still read local
    if (base + fa.np != n_payloads) fa.out2 = nullptr;
    fa.replace_only = replace_only ? 1 : 0;
    fa.zero_base = (zero_base || add_only) ? 1 : 0;
    fa.w_self = add_only ? 1.0f : w_self;
    int64_t kmax = -1;
    for (int i = 0; i < fa.np; ++i) {
      // an empty sparse payload gets a dummy non-null idx (never read: its range is empty)
      fa.p[i].idx = is_dense(base + i) ? nullptr
                    : ((idx && idx[base + i]) ? idx[base + i] : reinterpret_cast<const int32_t*>(starts));
      fa.p[i].val = vals[base + i];
      fa.p[i].k = k[base + i];
      fa.p[i].w = (replace_only || add_only) ? 1.0f : w[base + i];
      if (fa.p[i].idx && fa.p[i].k > kmax) kmax = fa.p[i].k;
    }
    // DPZ_FOLD_PHASES=1 forces the per-payload phase path (diagnostic build)
    const bool force_phases = DPZ_KNOB_INT(FOLD_PHASES, 0) != 0;
    fa.all_sparse = force_phases ? 0 : 1;
    fa.dense_mask = 0;
    for (int i = 0; i < fa.np; ++i)
      if (!fa.p[i].idx) {
        fa.all_sparse = 0;
        fa.dense_mask |= 1u << i;
      }
    // The walk fold (no offsets pre-pass) takes all-sparse groups of a fresh total where it
    // measured faster on MI355X (M = 25 M, tools/diag/fold_kinds.py): a node's few neighbours
    // at any alpha; 16 payloads at alpha 0.0175 .. 0.2 (16 x 0.015: hit-chain 137 vs walk 147 us,
    // 16 x 0.02: 163 vs 149 us, profiles/r03_s2_fold_a001.jsonl; the hit-chain fold below, the phase
    // fold above).  DPZ_FOLD_KIND=1 / 2 / 4 forces the classic /
    // 4-slot group / walk fold (A/B diagnostics; a forced kind that cannot take the group runs
    // the classic kernel).
    int64_t etot = 0;
    double dens = 0.0;
    for (int i = 0; i < fa.np; ++i)
      if (fa.p[i].idx) {
        etot += fa.p[i].k;
        if ((double)fa.p[i].k / (double)n > dens) dens = (double)fa.p[i].k / (double)n;
      }
    const int kind = (int)DPZ_KNOB_INT(FOLD_KIND, 0);
    const double avg = fa.np > 0 ? (double)etot / (double)fa.np / (double)n : 0.0;
    // the merge fold (round 6) for larger groups at sparse alpha, where it measured faster than
    // the walk on MI355X (M = 25 M, tools/diag/merge_time.py, profiles/r06_merge_time.jsonl:
    // 16 x 0.005 88 vs 125 us, 16 x 0.01 105 vs 126, 16 x 0.02 129 vs 133, 8 x 0.01 69 vs 79;
    // 16 x 0.03 173 vs 132, 3 x 0.01 at 64 MiB 41 vs 33: the walk); DPZ_FOLD_KIND=8 forces it
    bool use_merge = merge_ok(fa) && fa.np >= 6 && (double)etot <= 0.33 * (double)n;
    if (kind) use_merge = merge_ok(fa) && kind == 8;
    if (use_merge) {
      const int rc = launch_merge(fa, (double)etot / (double)n, st);
      if (rc != DPZ_OK) return rc;
      continue;
    }
    bool use_walk = walk_ok(fa) && (fa.np <= 4 || (avg >= 0.0175 && avg <= 0.21));
    if (kind) use_walk = walk_ok(fa) && kind == 4;
    if (use_walk) {
      const int rc = launch_walk(fa, vec && n >= 1024, dens, st);
      if (rc != DPZ_OK) return rc;
      continue;
    }
    if (kmax >= 0) {
      dim3 og((unsigned)((kmax + 1 + 1023) / 1024), (unsigned)fa.np);
      DPZ_TIMED(DPZ_KT_FOLD_OFFSETS, st, fold_offsets_kernel<FOLD_TILE_SHIFT><<<og, 256, 0, st>>>(fa, starts, ntiles));
    }
    // all-sparse groups of >= 8 payloads with FOLD_GROUP_MIN .. 2 FG_CAP entries per tile on
    // average take the slotted fold (measured on MI355X at 25 M x 16 payloads: alpha 0.04
    // 463 -> 193 us, 0.1 345 -> 284 us; the hit-chain path stays faster at alpha 0.01, the
    // phase path at alpha 0.2 x 16 and for a few dense payloads); DPZ_FOLD_GROUP=0 / 1 forces it
    if (fa.all_sparse && fa.np > 0 && !fa.replace_only) {
      bool use_group = fa.np >= 8 && etot > FOLD_GROUP_MIN * ntiles &&
                       etot <= 2 * (int64_t)FG_CAP * ntiles;
      if (DPZ_KNOB_STR(FOLD_GROUP)) use_group = DPZ_KNOB_INT(FOLD_GROUP, 0) != 0;
      if (kind) use_group = kind == 2;
      if (use_group) {
        if (vec) DPZ_TIMED(DPZ_KT_FOLD, st, fold_group_kernel<true><<<fold_grid<true>(ntiles, true), FOLD_THREADS, 0, st>>>(fa));
        else DPZ_TIMED(DPZ_KT_FOLD, st, fold_group_kernel<false><<<fold_grid<false>(ntiles, true), FOLD_THREADS, 0, st>>>(fa));
        continue;
      }
    }
    if (vec) DPZ_TIMED(DPZ_KT_FOLD, st, fold_kernel<true><<<fold_grid<true>(ntiles), FOLD_THREADS, 0, st>>>(fa));
    else DPZ_TIMED(DPZ_KT_FOLD, st, fold_kernel<false><<<fold_grid<false>(ntiles), FOLD_THREADS, 0, st>>>(fa));
  }
  return DPZ_OK;
}

extern "C" int dpz_replace_slice(const float* local, int64_t n, int64_t offset,
                                 const int32_t* idx, const float* vals, int64_t k, float* out,
                                 dpz_stream_t stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (n < 0 || k < 0 || offset < 0) return DPZ_ERR_ARG;
  if (n == 0) return DPZ_OK;
  if (!local || !out || local == out || (k > 0 && (!idx || !vals))) return DPZ_ERR_ARG;
  if (!aligned16(local) || !aligned16(out)) return DPZ_ERR_ARG;
  if (k == 0) {
    DPZ_HIP_TRY(hipMemcpyAsync(out, local, (size_t)n * sizeof(float), hipMemcpyDeviceToDevice, st));
    return DPZ_OK;
  }
  return launch_replace(ReplaceJob{local, idx, vals, k, n, out, 0, replace_chunks(k), 0, offset}, st);
}
