// Exact multi-pass radix top-k (any n, k; ties -> lowest index).  See dpz_topk.hip.
//
// Pass structure: three radix histogram passes over the key stream (10/11/10 bits, LDS-privatised
// histograms flushed with one atomic per non-empty bin), each followed by a 1-block resolve of the
// digit holding the k-th key; then a per-chunk count pass, a 1-block scan giving every chunk its
// output offset and tie allotment (ties go to the lowest indices), and an ordered-compaction pass
// that writes idx/val and applies the counter / rewind side effects.
#include "dpz_topk.h"

namespace dpz {

template <bool VEC, int P>
__global__ void __launch_bounds__(256) exact_hist_kernel(KeySrc s, int64_t n, const TopkCtrl* ctrl,
                                                         uint32_t* ghist, int store_acc) {
  constexpr int NB = (P == 1) ? 2048 : 1024;
  __shared__ uint32_t h[NB];
  for (int b = threadIdx.x; b < NB; b += 256) h[b] = 0;
  __syncthreads();
  const uint32_t pfx = (P == 0) ? 0u : ctrl->prefix;
  const int64_t ngroups = (n + 3) >> 2;
  for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < ngroups;
       g += (int64_t)gridDim.x * 256) {
    uint32_t key[4];
    const int cnt = load_keys4<VEC>(s, g * 4, n, store_acc != 0, key);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (e < cnt) {
        const uint32_t kk = key[e];
        if (P == 0) {
          atomicAdd(&h[kk >> 21], 1u);
        } else if (P == 1) {
          if ((kk >> 21) == (pfx >> 21)) atomicAdd(&h[(kk >> 10) & 2047u], 1u);
        } else {
          if ((kk >> 10) == (pfx >> 10)) atomicAdd(&h[kk & 1023u], 1u);
        }
      }
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < NB; b += 256) {
    const uint32_t v = h[b];
    if (v) atomicAdd(&ghist[b], v);
  }
}

// One block of 1024 threads: pick the digit holding the krem-th largest key.
template <int P>
__global__ void __launch_bounds__(1024) exact_resolve_kernel(TopkCtrl* ctrl, const uint32_t* ghist,
                                                             uint32_t k) {
  constexpr int NB = (P == 1) ? 2048 : 1024;
  constexpr int SH = (P == 0) ? 21 : (P == 1 ? 10 : 0);
  constexpr int PER = NB / 1024;
  __shared__ uint32_t wsum[16];
  const uint32_t krem = (P == 0) ? k : ctrl->krem;
  const uint32_t pfx = (P == 0) ? 0u : ctrl->prefix;
  // thread t owns descending positions j = t*PER .. t*PER+PER-1, bin = NB-1-j
  uint32_t hv[PER];
  uint32_t local = 0;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    hv[q] = ghist[NB - 1 - (threadIdx.x * PER + q)];
    local += hv[q];
  }
  uint32_t tot;
  uint32_t before = block_excl_scan(local, wsum, &tot);
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    if (before < krem && krem <= before + hv[q]) {
      const uint32_t d = NB - 1 - (threadIdx.x * PER + q);
      ctrl->prefix = pfx | (d << SH);
      ctrl->krem = krem - before;
    }
    before += hv[q];
  }
}

template <bool VEC>
__global__ void __launch_bounds__(256) exact_count_kernel(KeySrc s, int64_t n, const TopkCtrl* ctrl,
                                                          uint32_t* blk_gt, uint32_t* blk_eq) {
  __shared__ uint32_t wsum[16];
  const uint32_t T = ctrl->prefix;
  const int64_t lo = (int64_t)blockIdx.x * EX_CHUNK;
  uint32_t gt = 0, eq = 0;
  for (int r = 0; r < EX_CHUNK / 1024; ++r) {
    const int64_t i0 = lo + r * 1024 + threadIdx.x * 4;
    if (i0 >= n) break;
    uint32_t key[4];
    const int cnt = load_keys4<VEC>(s, i0, n, false, key);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (e < cnt) {
        gt += key[e] > T;
        eq += key[e] == T;
      }
    }
  }
  uint32_t tg, te;
  block_excl_scan(gt, wsum, &tg);
  block_excl_scan(eq, wsum, &te);
  if (threadIdx.x == 0) {
    blk_gt[blockIdx.x] = tg;
    blk_eq[blockIdx.x] = te;
  }
}

// One block of 1024 threads: per-block output offsets and tie allotments (in index order).
// Ties taken at the threshold T = ctrl->prefix: the k-th-key tie allotment (top-k), or with
// keep_ties (threshold selection, reference sharing/Choco.py:117-140) every tie — except when
// T == 0, where exact zeros are not selected (Choco sends nonzero(q), Choco.py:148-161).
__device__ __forceinline__ uint32_t exact_ties(const TopkCtrl* ctrl, int keep_ties) {
  if (!keep_ties) return ctrl->krem;
  return ctrl->prefix == 0u ? 0u : 0xFFFFFFFFu;
}

__global__ void __launch_bounds__(1024) exact_scan_kernel(TopkCtrl* ctrl, int64_t nblk,
                                                          const uint32_t* blk_gt,
                                                          const uint32_t* blk_eq, uint32_t* blk_off,
                                                          uint32_t* blk_eqb, int keep_ties) {
  __shared__ uint64_t wsum[16];
  const uint64_t ties = exact_ties(ctrl, keep_ties);
  uint64_t carry_eq = 0, carry_off = 0;
  for (int64_t base = 0; base < nblk; base += 1024) {
    const int64_t b = base + threadIdx.x;
    const uint64_t gt = b < nblk ? blk_gt[b] : 0;
    const uint64_t eq = b < nblk ? blk_eq[b] : 0;
    uint64_t te;
    const uint64_t eqb = block_excl_scan64(eq, wsum, &te) + carry_eq;
    uint64_t take = 0;
    if (ties > eqb) take = (ties - eqb) < eq ? (ties - eqb) : eq;
    uint64_t ts;
    const uint64_t off = block_excl_scan64(gt + take, wsum, &ts) + carry_off;
    if (b < nblk) {
      blk_off[b] = (uint32_t)off;
      blk_eqb[b] = (uint32_t)(eqb < ties ? eqb : ties);
    }
    carry_eq += te;
    carry_off += ts;
  }
  if (threadIdx.x == 0) ctrl->nbound = (uint32_t)carry_off;  // entries selected in total
}

template <bool VEC>
__global__ void __launch_bounds__(256) exact_write_kernel(KeySrc s, int64_t n, const TopkCtrl* ctrl,
                                                          const uint32_t* blk_off,
                                                          const uint32_t* blk_eqb,
                                                          const float* vals_src, int32_t* idx_out,
                                                          float* val_out, int32_t* counter,
                                                          float* rewind, int64_t k,
                                                          int keep_ties, int val_h) {
  __shared__ uint32_t wsum[16];
  const uint32_t T = ctrl->prefix;
  const uint32_t ties = exact_ties(ctrl, keep_ties);
  const uint32_t off0 = blk_off[blockIdx.x];
  const uint32_t eqb = blk_eqb[blockIdx.x];
  const uint32_t quota = ties > eqb ? ties - eqb : 0u;
  const int64_t lo = (int64_t)blockIdx.x * EX_CHUNK;
  uint32_t gt_run = 0, eq_run = 0;
  for (int r = 0; r < EX_CHUNK / 1024; ++r) {
    const int64_t i0 = lo + r * 1024 + threadIdx.x * 4;
    if (lo + r * 1024 >= n) break;  // uniform
    uint32_t key[4];
    const int cnt = load_keys4<VEC>(s, i0, n, false, key);
    uint32_t ng = 0, ne = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (e < cnt) {
        ng += key[e] > T;
        ne += key[e] == T;
      }
    }
    uint32_t tot;
    const uint32_t ex = block_excl_scan((ne << 16) | ng, wsum, &tot);
    uint32_t g = gt_run + (ex & 0xFFFFu);
    uint32_t q = eq_run + (ex >> 16);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (e < cnt) {
        bool sel = false;
        uint32_t pos = 0;
        if (key[e] > T) {
          sel = true;
          pos = off0 + g + (q < quota ? q : quota);
          ++g;
        } else if (key[e] == T) {
          if (q < quota) {
            sel = true;
            pos = off0 + g + q;
          }
          ++q;
        }
        if (sel && pos < (uint64_t)k) {
          const int64_t i = i0 + e;
          idx_out[pos] = (int32_t)i;
          store_val(val_out, val_h, pos, vals_src[i]);
          if (counter) counter[i] += 1;
          if (rewind) rewind[i] = 0.0f;
        }
      }
    }
    gt_run += tot & 0xFFFFu;
    eq_run += tot >> 16;
  }
}

template <bool VEC>
static int run_exact_t(const EncodeArgs& a, const WsLayout& L, int rekey, int keep_ties,
                       int64_t cap) {
  KeySrc s{a.x, a.x0, a.acc, a.acc_mode, rekey};
  TopkCtrl* ctrl = reinterpret_cast<TopkCtrl*>(a.ws + L.ctrl);
  uint32_t* hist = reinterpret_cast<uint32_t*>(a.ws + L.ex_hist);
  DPZ_HIP_TRY(hipMemsetAsync(a.ws + L.ctrl, 0, sizeof(TopkCtrl), a.st));
  DPZ_HIP_TRY(hipMemsetAsync(a.ws + L.ex_hist, 0, 4096 * 4, a.st));
  const int64_t groups = (a.n + 3) / 4;
  int hb = (int)((groups + 255) / 256);
  if (hb > EX_HIST_BLOCKS) hb = EX_HIST_BLOCKS;
  if (hb < 1) hb = 1;
  const int store_acc = (a.acc_mode == DPZ_ACC_ACCUMULATE && !rekey) ? 1 : 0;
  DPZ_TIMED(DPZ_KT_EXACT_HIST, a.st, exact_hist_kernel<VEC, 0><<<hb, 256, 0, a.st>>>(s, a.n, ctrl, hist, store_acc));
  s.rekey = 1;
  DPZ_TIMED(DPZ_KT_EXACT_RESOLVE, a.st, exact_resolve_kernel<0><<<1, 1024, 0, a.st>>>(ctrl, hist, (uint32_t)a.k));
  DPZ_TIMED(DPZ_KT_EXACT_HIST, a.st, exact_hist_kernel<VEC, 1><<<hb, 256, 0, a.st>>>(s, a.n, ctrl, hist + 1024, 0));
  DPZ_TIMED(DPZ_KT_EXACT_RESOLVE, a.st, exact_resolve_kernel<1><<<1, 1024, 0, a.st>>>(ctrl, hist + 1024, (uint32_t)a.k));
  DPZ_TIMED(DPZ_KT_EXACT_HIST, a.st, exact_hist_kernel<VEC, 2><<<hb, 256, 0, a.st>>>(s, a.n, ctrl, hist + 3072, 0));
  DPZ_TIMED(DPZ_KT_EXACT_RESOLVE, a.st, exact_resolve_kernel<2><<<1, 1024, 0, a.st>>>(ctrl, hist + 3072, (uint32_t)a.k));
  uint32_t* bgt = reinterpret_cast<uint32_t*>(a.ws + L.ex_gt);
  uint32_t* beq = reinterpret_cast<uint32_t*>(a.ws + L.ex_eq);
  uint32_t* boff = reinterpret_cast<uint32_t*>(a.ws + L.ex_off);
  uint32_t* beqb = reinterpret_cast<uint32_t*>(a.ws + L.ex_eqb);
  DPZ_TIMED(DPZ_KT_EXACT_COUNT, a.st, exact_count_kernel<VEC><<<(unsigned)L.ex_nblk, 256, 0, a.st>>>(s, a.n, ctrl, bgt, beq));
  DPZ_TIMED(DPZ_KT_EXACT_SCAN, a.st, exact_scan_kernel<<<1, 1024, 0, a.st>>>(ctrl, L.ex_nblk, bgt, beq, boff, beqb, keep_ties));
  // sliced side effects (dpz_topk_encode_sliced): no rewind here, the caller applies selmask
  float* rewind = (a.acc && a.acc_mode != DPZ_ACC_NONE && !a.selmask) ? a.acc : nullptr;
  DPZ_TIMED(DPZ_KT_EXACT_WRITE, a.st, exact_write_kernel<VEC><<<(unsigned)L.ex_nblk, 256, 0, a.st>>>(
      s, a.n, ctrl, boff, beqb, a.vals_src, a.idx_out, a.val_out, a.counter, rewind,
      keep_ties ? cap : a.k, keep_ties, a.val_h));
  return DPZ_OK;
}


int run_exact(const EncodeArgs& a, const WsLayout& L, int rekey, bool vec, int keep_ties,
              int64_t cap) {
  return vec ? run_exact_t<true>(a, L, rekey, keep_ties, cap)
             : run_exact_t<false>(a, L, rekey, keep_ties, cap);
}

}  // namespace dpz
