// Top-k magnitude encode for the decentralizepy Sharing plugins (PartialModel / Wavelet / JWINS).
//
// Replaces (reference sacs-epfl/decentralizepy, src/decentralizepy/):
//   sharing/PartialModel.py:164-186  extract_top_gradients: |change|, torch.topk, torch.sort(index)
//   sharing/PartialModel.py:205-246  counter[idx] += 1, rewind_accumulation(idx), x[idx]
//   sharing/PartialModel.py:305-331  _pre_step change / accumulation (fused into the first pass)
//   sharing/JWINS/Wavelet.py:142-197 apply_wavelet + the same bookkeeping on coefficients
//
// Selection rule: the k largest uint32 keys (|change| bits, sign cleared, NaN canonical), ties at
// the k-th key broken by lowest index; output in ascending index order (no sort is needed:
// compaction preserves index order).
//
// Two device paths:
//  * EXACT  — three radix histogram passes (10/11/10 bits) resolve the k-th key T and the number
//             of ties to take, then a count pass, a 1-block scan and an ordered-compaction pass.
//             Works for every n, k (also k = n, heavy ties, NaN).  ~5 reads of the key stream.
//  * SAMPLED (k <= n/16, n >= 2^18) — one read of the inputs, four launches
//             (dpz_topk_sampled.hip): sample -> filter (window [lo, hi) around the k-th key,
//             candidates >= lo appended per wave segment in index order, window histogram) ->
//             select (threshold bin b*, per-block counts above it, bin-b* boundary list) ->
//             compact (exact T and tie cut resolved redundantly per block, ordered write of
//             idx/val + counter / rewind side effects).
//    Any miss (window did not bracket the k-th key, boundary overflow) sets ctrl->status; the
//    compact kernel then writes nothing and the host re-runs the EXACT path with keys re-derived
//    from the post-filter state ("rekey").  A segment whose candidates overflow its list is marked
//    dense and re-reads its own input range in select / compact instead (still exact).
#include "dpz_topk.h"

namespace dpz {

// acc += x - x0 only (k == 0 with accumulation: the reference still accumulates).
template <bool VEC>
__global__ void __launch_bounds__(256) accumulate_only_kernel(KeySrc s, int64_t n) {
  const int64_t ngroups = (n + 3) >> 2;
  for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < ngroups;
       g += (int64_t)gridDim.x * 256) {
    uint32_t key[4];
    load_keys4<VEC>(s, g * 4, n, true, key);
  }
}

// ================================================================================================
// host side
// ================================================================================================
template <bool VEC>
static int run_accumulate_only(const EncodeArgs& a) {
  KeySrc s{a.x, a.x0, a.acc, a.acc_mode, 0};
  const int64_t groups = (a.n + 3) / 4;
  int nb = (int)((groups + 255) / 256);
  if (nb > 4096) nb = 4096;
  if (nb < 1) nb = 1;
  DPZ_TIMED(DPZ_KT_ACCUMULATE, a.st, accumulate_only_kernel<VEC><<<nb, 256, 0, a.st>>>(s, a.n));
  return DPZ_OK;
}

static bool all_aligned(const EncodeArgs& a) {
  auto al = [](const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15u) == 0; };
  return al(a.x) && al(a.x0) && al(a.acc) && al(a.vals_src);
}

static int validate(const EncodeArgs& a, size_t ws_bytes) {
  if (a.n < 0 || a.k < 0 || a.k > a.n || a.n >= (int64_t(1) << 31)) return DPZ_ERR_ARG;
  if (a.acc_mode < DPZ_ACC_NONE || a.acc_mode > DPZ_ACC_ADD) return DPZ_ERR_ARG;
  if (a.n > 0 && !a.x) return DPZ_ERR_ARG;
  if (a.acc_mode != DPZ_ACC_NONE && !a.acc) return DPZ_ERR_ARG;
  if (a.k > 0 && (!a.idx_out || !a.val_out || !a.vals_src)) return DPZ_ERR_ARG;
  if (a.n > 0 && (!a.ws || ws_bytes < ws_bytes_needed(a.n, a.k))) return DPZ_ERR_WORKSPACE;
  return DPZ_OK;
}

}  // namespace dpz

using namespace dpz;

extern "C" size_t dpz_topk_workspace_bytes(int64_t n, int64_t k) {
  (void)k;
  return ws_bytes_needed(n > 0 ? n : 1, k);
}

static int dpz_topk_dispatch(EncodeArgs a, int flags) {
  if (flags & DPZ_TOPK_SHARED) a.shared = true;
  if (flags & DPZ_TOPK_VAL_FP16) a.val_h = 1;
  if (flags & DPZ_TOPK_KEEP_X) a.keep_x = true;
  // a prior-round window (DPZ_TOPK_HINT): not with ACCUMULATE, whose first pass stores acc (a
  // missed call could not simply be re-run on the sampled path)
  if ((flags & DPZ_TOPK_HINT) && a.acc_mode != DPZ_ACC_ACCUMULATE)
    a.hint_sig = hint_signature(a.n, a.k, a.shared, a.acc_mode, a.x0 != nullptr);
  const WsLayout L = ws_layout(a.n, a.k, a.shared);
  const bool vec = all_aligned(a);
  if (a.k == 0) {
    if (a.acc_mode == DPZ_ACC_ACCUMULATE && a.n > 0)
      return vec ? run_accumulate_only<true>(a) : run_accumulate_only<false>(a);
    return DPZ_OK;
  }
  const int phases = (flags & DPZ_TOPK_STREAM) ? 1 : ((flags & DPZ_TOPK_TAIL) ? 2 : 3);
  if (phases != 3) flags |= DPZ_TOPK_ASYNC;
  if (!(flags & DPZ_TOPK_EXACT) && use_sampled(a.n, a.k)) {
    int rc = run_sampled(a, L, vec, phases);
    if (rc != DPZ_OK) return rc;
    if (flags & DPZ_TOPK_ASYNC) return DPZ_OK;
    int fb = 0;
    return dpz_topk_complete(a.x, a.x0, a.acc, a.acc_mode, a.vals_src, a.n, a.k, a.idx_out,
                             a.val_out, a.counter, a.ws, ws_bytes_needed(a.n, a.k), &fb, a.st);
  }
  if (phases == 2) return DPZ_OK;  // the exact path ran whole in the STREAM call
  int rc = run_exact(a, L, 0, vec);
  if (rc != DPZ_OK) return rc;
  if (!(flags & DPZ_TOPK_ASYNC)) DPZ_HIP_TRY(hipStreamSynchronize(a.st));
  return DPZ_OK;
}

extern "C" int dpz_topk_encode(const float* x, const float* x0, float* acc, int acc_mode,
                               const float* vals_src, int64_t n, int64_t k, int32_t* idx_out,
                               float* val_out, int32_t* counter, void* ws, size_t ws_bytes,
                               int flags, dpz_stream_t stream) {
  EncodeArgs a{x, x0, acc, acc_mode, vals_src, n, k, idx_out, val_out, counter,
               static_cast<char*>(ws), static_cast<hipStream_t>(stream)};
  int rc = validate(a, ws_bytes);
  if (rc != DPZ_OK) return rc;
  if (n == 0) return DPZ_OK;
  return dpz_topk_dispatch(a, flags);
}

namespace dpz {
int topk_encode_status(const float* x, const float* x0, float* acc, int acc_mode,
                       const float* vals_src, int64_t n, int64_t k, int32_t* idx_out,
                       float* val_out, int32_t* counter, void* ws, size_t ws_bytes,
                       hipStream_t st, int32_t* status_out, bool shared, bool val_fp16,
                       bool hint) {
  EncodeArgs a{x, x0, acc, acc_mode, vals_src, n, k, idx_out, val_out, counter,
               static_cast<char*>(ws), st};
  a.shared = shared;
  a.val_h = val_fp16 ? 1 : 0;
  int rc = validate(a, ws_bytes);
  if (rc != DPZ_OK) return rc;
  if (n == 0 || k == 0 || !use_sampled(n, k)) {  // no sampled tail writes it: status 0
    if (n > 0) rc = dpz_topk_dispatch(a, DPZ_TOPK_ASYNC | (val_fp16 ? DPZ_TOPK_VAL_FP16 : 0));
    if (rc != DPZ_OK) return rc;
    if (status_out) DPZ_HIP_TRY(hipMemsetAsync(status_out, 0, sizeof(int32_t), st));
    return DPZ_OK;
  }
  a.status_out = status_out;
  return dpz_topk_dispatch(a, DPZ_TOPK_ASYNC | (val_fp16 ? DPZ_TOPK_VAL_FP16 : 0) |
                                  (hint ? DPZ_TOPK_HINT : 0));
}
}  // namespace dpz

extern "C" int dpz_topk_encode_status(const float* x, const float* x0, float* acc, int acc_mode,
                                      const float* vals_src, int64_t n, int64_t k,
                                      int32_t* idx_out, float* val_out, int32_t* counter,
                                      void* ws, size_t ws_bytes, int32_t* status_out,
                                      int flags, dpz_stream_t stream) {
  if (!status_out) return DPZ_ERR_ARG;
  // only DPZ_TOPK_SHARED applies (the call is asynchronous, sampled-path, unsplit by contract)
  if (flags & ~(DPZ_TOPK_SHARED | DPZ_TOPK_VAL_FP16)) return DPZ_ERR_ARG;
  return topk_encode_status(x, x0, acc, acc_mode, vals_src, n, k, idx_out, val_out, counter, ws,
                            ws_bytes, static_cast<hipStream_t>(stream), status_out,
                            (flags & DPZ_TOPK_SHARED) != 0, (flags & DPZ_TOPK_VAL_FP16) != 0);
}

static bool overlaps(const void* p, size_t pb, const void* q, size_t qb) {
  if (!p || !q || pb == 0 || qb == 0) return false;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p), b = reinterpret_cast<uintptr_t>(q);
  return a < b + qb && b < a + pb;
}

extern "C" int dpz_topk_encode_foldbase(const float* x, const float* x0, float* acc, int acc_mode,
                                        const float* vals_src, int64_t n, int64_t k,
                                        int32_t* idx_out, float* val_out, int32_t* counter,
                                        void* ws, size_t ws_bytes, int flags, int n_weights,
                                        const float* w, float w_self, float* base_out,
                                        dpz_stream_t stream) {
  EncodeArgs a{x, x0, acc, acc_mode, vals_src, n, k, idx_out, val_out, counter,
               static_cast<char*>(ws), static_cast<hipStream_t>(stream)};
  int rc = validate(a, ws_bytes);
  if (rc != DPZ_OK) return rc;
  if (flags & (DPZ_TOPK_STREAM | DPZ_TOPK_TAIL)) return DPZ_ERR_ARG;
  if (n_weights < 1 || n_weights > FOLDBASE_MAXW || !w) return DPZ_ERR_ARG;
  if (n > 0 && !base_out) return DPZ_ERR_ARG;
  // the base is an output of its own: it may not overlap anything the encode reads or writes
  const size_t nb = (size_t)n * 4;
  if (overlaps(base_out, nb, x, nb) || overlaps(base_out, nb, x0, nb) ||
      overlaps(base_out, nb, acc, nb) || overlaps(base_out, nb, vals_src, nb) ||
      overlaps(base_out, nb, counter, nb) || overlaps(base_out, nb, idx_out, (size_t)k * 4) ||
      overlaps(base_out, nb, val_out, (size_t)k * 4) || overlaps(base_out, nb, ws, ws_bytes))
    return DPZ_ERR_ARG;
  if (n == 0) return DPZ_OK;
  FoldBase fb{};
  fb.nw = n_weights;
  for (int i = 0; i < n_weights; ++i) fb.w[i] = w[i];
  fb.ws = w_self;
  a.fbase = &fb;
  a.base_out = base_out;
  if (!(flags & DPZ_TOPK_EXACT) && k > 0 && fused_foldbase_ok(a, all_aligned(a)))
    return dpz_topk_dispatch(a, flags);  // the filter writes the base as it streams x
  rc = launch_fold_base(x, n, fb, base_out, a.st);
  if (rc != DPZ_OK) return rc;
  a.fbase = nullptr;
  a.base_out = nullptr;
  return dpz_topk_dispatch(a, flags);
}

extern "C" int dpz_topk_encode_replace(const float* x, const float* x0, float* acc, int acc_mode,
                                       const float* vals_src, int64_t n, int64_t k,
                                       int32_t* idx_out, float* val_out, int32_t* counter,
                                       void* ws, size_t ws_bytes, int flags,
                                       const float* r_local, const int32_t* r_idx,
                                       const float* r_val, int64_t r_k, int64_t r_n, float* r_out,
                                       void* r_ws, size_t r_ws_bytes, dpz_stream_t stream) {
  EncodeArgs a{x, x0, acc, acc_mode, vals_src, n, k, idx_out, val_out, counter,
               static_cast<char*>(ws), static_cast<hipStream_t>(stream)};
  int rc = validate(a, ws_bytes);
  if (rc != DPZ_OK) return rc;
  if (flags & (DPZ_TOPK_STREAM | DPZ_TOPK_TAIL)) return DPZ_ERR_ARG;
  if (r_n <= 0 || r_k < 0 || r_k > r_n || !r_local || !r_out) return DPZ_ERR_ARG;
  if (r_k > 0 && (!r_idx || !r_val)) return DPZ_ERR_ARG;
  // the replace job is independent work: its output may not overlap anything the encode touches
  const size_t ob = (size_t)r_n * 4;
  if (overlaps(r_out, ob, r_local, ob) || overlaps(r_out, ob, x, (size_t)n * 4) ||
      overlaps(r_out, ob, x0, (size_t)n * 4) || overlaps(r_out, ob, acc, (size_t)n * 4) ||
      overlaps(r_out, ob, vals_src, (size_t)n * 4) || overlaps(r_out, ob, counter, (size_t)n * 4) ||
      overlaps(r_out, ob, idx_out, (size_t)k * 4) || overlaps(r_out, ob, val_out, (size_t)k * 4) ||
      overlaps(r_out, ob, ws, ws_bytes) || overlaps(r_out, ob, r_ws, r_ws_bytes))
    return DPZ_ERR_ARG;
  ReplaceJob job{r_local, r_idx, r_val, r_k, r_n, r_out, 0, replace_chunks(r_k), 0};
  const bool r_vec = ((reinterpret_cast<uintptr_t>(r_local) | reinterpret_cast<uintptr_t>(r_out)) & 15u) == 0;
  const bool carried = n > 0 && k > 0 && r_k > 0 && r_vec && !(flags & DPZ_TOPK_EXACT) &&
                       use_sampled(n, k);
  // Decoding over the very tensor being encoded (reference: deserialized_model starts from the
  // node's current state_dict, the model its serialized_model just encoded): the filter, which
  // streams x anyway, writes out = x, and only the payload entries are scattered afterwards —
  // 4n bytes of reads fewer than an independent replace (DPZ_FUSED_COPY=0 disables it in the
  // diagnostic build, A/B).
  if (carried && DPZ_KNOB_INT(FUSED_COPY, 1) != 0 && r_local == x && r_n == n &&
      acc_mode == DPZ_ACC_NONE) {
    job.scatter = 1;
    job.c1 = scatter_chunks(r_k);
  }
  if (!carried) {  // run it on its own first (same stream), then the plain encode
    const float* vp = r_val;
    const int32_t* ip = r_idx;
    const int64_t kk = r_k;
    rc = dpz_decode_average(r_local, r_n, 1, &ip, &vp, &kk, nullptr, 0.0f, DPZ_FOLD_REPLACE_ONLY,
                            r_out, r_ws, r_ws_bytes, stream);
    if (rc != DPZ_OK) return rc;
    if (n == 0) return DPZ_OK;
    return dpz_topk_dispatch(a, flags);
  }
  a.job = &job;
  return dpz_topk_dispatch(a, flags);
}

// ---- coalesced side effects (dpz_topk_encode_sliced) ------------------------------------------
namespace dpz {

static unsigned grid_of(int64_t items, int64_t cap = 8192) {
  int64_t g = (items + 255) / 256;
  if (g > cap) g = cap;
  return (unsigned)(g < 1 ? 1 : g);
}

// bit idx of mask for every selected index (the exact path / a sampled miss: the sorted indices
// are unique, the atomics go to distinct bits).  guard: the sampled run's status word — after a
// miss compact wrote nothing and idx holds whatever the buffer held before, so nothing is read;
// an index outside [0, n) is never followed either
__global__ void __launch_bounds__(256) selmask_from_idx_kernel(const int32_t* __restrict__ idx,
                                                               int64_t k, int64_t n,
                                                               uint32_t* mask,
                                                               const uint32_t* guard) {
  if (guard && *guard) return;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < k; i += (int64_t)gridDim.x * 256) {
    const uint32_t v = (uint32_t)idx[i];
    if ((int64_t)v < n) atomicOr(&mask[v >> 5], 1u << (v & 31));
  }
}

// planes += mask, word by word (ripple carry over the bit planes; stops at the first plane with
// no carry left, usually within two or three)
__global__ void __launch_bounds__(256) planes_add_kernel(uint32_t* planes,
                                                         const uint32_t* __restrict__ mask,
                                                         int64_t nw, const uint32_t* guard) {
  if (guard && *guard) return;
  for (int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x; w < nw; w += (int64_t)gridDim.x * 256) {
    uint32_t carry = mask[w];
    for (int p = 0; p < 32 && carry != 0u; p += 4) {  // four planes' words read together
      uint32_t o[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = planes[(int64_t)(p + q) * nw + w];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (carry != 0u) {
          planes[(int64_t)(p + q) * nw + w] = o[q] ^ carry;
          carry &= o[q];
        }
      }
    }
  }
}

// counter[i] = sum_p bit(planes[p][i / 32], i % 32) << p
__global__ void __launch_bounds__(256) counter_unslice_kernel(const uint32_t* __restrict__ planes,
                                                              int64_t n, int64_t nw,
                                                              int32_t* out) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t w = i >> 5;
    const uint32_t b = (uint32_t)(i & 31);
    uint32_t v = 0;
#pragma unroll 8
    for (int p = 0; p < 32; ++p) v |= ((planes[(int64_t)p * nw + w] >> b) & 1u) << p;
    out[i] = (int32_t)v;
  }
}

// planes from an int32 counter: one word (32 counters) per thread
__global__ void __launch_bounds__(256) counter_slice_kernel(const int32_t* __restrict__ c,
                                                            int64_t n, int64_t nw,
                                                            uint32_t* planes) {
  for (int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x; w < nw; w += (int64_t)gridDim.x * 256) {
    uint32_t v[32];
#pragma unroll
    for (int b = 0; b < 32; ++b) {
      const int64_t i = w * 32 + b;
      v[b] = i < n ? (uint32_t)c[i] : 0u;
    }
#pragma unroll
    for (int p = 0; p < 32; ++p) {
      uint32_t word = 0;
#pragma unroll
      for (int b = 0; b < 32; ++b) word |= ((v[b] >> p) & 1u) << b;
      planes[(int64_t)p * nw + w] = word;
    }
  }
}

// acc[i] = 0 where the mask bit is set (the deferred rewind on its own)
__global__ void __launch_bounds__(256) rewind_apply_kernel(float* acc,
                                                           const uint32_t* __restrict__ mask,
                                                           int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    if ((mask[i >> 5] >> (i & 31)) & 1u) acc[i] = 0.0f;
}

int sliced_from_idx(const EncodeArgs& a, const uint32_t* guard) {
  const int64_t nw = mask_words(a.n);
  DPZ_HIP_TRY(hipMemsetAsync(a.selmask, 0, (size_t)nw * 4, a.st));
  if (a.k > 0)
    DPZ_TIMED(DPZ_KT_TOPK_COMPACT, a.st,
              selmask_from_idx_kernel<<<grid_of(a.k), 256, 0, a.st>>>(a.idx_out, a.k, a.n,
                                                                      a.selmask, guard));
  if (a.planes && a.k > 0)
    DPZ_TIMED(DPZ_KT_TOPK_COMPACT, a.st,
              planes_add_kernel<<<grid_of(nw), 256, 0, a.st>>>(a.planes, a.selmask, nw, guard));
  return DPZ_OK;
}

}  // namespace dpz

extern "C" int64_t dpz_mask_words(int64_t n) { return n > 0 ? mask_words(n) : 0; }

extern "C" int dpz_topk_encode_sliced(const float* x, const float* x0, const float* acc,
                                      int acc_mode, const float* vals_src, int64_t n, int64_t k,
                                      int32_t* idx_out, float* val_out, uint32_t* planes,
                                      uint32_t* sel_mask, void* ws, size_t ws_bytes,
                                      int32_t* status_out, int flags, dpz_stream_t stream) {
  if (acc_mode != DPZ_ACC_NONE && acc_mode != DPZ_ACC_ADD) return DPZ_ERR_ARG;
  if (flags & ~(DPZ_TOPK_EXACT | DPZ_TOPK_SHARED | DPZ_TOPK_VAL_FP16 | DPZ_TOPK_HINT))
    return DPZ_ERR_ARG;
  // acc is only read (ADD): the rewind is the caller's, through sel_mask
  EncodeArgs a{x, x0, const_cast<float*>(acc), acc_mode, vals_src, n, k, idx_out, val_out, nullptr,
               static_cast<char*>(ws), static_cast<hipStream_t>(stream)};
  int rc = validate(a, ws_bytes);
  if (rc != DPZ_OK) return rc;
  if (n > 0 && !sel_mask) return DPZ_ERR_ARG;
  const size_t mb = (size_t)mask_words(n) * 4;
  if (overlaps(sel_mask, mb, planes, mb * 32) || overlaps(sel_mask, mb, ws, ws_bytes) ||
      overlaps(planes, mb * 32, ws, ws_bytes))
    return DPZ_ERR_ARG;
  a.shared = (flags & DPZ_TOPK_SHARED) != 0;
  a.val_h = (flags & DPZ_TOPK_VAL_FP16) ? 1 : 0;
  a.selmask = sel_mask;
  a.planes = planes;
  // a prior-round window (DPZ_TOPK_HINT): the keys (NONE / ADD) are a pure function of the
  // inputs and a miss writes nothing, so a missed call simply runs the sampled path again
  if (flags & DPZ_TOPK_HINT)
    a.hint_sig = hint_signature(a.n, a.k, a.shared, a.acc_mode, a.x0 != nullptr);
  if (n == 0) {
    if (status_out) DPZ_HIP_TRY(hipMemsetAsync(status_out, 0, sizeof(int32_t), a.st));
    return DPZ_OK;
  }
  const WsLayout L = ws_layout(n, k, a.shared);
  const bool vec = all_aligned(a);
  if (!(flags & DPZ_TOPK_EXACT) && use_sampled(n, k)) {
    // segments of at most SL_RMAX elements: compact writes the mask words and the planes from
    // its LDS rows; longer ones (n > SL_RMAX * W_MAX): compact writes idx / val only and the
    // mask and planes are built from idx_out after it (skipped on the device after a miss)
    const bool post = L.fg.R > SL_RMAX;
    a.status_out = status_out;
    const uint32_t* ctrl_status =
        reinterpret_cast<const uint32_t*>(a.ws + L.ctrl + offsetof(TopkCtrl, status));
    // blocking: a hinted call that misses runs the sampled path once more (its own sample
    // launch), then the exact path; asynchronous: the caller re-runs with EXACT
    for (int pass = 0; pass < (a.hint_sig && !status_out ? 2 : 1); ++pass) {
      if (pass == 1) a.hint_sig = 0u;
      rc = run_sampled(a, L, vec, 3);
      if (rc != DPZ_OK) return rc;
      if (post) {
        rc = sliced_from_idx(a, ctrl_status);
        if (rc != DPZ_OK) return rc;
      }
      if (status_out) return DPZ_OK;  // asynchronous: a nonzero status -> re-run with EXACT
      DPZ_HIP_TRY(hipStreamSynchronize(a.st));
      uint32_t st = 0;
      DPZ_HIP_TRY(hipMemcpy(&st, ctrl_status, sizeof(st), hipMemcpyDeviceToHost));
      if (st == 0) return DPZ_OK;
    }
    a.status_out = nullptr;  // the miss wrote nothing: the exact path below
  }
  if (k > 0) {
    rc = run_exact(a, L, 0, vec);
    if (rc != DPZ_OK) return rc;
  }
  rc = sliced_from_idx(a);
  if (rc != DPZ_OK) return rc;
  if (status_out) DPZ_HIP_TRY(hipMemsetAsync(status_out, 0, sizeof(int32_t), a.st));
  else DPZ_HIP_TRY(hipStreamSynchronize(a.st));
  return DPZ_OK;
}

extern "C" int dpz_counter_slice(const int32_t* counter, int64_t n, uint32_t* planes,
                                 dpz_stream_t stream) {
  if (n < 0 || (n > 0 && (!counter || !planes))) return DPZ_ERR_ARG;
  if (n == 0) return DPZ_OK;
  const int64_t nw = mask_words(n);
  hipStream_t st = static_cast<hipStream_t>(stream);
  counter_slice_kernel<<<grid_of(nw), 256, 0, st>>>(counter, n, nw, planes);
  DPZ_HIP_TRY(hipGetLastError());
  return DPZ_OK;
}

extern "C" int dpz_counter_unslice(const uint32_t* planes, int64_t n, int32_t* counter,
                                   dpz_stream_t stream) {
  if (n < 0 || (n > 0 && (!counter || !planes))) return DPZ_ERR_ARG;
  if (n == 0) return DPZ_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  counter_unslice_kernel<<<grid_of(n), 256, 0, st>>>(planes, n, mask_words(n), counter);
  DPZ_HIP_TRY(hipGetLastError());
  return DPZ_OK;
}

extern "C" int dpz_rewind_apply(float* acc, const uint32_t* sel_mask, int64_t n,
                                dpz_stream_t stream) {
  if (n < 0 || (n > 0 && (!acc || !sel_mask))) return DPZ_ERR_ARG;
  if (n == 0) return DPZ_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  rewind_apply_kernel<<<grid_of(n), 256, 0, st>>>(acc, sel_mask, n);
  DPZ_HIP_TRY(hipGetLastError());
  return DPZ_OK;
}

extern "C" int dpz_topk_threshold(const float* x, int64_t n, int64_t k, int32_t* idx_out,
                                  float* val_out, int64_t cap, void* ws, size_t ws_bytes,
                                  int64_t* count, dpz_stream_t stream) {
  EncodeArgs a{x, nullptr, nullptr, DPZ_ACC_NONE, x, n, k, idx_out, val_out, nullptr,
               static_cast<char*>(ws), static_cast<hipStream_t>(stream)};
  if (cap < 0 || !count) return DPZ_ERR_ARG;
  int rc = validate(a, ws_bytes);
  if (rc != DPZ_OK) return rc;
  *count = 0;
  if (n == 0) return DPZ_OK;
  if (cap > 0 && (!idx_out || !val_out)) return DPZ_ERR_ARG;
  const WsLayout L = ws_layout(n, k);
  rc = run_exact(a, L, 0, all_aligned(a), 1, cap);
  if (rc != DPZ_OK) return rc;
  uint32_t c = 0;
  DPZ_HIP_TRY(hipMemcpyAsync(&c, a.ws + L.ctrl + offsetof(TopkCtrl, nbound), sizeof(c),
                             hipMemcpyDeviceToHost, a.st));
  DPZ_HIP_TRY(hipStreamSynchronize(a.st));
  *count = c;
  return c > (uint64_t)cap ? DPZ_ERR_ARG : DPZ_OK;
}

extern "C" int dpz_topk_complete(const float* x, const float* x0, float* acc, int acc_mode,
                                 const float* vals_src, int64_t n, int64_t k, int32_t* idx_out,
                                 float* val_out, int32_t* counter, void* ws, size_t ws_bytes,
                                 int* used_fallback, dpz_stream_t stream) {
  EncodeArgs a{x, x0, acc, acc_mode, vals_src, n, k, idx_out, val_out, counter,
               static_cast<char*>(ws), static_cast<hipStream_t>(stream)};
  int rc = validate(a, ws_bytes);
  if (rc != DPZ_OK) return rc;
  if (used_fallback) *used_fallback = 0;
  DPZ_HIP_TRY(hipStreamSynchronize(a.st));
  if (n == 0 || k == 0 || !use_sampled(n, k)) return DPZ_OK;
  const WsLayout L = ws_layout(n, k);
  TopkCtrl c;
  DPZ_HIP_TRY(hipMemcpy(&c, a.ws + L.ctrl, sizeof(c), hipMemcpyDeviceToHost));
  if (c.status == 0) return DPZ_OK;
  if (used_fallback) *used_fallback = 1;
  a.val_h = c.val_h ? 1 : 0;  // the value format the sampled call was issued with
  const bool vec = all_aligned(a);
  if (c.hinted && a.acc_mode != DPZ_ACC_ACCUMULATE) {
    // the prior-round window missed (or there was none): the sampled path again, with its own
    // sample launch; nothing of the missed call was applied (compact writes nothing after a
    // miss) and NONE / ADD keys are a pure function of the inputs
    rc = run_sampled(a, L, vec, 3);
    if (rc != DPZ_OK) return rc;
    DPZ_HIP_TRY(hipStreamSynchronize(a.st));
    DPZ_HIP_TRY(hipMemcpy(&c, a.ws + L.ctrl, sizeof(c), hipMemcpyDeviceToHost));
    if (c.status == 0) return DPZ_OK;
  }
  // keys are re-derived from the post-filter state: ACCUMULATE already stored acc += change
  rc = run_exact(a, L, 1, vec);
  if (rc != DPZ_OK) return rc;
  DPZ_HIP_TRY(hipStreamSynchronize(a.st));
  return DPZ_OK;
}

extern "C" int dpz_topk_encode_nodes(int m, const void* node_table, int64_t n, int64_t k,
                                     size_t ws_bytes, int flags, dpz_stream_t stream) {
  return topk_encode_nodes(m, node_table, n, k, ws_bytes, flags,
                           static_cast<hipStream_t>(stream));
}

extern "C" int dpz_topk_sticky_status(void* ws, size_t ws_bytes, int clear, int32_t* out,
                                      dpz_stream_t stream) {
  if (!ws || ws_bytes < sizeof(TopkCtrl)) return DPZ_ERR_ARG;
  hipStream_t st = static_cast<hipStream_t>(stream);
  char* p = static_cast<char*>(ws) + offsetof(TopkCtrl, sticky);
  uint32_t v = 0;
  DPZ_HIP_TRY(hipMemcpyAsync(&v, p, sizeof(v), hipMemcpyDeviceToHost, st));
  DPZ_HIP_TRY(hipStreamSynchronize(st));
  if (clear && v) {
    DPZ_HIP_TRY(hipMemsetAsync(p, 0, sizeof(uint32_t), st));
    DPZ_HIP_TRY(hipStreamSynchronize(st));
  }
  if (out) *out = (int32_t)v;
  return DPZ_OK;
}
