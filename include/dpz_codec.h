/*
 * dpz_codec.h — C ABI of the MI355X-native decentralizepy model-update codec (libdpzcodec.so).
 *
 * Every pointer argument is caller-owned DEVICE memory (e.g. torch.Tensor.data_ptr() of a
 * CUDA/HIP tensor) unless the comment says "host".  `stream` is a hipStream_t (NULL = default
 * stream).  Every entry point returns an int status: 0 = success, a hipError_t value for HIP
 * failures, or one of the DPZ_ERR_* codes below.  No entry point allocates device memory:
 * workspace is sized by the *_workspace_bytes() queries and passed in by the caller.
 * Codec entry points are reentrant; the only mutable global state is the opt-in per-kernel
 * timing facility (dpz_timing_*), a measurement aid.
 *
 * Each function names the reference (sacs-epfl/decentralizepy, src/decentralizepy/...) code it
 * replaces.  The reference itself has no native layer: these replace ATen-CPU / PyWavelets /
 * numpy call sites inside its Sharing and Compression plugins (see INTEGRATION.md for the
 * ctypes binding and DESIGN.md for the kernels behind each call).
 */
#ifndef DPZ_CODEC_H
#define DPZ_CODEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* dpz_stream_t; /* hipStream_t */

/* ---- status codes ------------------------------------------------------------------------ */
#define DPZ_OK 0
#define DPZ_ERR_ARG 1001         /* invalid argument (null pointer, negative size, k > n, ...) */
#define DPZ_ERR_WORKSPACE 1002   /* workspace smaller than the matching *_workspace_bytes()   */
#define DPZ_ERR_UNSUPPORTED 1003 /* size/config outside what the kernels implement            */
#define DPZ_ERR_INTERNAL 1004    /* an internal consistency check failed on the device        */

/* ---- key modes for top-k: how the selection key is formed (reference PartialModel.py:305-331)
 *   DPZ_ACC_NONE       change = x - x0              key = |change|
 *   DPZ_ACC_ACCUMULATE acc += change (written back)  key = |acc|           (:321-325)
 *   DPZ_ACC_ADD        key = |change + acc|, acc unchanged before the rewind (:326-329)
 * With x0 == NULL, change = x (x is already a change vector, e.g. W(x - x0) for JWINS).      */
#define DPZ_ACC_NONE 0
#define DPZ_ACC_ACCUMULATE 1
#define DPZ_ACC_ADD 2

/* ---- top-k flags ---- */
#define DPZ_TOPK_EXACT 0x1 /* force the exact multi-pass radix path (skip the sampled path)  */
#define DPZ_TOPK_ASYNC 0x2 /* enqueue only; the caller must call dpz_topk_complete() later   */
/* Split enqueue (implies DPZ_TOPK_ASYNC), for callers that overlap independent work with the
 * latency-bound part of the encode: STREAM enqueues the pass that reads the inputs (sample +
 * filter); a second call with TAIL and the SAME arguments, on the same stream or one ordered
 * after it, enqueues the selection tail (select, resolve, compact).  On the exact path STREAM
 * enqueues everything and TAIL nothing.                                                       */
#define DPZ_TOPK_STREAM 0x4
#define DPZ_TOPK_TAIL 0x8
/* Several codecs share the GPU (concurrent streams): up to ~2^24 elements the sampled path's
 * filter uses a smaller grid that leaves CU slots to the other streams' kernels; a lone codec
 * (the default) takes the larger, faster-alone grid.  Results are identical either way; STREAM
 * and TAIL calls of one encode must pass the same choice.                                     */
#define DPZ_TOPK_SHARED 0x10
/* val_out receives fp16 values (uint16 words, round to nearest even: torch.Tensor.half(), the
 * C5 payload's value packing) written by the encode itself — no separate packing
 * launch.  val_out then holds k * 2 bytes.  A later dpz_topk_complete re-runs a missed sampled
 * call in the same format.                                                                    */
#define DPZ_TOPK_VAL_FP16 0x20
/* Prior-round key window: the sampled path takes the filter's key window from the exact
 * threshold of the previous sampled call on this workspace — same n, k, DPZ_TOPK_SHARED choice,
 * acc_mode and x0 presence, completed without a miss — as [0.9375 T, 1.0625 T], and skips its
 * sample launch (a node's consecutive rounds: the k-th largest |change| drifts slowly).  The
 * window is validated like a sampled one; when it does not bracket the k-th key (or no such
 * previous call exists) the call misses: a blocking call / dpz_topk_complete then re-runs the
 * SAMPLED path (sample launch included) and only if that misses too the exact path; an
 * asynchronous caller sees the miss in the status word.  Ignored with DPZ_ACC_ACCUMULATE and on
 * the paths without the pipelined filter (unaligned operands).  Results are identical.       */
#define DPZ_TOPK_HINT 0x40
/* x is streamed with the default cache policy instead of non-temporal loads: for a caller that
 * reads x again right after the encode (a node's Metro-Hastings fold over its own model,
 * sharing/Sharing.py:156-190 after PartialModel.py:188-255), whose re-read may then be served
 * by the 256 MiB Infinity Cache.  Results are identical.                                       */
#define DPZ_TOPK_KEEP_X 0x80
/* dpz_topk_encode_nodes only: every node's shared_parameters_counter in bit-sliced form (as
 * dpz_topk_encode_sliced): the node table's counter word points at its planes
 * (uint32[32 * dpz_mask_words(n)]) and its last word at a selection mask
 * (uint32[dpz_mask_words(n)]); compact writes every mask word and adds the mask to the planes
 * instead of the scattered counter[idx] += 1.  DPZ_ERR_UNSUPPORTED when a node's wave segment is
 * longer than one LDS mask row (n past ~25 M at the shared grid).                           */
#define DPZ_TOPK_SLICED 0x100

/* ---- fold flags ---- */
#define DPZ_FOLD_SELF 0x1         /* add the local term w_self*local after the payloads        */
#define DPZ_FOLD_REPLACE_ONLY 0x2 /* out = local with payload[0] values replaced (no weights)  */
#define DPZ_FOLD_ZERO_BASE 0x4    /* sparse payloads are zero off their indices, not local, and
                                     the fold starts from +0.0 (reference STC.py:181-206, 336-361:
                                     T = zeros; T[idx] = params; total = zeros; total += w*T)  */
#define DPZ_FOLD_ACCUMULATE 0x10  /* out holds the running total on entry: the fold continues
                                     from it instead of starting a new one (Choco.py:433-441:
                                     s += w * T_i; s += (1 - sum w) * q)                      */
#define DPZ_FOLD_ADD_ONLY 0x8     /* n_payloads == 1: out = local + T_0 with T_0 zero-based
                                     (reference STC.py:290-303 process_received)              */
#define DPZ_FOLD_BASE_READY 0x40 /* out already holds this fold's no-hit base over local (written
                                  * by dpz_topk_encode_foldbase with the same w / w_self): only the
                                  * elements the (sparse) payloads hit are rewritten.  Only with
                                  * DPZ_FOLD_SELF, 1 <= n_payloads <= 16, no dense payload.      */
#define DPZ_FOLD_ALSO_LOCAL 0x20  /* the result is ALSO written over local, in place (the
                                     reference's load_state_dict of the averaged model while
                                     _post_step makes it init_model, Sharing.py:186-190,
                                     PartialModel.py:333-353): saves a model copy per round.
                                     Not with REPLACE_ONLY / ADD_ONLY.                       */

int dpz_abi_version(void);
/* First 16 hex digits of the SHA-256 of the sources the library was built from (csrc/ *.cpp, *.h,
 * *.hip in name order, then csrc/Makefile, then this header): the Python binding compares it
 * with the checked-out tree and refuses a stale binary.                                        */
const char* dpz_build_id(void);
const char* dpz_error_string(int code);

/* Top-k magnitude encode.
 * Replaces reference sharing/PartialModel.py:164-255 (extract_top_gradients: abs + torch.topk +
 * torch.sort; serialized_model: shared_parameters_counter[idx] += 1, rewind_accumulation(idx)
 * (models/Model.py:53-64), values pre_share_model[idx]) and sharing/JWINS/Wavelet.py:142-197
 * (apply_wavelet + the same bookkeeping on wavelet coefficients).
 * Selects the k largest keys (see DPZ_ACC_*), ties at the k-th key broken by lowest index,
 * and writes them in ascending index order:  idx_out[j] (int32), val_out[j] = vals_src[idx_out[j]].
 * Side effects: counter[idx] += 1 if counter != NULL; acc[idx] = 0 if acc != NULL and
 * acc_mode != DPZ_ACC_NONE; acc += change everywhere first when acc_mode == DPZ_ACC_ACCUMULATE.
 * n < 2^31, 0 <= k <= n.  Without DPZ_TOPK_ASYNC the call blocks until the result is final.
 * ws: device scratch of at least dpz_topk_workspace_bytes(n, k) bytes, ZERO-FILLED before its
 * first use (hipMemset once); the library keeps the small region it relies on zeroed after.   */
size_t dpz_topk_workspace_bytes(int64_t n, int64_t k);
int dpz_topk_encode(const float* x, const float* x0, float* acc, int acc_mode,
                    const float* vals_src, int64_t n, int64_t k, int32_t* idx_out,
                    float* val_out, int32_t* counter, void* ws, size_t ws_bytes, int flags,
                    dpz_stream_t stream);
/* dpz_topk_encode (same arguments, flags and result) that ALSO writes the no-hit base of the
 * node's coming Metro-Hastings average over x (reference sharing/Sharing.py:156-190 with the
 * local model x, the fold of PartialModel payloads deserialized over it, PartialModel.py:257-303):
 *   base_out[j] = fl(...fl(fl(x[j]*w[0]) + fl(x[j]*w[1])) ... + fl(x[j]*w_self))
 * i.e. what dpz_decode_average(x, ..., w, w_self, DPZ_FOLD_SELF) computes at an element no
 * payload hits.  On the sampled path with 16-byte aligned operands and DPZ_ACC_NONE the filter
 * writes it as it streams x (4n bytes written, no extra read); otherwise a separate pass writes it.
 * A later dpz_decode_average(local = x, the payloads, the SAME w / w_self, DPZ_FOLD_SELF |
 * DPZ_FOLD_BASE_READY, out = base_out) then rewrites only the elements its payloads hit — the
 * decode's 8n bytes of streaming become a gather per hit element.  1 <= n_weights <= 16;
 * base_out (n floats) may not overlap any buffer of the encode (DPZ_ERR_ARG); no STREAM / TAIL
 * split.                                                                                       */
int dpz_topk_encode_foldbase(const float* x, const float* x0, float* acc, int acc_mode,
                             const float* vals_src, int64_t n, int64_t k, int32_t* idx_out,
                             float* val_out, int32_t* counter, void* ws, size_t ws_bytes,
                             int flags, int n_weights, const float* w, float w_self,
                             float* base_out, dpz_stream_t stream);

/* Top-k encode (exactly dpz_topk_encode with the same arguments) TOGETHER WITH one independent
 * replace decode (exactly dpz_decode_average(r_local, r_n, 1, &r_idx, &r_val, &r_k, NULL, 0,
 * DPZ_FOLD_REPLACE_ONLY, r_out, r_ws, r_ws_bytes) — reference sharing/PartialModel.py:257-303,
 * `T[idx] = params` on a neighbour's payload).  A node's round does both (encode its own model,
 * decode a received payload); on the sampled path the decode's chunks run in blocks appended to
 * the encoder's four latency-bound selection launches, so its HBM streaming fills the CUs those
 * leave idle (a cross-stream event wait costs ~15 us on ROCm 7.2, measured, so a second stream
 * does not pay).  Otherwise the decode is enqueued first on `stream`, then the encode.
 * r_out may not overlap r_local or any buffer of the encode (DPZ_ERR_ARG).  The decode is
 * complete when the encode's stream work is (DPZ_TOPK_ASYNC applies to both); the STREAM / TAIL
 * phase flags are not accepted.  r_ws: the decode workspace (only used when not carried).
 * Decoding over the tensor being encoded (r_local == x, r_n == n, acc_mode DPZ_ACC_NONE: the
 * reference decodes a neighbour's payload over the node's own model, the one it just encoded)
 * is FUSED: the encoder's streaming filter writes r_out = x while it reads x, and only the r_k
 * entries are scattered afterwards, in blocks of the compact launch (4n fewer bytes read). */
int dpz_topk_encode_replace(const float* x, const float* x0, float* acc, int acc_mode,
                            const float* vals_src, int64_t n, int64_t k, int32_t* idx_out,
                            float* val_out, int32_t* counter, void* ws, size_t ws_bytes, int flags,
                            const float* r_local, const int32_t* r_idx, const float* r_val,
                            int64_t r_k, int64_t r_n, float* r_out, void* r_ws, size_t r_ws_bytes,
                            dpz_stream_t stream);
/* Threshold selection keeping every tie (reference sharing/Choco.py:117-161:
 * cutoff = kthvalue(-|x|, k); x[|x| < -cutoff] = 0; then nonzero()): T = the k-th largest key
 * |x| (T = 0 when k == 0), selects every i with key(x[i]) >= T and x[i] != 0, in ascending
 * index order: idx_out[j], val_out[j] = x[idx_out[j]], at most cap entries.  Blocks; *count
 * (host) = the number selected; returns DPZ_ERR_ARG (with *count set) if it exceeds cap.
 * The selected threshold key stays readable on the device for dpz_mask_below_threshold.       */
int dpz_topk_threshold(const float* x, int64_t n, int64_t k, int32_t* idx_out, float* val_out,
                       int64_t cap, void* ws, size_t ws_bytes, int64_t* count,
                       dpz_stream_t stream);
/* out[i] = key(x[i]) < T ? +0.0f : x[i], T = the threshold key of the last dpz_topk_threshold on
 * this workspace (Choco's in-place sparsification of q, Choco.py:117-140).  out may alias x.   */
int dpz_mask_below_threshold(const float* x, int64_t n, const void* ws, float* out,
                             dpz_stream_t stream);
/* Elementwise fp32 helpers of the Choco update (reference Choco.py:353-447), one rounding per op:
 *   DPZ_EW_SUB   out = a - b
 *   DPZ_EW_ADD   out = a + b
 *   DPZ_EW_CHOCO out = a + c * (b - d)      (x + gamma * (s - x_hat))
 *   DPZ_EW_MHCOMBINE out = a * (c - b) + d  (the reduce-scatter gossip round's owner combine:
 *                x * (weight total - hit weights) + weighted hit values, decentralizepy_amd/gossip.py)
 * out may alias a.  c is rounded to fp32 like a torch scalar multiply.                        */
#define DPZ_EW_SUB 1
#define DPZ_EW_ADD 2
#define DPZ_EW_CHOCO 3
#define DPZ_EW_MHCOMBINE 4
int dpz_elementwise(int op, const float* a, const float* b, const float* d, float c, int64_t n,
                    float* out, dpz_stream_t stream);
/* Helpers of the sharded top-k (one tensor split over ranks, decentralizepy_amd/shard.py,
 * SURVEY §8e): out[j] = x[idx[j]] - x0[idx[j]] (x0 may be NULL); out[j] = src[pos[j]] for 32-bit
 * words (dpz_gather_u16: 16-bit words, the fp16 values of a C5 payload); dst[idx[j] - offset] +=
 * value where idx[j] - offset lies in [0, n).                                                   */
int dpz_gather_change(const float* x, const float* x0, int64_t n, const int32_t* idx, int64_t k,
                      float* out, dpz_stream_t stream);
int dpz_gather_u32(const void* src, int64_t m, const int32_t* pos, int64_t k, void* out,
                   dpz_stream_t stream);
int dpz_gather_u16(const void* src, int64_t m, const int32_t* pos, int64_t k, void* out,
                   dpz_stream_t stream);
int dpz_scatter_add_i32(int32_t* dst, int64_t n, const int32_t* idx, int64_t k, int64_t offset,
                        int32_t value, dpz_stream_t stream);
/* Completes a DPZ_TOPK_ASYNC encode issued with the SAME arguments: synchronises `stream`,
 * and if the sampled path reported a miss, re-runs the selection exactly (blocking).
 * *used_fallback (host, may be NULL) is set to 1 when that happened.                         */
int dpz_topk_complete(const float* x, const float* x0, float* acc, int acc_mode,
                      const float* vals_src, int64_t n, int64_t k, int32_t* idx_out,
                      float* val_out, int32_t* counter, void* ws, size_t ws_bytes,
                      int* used_fallback, dpz_stream_t stream);

/* dpz_topk_encode with DPZ_TOPK_ASYNC (same arguments, any acc_mode) that also writes the call's
 * final status word to status_out (DEVICE int32, on `stream`, as the encode's last write): 0 =
 * the result is final; otherwise the sampled path missed, nothing was written or updated, and the
 * caller re-runs the encode with DPZ_TOPK_EXACT.  Lets a caller enqueue many encodes that share
 * one workspace (a gossip round's nodes, decentralizepy_amd/gossip_jwins.py) and read every
 * status once; replaces the same reference lines as dpz_topk_encode.  flags: DPZ_TOPK_SHARED
 * and / or DPZ_TOPK_VAL_FP16 (any other bit is DPZ_ERR_ARG).                                   */
int dpz_topk_encode_status(const float* x, const float* x0, float* acc, int acc_mode,
                           const float* vals_src, int64_t n, int64_t k, int32_t* idx_out,
                           float* val_out, int32_t* counter, void* ws, size_t ws_bytes,
                           int32_t* status_out, int flags, dpz_stream_t stream);

/* ---- the encode's side effects in coalesced form (JWINS / Wavelet with accumulation) ----------
 * Selection mask: ceil(n/32) uint32 words (dpz_mask_words), bit b of word w <-> element 32w + b.
 * Sliced counter: the share counter (reference shared_parameters_counter, int32 per element,
 * sharing/PartialModel.py:143-145) as 32 bit planes of ceil(n/32) words, 4 * 32 * ceil(n/32)
 * bytes: bit b of planes[p * ceil(n/32) + w] is bit p of counter[32w + b].
 * dpz_topk_encode_sliced: the selection of dpz_topk_encode (same keys, ties, idx_out / val_out;
 * acc_mode DPZ_ACC_NONE or DPZ_ACC_ADD, acc only read) with its bookkeeping
 * (sharing/JWINS/Wavelet.py:194-197: shared_parameters_counter[idx] += 1,
 * rewind_accumulation(idx)) as: planes (may be NULL) += 1 at every selected index, and every word
 * of sel_mask written with the selected bits.  The rewind acc[idx] = 0 is NOT applied: the caller
 * folds it into the next pass that rewrites acc — dpz_dwt_sym2_rewind / dpz_dwt_haar_rewind
 * (the accumulating post-step, sharing/PartialModel.py:346-349: acc = (bit ? 0 : acc) + T(x - x0),
 * the reference's rewind-then-add) or dpz_rewind_apply.  Scattered 4-byte counter / accumulator
 * updates over 10 % of a 25 M array touch ~97 % of their 128-byte lines; this form writes
 * n/8 mask bytes and the few planes a carry reaches.  status_out (DEVICE int32, may be NULL):
 * non-NULL = asynchronous, the final status written on `stream` (nonzero: the sampled path
 * missed, nothing was written; re-run with DPZ_TOPK_EXACT); NULL = blocking, a miss re-run
 * exactly inside the call (a DPZ_TOPK_HINT call that missed first runs the sampled path once
 * more).  flags: DPZ_TOPK_EXACT, DPZ_TOPK_SHARED, DPZ_TOPK_VAL_FP16, DPZ_TOPK_HINT (the key
 * window from the previous sampled encode's exact threshold on ws, as dpz_topk_encode).
 * dpz_counter_unslice / dpz_counter_slice convert between the sliced and the int32 counter
 * (DeviceCounter materialises on read); dpz_rewind_apply: acc[i] = 0 where the bit is set.      */
int64_t dpz_mask_words(int64_t n);
int dpz_topk_encode_sliced(const float* x, const float* x0, const float* acc, int acc_mode,
                           const float* vals_src, int64_t n, int64_t k, int32_t* idx_out,
                           float* val_out, uint32_t* planes, uint32_t* sel_mask, void* ws,
                           size_t ws_bytes, int32_t* status_out, int flags, dpz_stream_t stream);
int dpz_counter_unslice(const uint32_t* planes, int64_t n, int32_t* counter, dpz_stream_t stream);
int dpz_counter_slice(const int32_t* counter, int64_t n, uint32_t* planes, dpz_stream_t stream);
int dpz_rewind_apply(float* acc, const uint32_t* sel_mask, int64_t n, dpz_stream_t stream);

/* ---- the int32 share counter applied on read (ring of sent payload indices) -----------------
 * Replaces the per-round `shared_parameters_counter[indices] += 1` of reference
 * sharing/PartialModel.py:205-207 / sharing/JWINS/Wavelet.py:194-195, whose only reader is the
 * end-of-run dump (node/DPSGDNode.py:186-194): the plugin keeps every round's payload indices (the
 * encode's idx_out, strictly ascending int32 in [0, n)) in one device ring and, before any read
 * of the counter or when the ring is full, applies them all:
 *   counter[ring[j]] += 1 for every j < seg_off[m], segment r = ring[seg_off[r], seg_off[r + 1])
 * seg_off: HOST int64[m + 1], seg_off[0] = 0, ascending; each segment strictly ascending indices
 * in [0, n) (an index outside is skipped).  mode DPZ_COUNTER_SCATTER: one atomic per entry;
 * DPZ_COUNTER_SWEEP: every tile of the counter read, incremented in LDS and written once (8n
 * coalesced bytes + 8 per entry, per 64 segments; ws: device scratch of
 * dpz_counter_flush_workspace_bytes(n) bytes, only the sweep uses it); DPZ_COUNTER_AUTO picks
 * the cheaper.                                                                                 */
#define DPZ_COUNTER_AUTO 0
#define DPZ_COUNTER_SCATTER 1
#define DPZ_COUNTER_SWEEP 2
size_t dpz_counter_flush_workspace_bytes(int64_t n);
int dpz_counter_flush(int32_t* counter, int64_t n, const int32_t* ring, const int64_t* seg_off,
                      int m, int mode, void* ws, size_t ws_bytes, dpz_stream_t stream);

/* Batched decode + Metro-Hastings fold over n_payloads neighbour payloads.
 * Replaces reference sharing/PartialModel.py:257-303 (T = cat(local); T[idx] = params),
 * sharing/Sharing.py:156-229 (_averaging / _averaging_server fold) and
 * sharing/JWINS/Wavelet.py:269-309, 336-366 (the same fold on wavelet coefficients).
 *   out[j] = fl( ... fl(fl(t_0[j]*w[0]) + fl(t_1[j]*w[1])) ... + fl(local[j]*w_self) )
 *   t_i[j] = vals[i][m] if idx[i][m] == j for some m, else local[j].
 * Payload i is DENSE (a full model: t_i = vals[i]) iff idx[i] == NULL and k[i] == n; otherwise
 * idx[i] holds k[i] strictly ascending indices (idx[i] may be NULL when k[i] == 0).
 * The local term is present only with DPZ_FOLD_SELF.  idx/vals/k/w are HOST arrays of length
 * n_payloads holding DEVICE pointers / sizes / fp32 weights.  out may not alias local.
 * DPZ_FOLD_REPLACE_ONLY: n_payloads == 1, out = t_0 (no multiply).
 * DPZ_FOLD_ZERO_BASE: t_i[j] = 0 where payload i has no entry (instead of local[j]) and the
 *   first term is fl(+0.0 + fl(t_0[j]*w[0])).  DPZ_FOLD_ADD_ONLY: n_payloads == 1,
 *   out[j] = fl(local[j] + T_0[j]) with T_0 zero-based (no weights).
 * ws: device scratch of at least dpz_decode_workspace_bytes(n, n_payloads) bytes.              */
size_t dpz_decode_workspace_bytes(int64_t n, int n_payloads);
int dpz_decode_average(const float* local, int64_t n, int n_payloads, const int32_t* const* idx,
                       const float* const* vals, const int64_t* k, const float* w, float w_self,
                       int flags, float* out, void* ws, size_t ws_bytes, dpz_stream_t stream);

/* Replace decode of a GLOBAL payload into one rank's slice of a model sharded over ranks
 * (SURVEY §8e "one tensor, decode: no collective"; reference sharing/PartialModel.py:292-295
 * `T[idx] = params` restricted to the slice): local / out hold global elements
 * [offset, offset + n); out[i] = local[i], then out[idx[j] - offset] = vals[j] for every entry
 * inside the slice (entries outside are skipped).  idx: k strictly ascending global indices.
 * local and out 16-byte aligned, out may not alias local.                                      */
int dpz_replace_slice(const float* local, int64_t n, int64_t offset, const int32_t* idx,
                      const float* vals, int64_t k, float* out, dpz_stream_t stream);

/* Batched enqueue for a simulated gossip round (decentralizepy_amd/gossip.py): m node codecs,
 * node j on streams[j % n_streams] with workspace ws[j % n_streams].
 * dpz_topk_encode_batch == for each j: dpz_topk_encode(x[j], x0[j], NULL, DPZ_ACC_NONE, x[j], n,
 *   k, idx_out[j], val_out[j], counter[j], ws[q], ws_bytes, DPZ_TOPK_ASYNC, streams[q]), then the
 *   node's sampled-path status word is copied to status[j] (DEVICE int32[m], may be NULL) on the
 *   same stream (0 = final; otherwise re-run that node with DPZ_TOPK_EXACT).
 * dpz_decode_average_batch == for each j: dpz_decode_average(local[j], n, n_payloads[j],
 *   idx + o_j, vals + o_j, k + o_j, w + o_j, w_self[j], flags, out[j], ws[q], ws_bytes,
 *   streams[q]) with o_j = sum of n_payloads[< j] (all arrays HOST, holding device pointers).
 * Replaces the per-node loops of reference node processes (sharing/PartialModel.py:188-255,
 * sharing/Sharing.py:156-190) run side by side.                                               */
int dpz_topk_encode_batch(int m, const float* const* x, const float* const* x0, int64_t n,
                          int64_t k, int32_t* const* counter, int32_t* const* idx_out,
                          float* const* val_out, void* const* ws, size_t ws_bytes, int n_streams,
                          const dpz_stream_t* streams, int32_t* status);
/* dpz_topk_encode_batch with batch flags: DPZ_BATCH_HINT / DPZ_BATCH_HINT_ALL (the encodes'
 * prior window, as in dpz_encode_replace_batch; a miss shows in status[j] like any other).    */
int dpz_topk_encode_batch_ex(int m, const float* const* x, const float* const* x0, int64_t n,
                             int64_t k, int32_t* const* counter, int32_t* const* idx_out,
                             float* const* val_out, void* const* ws, size_t ws_bytes,
                             int n_streams, const dpz_stream_t* streams, int32_t* status,
                             int flags);
/* The encodes of m nodes of one size (n, k) — each exactly dpz_topk_encode(x, x0, NULL,
 * DPZ_ACC_NONE, x, n, k, idx_out, val_out, counter, ws, ws_bytes, DPZ_TOPK_ASYNC) with its
 * final status word also written to status_out (as dpz_topk_encode_status) — with ONE launch per
 * phase of the sampled path for all of them (sample, filter, select, compact over a grid of m x
 * the per-node grid), so the nodes' latency-bound selection tails overlap each other.
 * node_table: DEVICE array of m entries of 8 64-bit words {x, x0, counter (or 0), idx_out,
 * val_out, ws, status_out, 0}; every node its own workspace of ws_bytes >= dpz_topk_workspace_
 * bytes(n, k) bytes (zero-filled before its first use), x / x0 16-byte aligned.  flags:
 * DPZ_TOPK_HINT (every node's window from its workspace's previous encode, no sample launch; a
 * node without a usable prior misses).  Asynchronous: a nonzero status_out[j] means node j
 * wrote nothing and is re-run with DPZ_TOPK_EXACT.  DPZ_ERR_UNSUPPORTED when (n, k) is not on
 * the sampled path (n >= 2^18, 1 <= k <= n / 2).  Replaces the per-node loops of reference node
 * processes (sharing/PartialModel.py:164-255) run side by side.                               */
int dpz_topk_encode_nodes(int m, const void* node_table, int64_t n, int64_t k, size_t ws_bytes,
                          int flags, dpz_stream_t stream);
int dpz_decode_average_batch(int m, const float* const* local, float* const* out, int64_t n,
                             const int* n_payloads, const int32_t* const* idx,
                             const float* const* vals, const int64_t* k, const float* w,
                             const float* w_self, int flags, void* const* ws, size_t ws_bytes,
                             int n_streams, const dpz_stream_t* streams);
/* dpz_decode_average_batch's one-launch fold of a gossip round (every node 1..4 sparse payloads,
 * flags within DPZ_FOLD_SELF | DPZ_FOLD_ALSO_LOCAL, 16-byte aligned rows, out[j] != local[j]) on
 * ONE stream, guarded by the round's encodes: each launch first reads guard[0, guard_n) (DEVICE
 * int32, e.g. dpz_topk_encode_nodes' status words) and, if any word is nonzero, writes nothing
 * (out and, with DPZ_FOLD_ALSO_LOCAL, local unchanged), so the caller checks the encodes once
 * after the round instead of between encode and fold, and re-runs the round's folds after
 * re-running a missed encode exactly.  DPZ_ERR_UNSUPPORTED (nothing enqueued) when the batch
 * does not qualify.  Replaces the reference's encode -> send -> receive -> _averaging order of
 * every node (sharing/PartialModel.py:188-255, sharing/Sharing.py:156-190), run side by side. */
int dpz_decode_average_batch_guarded(int m, const float* const* local, float* const* out,
                                     int64_t n, const int* n_payloads,
                                     const int32_t* const* idx, const float* const* vals,
                                     const int64_t* k, const float* w, const float* w_self,
                                     int flags, const int32_t* guard, int64_t guard_n,
                                     dpz_stream_t stream);

/* One codec step per node for m nodes of equal size (n, k): with DPZ_BATCH_ENCODE, node j's
 * dpz_topk_encode(x[j], x0[j], NULL, DPZ_ACC_NONE, x[j], n, k, idx_out[j], val_out[j],
 * counter[j], ws[q], ws_bytes, DPZ_TOPK_ASYNC, streams[q]); with DPZ_BATCH_DECODE, then the replace
 * decode dpz_decode_average(r_local[j], n, 1, &r_idx[j], &r_val[j], &r_k, NULL, 0,
 * DPZ_FOLD_REPLACE_ONLY, r_out[j], dws[q], dws_bytes, streams[q]); q = j % n_streams.  Arrays are
 * HOST arrays of device pointers.  A node's round (reference sharing/PartialModel.py:188-303:
 * serialized_model of its own model, deserialized_model of a received payload) with the host
 * loop in native code.  The encodes are asynchronous: a sampled-path miss is recorded in the
 * workspace's sticky status word (dpz_topk_sticky_status), never silently.                     */
#define DPZ_BATCH_ENCODE 0x1
#define DPZ_BATCH_DECODE 0x2
/* with DPZ_BATCH_ENCODE: the encodes pass DPZ_TOPK_HINT — each takes its key window from the
 * previous encode on its stream's workspace (another node of the same round or the node's own
 * previous round: the same change distribution), a miss recorded like any other.  HINT: every
 * encode but the first on each stream (fresh workspaces hold no prior); HINT_ALL: every encode
 * (the workspaces already hold one of this n, k from an earlier call).                        */
#define DPZ_BATCH_HINT 0x4
#define DPZ_BATCH_HINT_ALL 0x8
int dpz_encode_replace_batch(int m, int what, const float* const* x, const float* const* x0,
                             int64_t n, int64_t k, int32_t* const* counter,
                             int32_t* const* idx_out, float* const* val_out,
                             const float* const* r_local, const int32_t* const* r_idx,
                             const float* const* r_val, int64_t r_k, float* const* r_out,
                             void* const* ws, size_t ws_bytes, void* const* dws, size_t dws_bytes,
                             int n_streams, const dpz_stream_t* streams);
/* OR of the final status of every sampled-path encode run on this top-k workspace since the
 * last clear (0 = every one was final; nonzero = at least one missed and, if it was ASYNC and
 * not completed by dpz_topk_complete, published unverified output).  Synchronises `stream`;
 * clear != 0 resets the word afterwards.  *out is a HOST pointer.                              */
int dpz_topk_sticky_status(void* ws, size_t ws_bytes, int clear, int32_t* out,
                           dpz_stream_t stream);

/* Multilevel sym2 DWT, mode "symmetric", fp32, pywt-1.1.1-exact summation order.
 * Replaces reference sharing/JWINS/Wavelet.py:12-32 (pywt.wavedec + coeffs_to_array).
 * coeffs layout: [cA_L, cD_L, ..., cD_1], length dpz_wavedec_len(n, level).
 *   coeffs_x    (may be NULL) = W(x)
 *   coeffs_diff (may be NULL) = W(x - x0)   (x0 must be non-NULL), or += W(x - x0) when
 *   accumulate != 0 (PartialModel._post_step acc += T(init - prev), PartialModel.py:346-349).
 * Requires every level input length >= 4.                                                      */
int64_t dpz_wavedec_len(int64_t n, int level);
int dpz_dwt_sym2(const float* x, const float* x0, int64_t n, int level, float* coeffs_x,
                 float* coeffs_diff, int accumulate, dpz_stream_t stream);

/* dpz_dwt_sym2(x, x0, n, level, NULL, acc, 1) with the deferred rewind of
 * dpz_topk_encode_sliced: acc[i] = fl((bit i of sel_mask ? +0.0 : acc[i]) + W(x - x0)[i]). */
int dpz_dwt_sym2_rewind(const float* x, const float* x0, int64_t n, int level, float* acc,
                        const uint32_t* sel_mask, dpz_stream_t stream);

/* Multilevel sym2 IDWT (pywt.array_to_coeffs + pywt.waverec), first n outputs written.
 * Replaces reference sharing/JWINS/Wavelet.py:311-316.                                        */
int dpz_idwt_sym2(const float* coeffs, int64_t n, int level, float* out, dpz_stream_t stream);

/* Tile ranges of the two transforms, for one tensor sharded over ranks (SURVEY §8e "wavelet
 * DWT/IDWT: yes, with a halo"; decentralizepy_amd/shard.py sharded_wavedec / sharded_waverec).
 * The forward tile t owns level-L outputs [t*W, (t+1)*W) (W = dpz_dwt_tile_width()) and the
 * matching 2^(L-l)*W outputs of every detail level; it reads inputs [2^L*W*t - 2(2^L - 1),
 * 2^L*W*(t+1)) of x / x0 (clipped to [0, n)).  The inverse tile u writes outputs
 * [u*V, (u+1)*V) (V = dpz_idwt_tile_width()).  x, x0, coeffs and out are VIRTUAL bases: element i
 * of the global array is at base + i, and only the elements the tiles [tile_lo, tile_hi) touch
 * are dereferenced (a rank passes its halo'd slice buffer minus its first global index).        */
int64_t dpz_dwt_tile_width(void);
int64_t dpz_idwt_tile_width(void);
int dpz_dwt_sym2_tiles(const float* x, const float* x0, int64_t n, int level, int64_t tile_lo,
                       int64_t tile_hi, float* coeffs_x, float* coeffs_diff, int accumulate,
                       dpz_stream_t stream);
int dpz_idwt_sym2_tiles(const float* coeffs, int64_t n, int level, int64_t tile_lo,
                        int64_t tile_hi, float* out, dpz_stream_t stream);

/* ---- Haar DWT / IDWT (pywt "haar", mode "symmetric": the reference Wavelet's DEFAULT wavelet,
 * sharing/JWINS/Wavelet.py:56).  Same contracts as the sym2 entries above, levels 1..8; level
 * lengths len_l = ceil(len_{l-1} / 2), layout [cA_L, cD_L, ..., cD_1] (pywt.coeffs_to_array).
 * Bit-exact with PyWavelets 1.1.1 (csrc/dpz_haar.hip gives the summation order).              */
int64_t dpz_haar_wavedec_len(int64_t n, int level);
int dpz_dwt_haar(const float* x, const float* x0, int64_t n, int level, float* coeffs_x,
                 float* coeffs_diff, int accumulate, dpz_stream_t stream);
int dpz_idwt_haar(const float* coeffs, int64_t n, int level, float* out, dpz_stream_t stream);
/* the haar counterpart of dpz_dwt_sym2_rewind */
int dpz_dwt_haar_rewind(const float* x, const float* x0, int64_t n, int level, float* acc,
                        const uint32_t* sel_mask, dpz_stream_t stream);

/* ---- Any other pywt discrete wavelet (db1-32, sym2-20, coif1-10, bior / rbio, dmey: even filter
 * length flen <= 64), mode "symmetric", levels 1..8 with every level's input >= flen values.
 * Replaces reference sharing/JWINS/Wavelet.py:12-32 and :311-316 (pywt.wavedec / waverec with
 * the configured `wavelet`) for the wavelets the fused sym2 / haar kernels do not cover.
 * `bank` is DEVICE memory: 4*flen floats dec_lo, dec_hi, rec_lo, rec_hi — the fp32 taps pywt
 * applies to float32 data (decentralizepy_amd/wavelet_filters.json).  Level lengths
 * len_l = floor((len_{l-1} + flen - 1) / 2), layout [cA_L, cD_L, ..., cD_1].  Bit-exact with
 * PyWavelets 1.1.1 (csrc/dpz_wvgen.hip gives the summation order).  dpz_dwt_generic: W(x) into
 * coeffs_x and / or W(x - x0) into coeffs_diff (accumulate: added; sel_mask, with accumulate:
 * the deferred rewind of dpz_topk_encode_sliced, as dpz_dwt_sym2_rewind); ws of
 * dpz_wavelet_generic_workspace_bytes (levels >= 2).  Unsupported lengths: -1 / DPZ_ERR_UNSUPPORTED. */
int64_t dpz_wavedec_len_generic(int64_t n, int level, int flen);
size_t dpz_wavelet_generic_workspace_bytes(int64_t n, int level, int flen);
int dpz_dwt_generic(const float* x, const float* x0, int64_t n, int level, const float* bank,
                    int flen, float* coeffs_x, float* coeffs_diff, int accumulate,
                    const uint32_t* sel_mask, void* ws, size_t ws_bytes, dpz_stream_t stream);
int dpz_idwt_generic(const float* coeffs, int64_t n, int level, const float* bank, int flen,
                     float* out, void* ws, size_t ws_bytes, dpz_stream_t stream);


/* dst[idx[j]] = value for j < k (indices outside [0, n) are ignored).
 * Replaces reference models/Model.py:53-64 (rewind_accumulation: acc[idx] = 0) where the rewind
 * is not fused into dpz_topk_encode (Wavelet with change_based_selection = False).             */
int dpz_scatter_fill(float* dst, int64_t n, const int32_t* idx, int64_t k, float value,
                     dpz_stream_t stream);

/* fp16 value packing (round-to-nearest-even, torch.half semantics) and unpacking.
 * The build's own wire codec for values (BASELINE config C5); the reference's lossy float path
 * is fpzip (compression/EliasFpzipLossy.py:14-58), which is not byte-compatible.             */
int dpz_pack_fp16(const float* in, int64_t n, uint16_t* out, dpz_stream_t stream);
int dpz_unpack_fp16(const uint16_t* in, int64_t n, float* out, dpz_stream_t stream);

/* ---- Per-kernel timing (measurement only; not thread-safe) -----------------------------------
 * While enabled, every kernel launch records a HIP event pair on its own stream (launches into a
 * capturing stream are skipped).  dpz_timing_read waits for the pending pairs and fills the summed
 * milliseconds and launch counts per kernel id; it returns DPZ_KT_COUNT.                     */
enum {
  DPZ_KT_TOPK_SAMPLE = 0, DPZ_KT_TOPK_FILTER, DPZ_KT_TOPK_SELECT, DPZ_KT_TOPK_RESOLVE,
  DPZ_KT_TOPK_COMPACT,
  DPZ_KT_EXACT_HIST, DPZ_KT_EXACT_RESOLVE, DPZ_KT_EXACT_COUNT, DPZ_KT_EXACT_SCAN,
  DPZ_KT_EXACT_WRITE, DPZ_KT_ACCUMULATE,
  DPZ_KT_FOLD_OFFSETS, DPZ_KT_FOLD, DPZ_KT_DWT, DPZ_KT_IDWT, DPZ_KT_ELIAS_COUNT,
  DPZ_KT_ELIAS_SCAN, DPZ_KT_ELIAS_PACK, DPZ_KT_ELIAS_SPEC, DPZ_KT_ELIAS_RESOLVE,
  DPZ_KT_ELIAS_WRITE, DPZ_KT_FP16, DPZ_KT_SCATTER, DPZ_KT_FPZ_SIZE, DPZ_KT_FPZ_SCAN,
  DPZ_KT_FPZ_PACK, DPZ_KT_FPZ_DECODE, DPZ_KT_CPLX, DPZ_KT_FFT_SCALE, DPZ_KT_HAAR, DPZ_KT_LZ4,
  DPZ_KT_COUNTER, DPZ_KT_FFT, DPZ_KT_COUNT
};
int dpz_timing_enable(int on);  /* also clears the accumulators */
int dpz_timing_read(double* ms_sum, int64_t* count, int max_ids);
const char* dpz_kernel_name(int id);

/* ---- Elias-gamma index coding (byte-identical to the reference wire format) ------------------
 * Replaces compression/Elias.py:20-52 (Elias.compress) and :54-97 (Elias.decompress).
 * Format: l = floor(log2(gap)) zero bits then the gap in l+1 bits, MSB-first, for every gap of the
 * sorted int32 array; 128 zero bits; np.packbits byte order; bytes [-16:-8] = int64 LE first
 * value, [-8:] = int64 LE total bit count (code bits + 128).                                   */

/* Upper bound of the encoded size for k values (all gaps 2^31-1), rounded up to 4 bytes. */
int64_t dpz_elias_max_bytes(int64_t k);
/* Device workspace for an encode of k values or a decode of an nbytes stream (the max of both). */
size_t dpz_elias_workspace_bytes(int64_t k, int64_t nbytes);
/* idx: device int32[k], strictly increasing (k >= 2; the reference raises IndexError below 2).
 * out: device buffer, 4-byte aligned, out_cap >= dpz_elias_max_bytes(k).  Writes the stream and
 * returns its length in *nbytes_host (host pointer; the call synchronises `stream`).
 * DPZ_ERR_ARG if the indices are not strictly increasing.                                      */
int dpz_elias_encode(const int32_t* idx, int64_t k, uint8_t* out, int64_t out_cap,
                     int64_t* nbytes_host, void* ws, size_t ws_bytes, dpz_stream_t stream);
/* in: device copy of the stream, 4-byte aligned, readable up to round_up(nbytes, 4) + 16 bytes.
 * nbits/first: the stream's trailer (the caller holds the bytes).  Writes first + running gap
 * sums into out64 (int64, as the reference returns) and/or out32 (either may be NULL); the value
 * count goes to *count_host (host pointer; synchronises).  DPZ_ERR_ARG on a malformed stream,
 * DPZ_ERR_WORKSPACE if the count exceeds out_cap, DPZ_ERR_UNSUPPORTED above 2^26 code bits.    */
int dpz_elias_decode(const uint8_t* in, int64_t nbytes, int64_t nbits, int64_t first,
                     int64_t* out64, int32_t* out32, int64_t out_cap, int64_t* count_host,
                     void* ws, size_t ws_bytes, dpz_stream_t stream);
/* dpz_elias_decode without a host synchronisation, for a receiver that knows the value count
 * from the payload's other leg (the float header's n, or the raw values' length): decodes into
 * out64 / out32 (device, `count` entries) and ORs *status (DEVICE uint32) nonzero on `stream`
 * when the stream is malformed or holds a different number of values — the entries are then
 * unspecified (the fold kernels stay in bounds on any index values); the caller reads the status
 * word once after the round's folds.  Same workspace as dpz_elias_decode.  Replaces the same
 * reference lines (compression/Elias.py:54-97), called from PartialModel.py:156-162.          */
int dpz_elias_decode_async(const uint8_t* in, int64_t nbytes, int64_t nbits, int64_t first,
                           int64_t* out64, int32_t* out32, int64_t count, uint32_t* status,
                           void* ws, size_t ws_bytes, dpz_stream_t stream);

/* ---- Block-floating fp32 value coding (the float leg of EliasFpzip / EliasFpzipLossy) --------
 * Replaces compression/EliasFpzip.py:19-51 (fpzip.compress, precision 0) and
 * compression/EliasFpzipLossy.py:14-58 (precision p).  fpzip is absent, so the bytes are this
 * build's own format (csrc/dpz_fpz.hip): precision 0 (or >= 32) is lossless for every bit pattern;
 * 1 <= p < 32 keeps the top p bits of each value's bit pattern (the rest truncated; from p = 10 on
 * a NaN stays a NaN); p < 0 returns DPZ_ERR_UNSUPPORTED.  Stream: 16-byte header ('DPFZ', n, precision, nblk), a table of
 * nblk + 1 block offsets, then per 256 values a meta word and sign / exponent / mantissa planes. */

/* Upper bound of the stream size for n values (every block at full exponent width). */
int64_t dpz_fpz_max_bytes(int64_t n);
/* Device workspace for an encode of n values. */
size_t dpz_fpz_workspace_bytes(int64_t n);
/* x: device fp32[n] (n <= 2^30); out: device buffer, 4-byte aligned, out_cap >=
 * dpz_fpz_max_bytes(n).  Writes the stream, its length to *nbytes_host (host; synchronises).   */
int dpz_fpz_encode(const float* x, int64_t n, int precision, uint8_t* out, int64_t out_cap,
                   int64_t* nbytes_host, void* ws, size_t ws_bytes, dpz_stream_t stream);
/* in: device copy of a stream of nbytes (a multiple of 4, 4-byte aligned); n and precision from
 * its header (the caller holds the bytes).  Writes out[n]; asynchronous.  Every block is checked
 * against the header, the offset table and the buffer bounds: a malformed block is not decoded
 * and sets *status (device uint32, OR-ed) to nonzero; the caller reads it after the stream.   */
int dpz_fpz_decode(const uint8_t* in, int64_t nbytes, int64_t n, int precision, float* out,
                   uint32_t* status, dpz_stream_t stream);

/* ---- FFT sharing plugin: real FFTs and complex coefficients (decentralizepy_amd/sharing/JWINS/FFT.py)
 * Replaces sharing/JWINS/FFT.py:12-25 (torch.fft.rfft), :301 (torch.fft.irfft, 1/n on the
 * inverse), :143-156 (top-k over |complex change|, flat_fft[index]), PartialModel.py:315-329 on
 * the complex change, Model.py:53-64 (complex rewind).  Complex = interleaved fp32 (re, im), the
 * torch.complex64 layout; m = n / 2 + 1 coefficients for n reals.  The transforms are this
 * build's mixed-radix Stockham kernels (csrc/dpz_fft.hip) whenever every prime factor of the
 * complex length (n / 2 for even n, n for odd) is <= 4096; other sizes fall back to hipFFT
 * (rocFFT, plans cached per device / n / direction).  The library's device allocations are the
 * per-size twiddle tables (and rocFFT's, on the fallback); the work area is the caller's.      */
/* Work area for dpz_rfft / dpz_irfft of n reals (the max of both directions); -1 if unsupported
 * (n < 2 or n > 2^31 - 1).  Creates (and caches) the hipFFT plans of a fallback size.            */
int64_t dpz_fft_workspace_bytes(int64_t n);
/* 1 when dpz_rfft / dpz_irfft of n reals run the native kernels, 0 when they fall back to hipFFT. */
int dpz_fft_native(int64_t n);
/* out[m complex] = rfft(x[n]).  Asynchronous on stream.                                          */
int dpz_rfft(const float* x, int64_t n, float* out, void* ws, size_t ws_bytes, dpz_stream_t stream);
/* out[n] = irfft(coeffs[m complex], n) with torch's "backward" normalisation (1/n).  coeffs may be
 * OVERWRITTEN (the hipFFT fallback's C2R works in place on its input; the native passes only
 * read it).                                                                                       */
int dpz_irfft(float* coeffs, int64_t n, float* out, void* ws, size_t ws_bytes, dpz_stream_t stream);
/* key[i] = |c[i]| (fp32 sqrt(re^2 + im^2)) of the complex change after the DPZ_ACC_* step
 * (ACCUMULATE: acc += change, key = |acc|; ADD: key = |change + acc|, acc unchanged).          */
int dpz_cplx_key(const float* change, float* acc, int acc_mode, int64_t m, float* key,
                 dpz_stream_t stream);
/* out[j] = src[idx[j]] (complex); acc[idx[j]] = 0 when acc is not NULL.                          */
int dpz_cplx_gather(const float* src, int64_t m, const int32_t* idx, int64_t k, float* out,
                    float* acc, dpz_stream_t stream);
/* pair[2j] = 2 idx[j], pair[2j+1] = 2 idx[j] + 1 (8-byte aligned pair): a complex payload as a
 * float payload of the interleaved view, for dpz_decode_average.                                  */
int dpz_cplx_pair_indices(const int32_t* idx, int64_t k, int32_t* pair, dpz_stream_t stream);

/* ---- LZ4 frames (the wire format of compression/Lz4Wrapper.py:20-98, lz4.frame) -------------
 * Encoder: independent 2 KB blocks, one wave each (B.Indep, BD = 64 KB, content size stored, no
 * checksums): a valid LZ4 frame any decoder reads; the bytes are this build's (greedy parse over a
 * 11-bit hash of 4-byte words; python-lz4's match finder is not reproduced, so byte parity is
 * unpinned).  Decoder: any LZ4 frame with 64 KB (or smaller) blocks, linked (python-lz4's
 * default, decoded by one workgroup) or independent (one workgroup per block); content and
 * block checksums are skipped, dictionary IDs rejected.                                         */
/* Upper bound of the frame size for n input bytes. */
int64_t dpz_lz4_max_bytes(int64_t n);
/* Device workspace for an encode of n bytes (nblk = bmax = 0) or a decode of a frame of nblk
 * blocks of at most bmax bytes (n = 0); the max of what the calls ask is always enough.       */
size_t dpz_lz4_workspace_bytes(int64_t n, int64_t nblk, int64_t bmax);
/* in: device bytes[n]; out: device, out_cap >= dpz_lz4_max_bytes(n).  The frame length goes to
 * *nbytes_host (host; synchronises).                                                            */
int dpz_lz4_compress(const uint8_t* in, int64_t n, uint8_t* out, int64_t out_cap,
                     int64_t* nbytes_host, void* ws, size_t ws_bytes, dpz_stream_t stream);
/* Frame header and block walk of a HOST copy of a frame: content size (-1 if absent), block
 * count, linked flag, block max.  DPZ_ERR_ARG on a malformed frame (bad magic, version, header
 * checksum, truncated blocks).                                                                  */
int dpz_lz4_frame_info(const uint8_t* frame_host, int64_t nbytes, int64_t* content_size,
                       int64_t* nblk, int* linked, int64_t* block_max);
/* frame_dev / frame_host: the same nbytes of frame on the device and on the host (the host walks
 * the block headers).  Writes the content to out (device) and its length to *n_host (host;
 * synchronises).  DPZ_ERR_ARG on a malformed block or a content-size mismatch,
 * DPZ_ERR_WORKSPACE if the content exceeds out_cap, DPZ_ERR_UNSUPPORTED above 64 KB blocks.   */
int dpz_lz4_decompress(const uint8_t* frame_dev, const uint8_t* frame_host, int64_t nbytes,
                       uint8_t* out, int64_t out_cap, int64_t* n_host, void* ws, size_t ws_bytes,
                       dpz_stream_t stream);
/* out[j] = in[j] - in[j-1] (in[-1] = 0), int32 wrap-around: np.diff(a, prepend=0).astype(int32)
 * (Lz4Wrapper.py:35-37).  in and out must not alias.                                           */
int dpz_delta_i32(const int32_t* in, int64_t k, int32_t* out, dpz_stream_t stream);
/* Inclusive running sum of int32 values as int64 (np.cumsum, Lz4Wrapper.py:58-59) into out64
 * and / or its int32 truncation into out32 (either may be NULL).                                */
size_t dpz_running_sum_workspace_bytes(int64_t k);
int dpz_running_sum_i32(const int32_t* in, int64_t k, int64_t* out64, int32_t* out32, void* ws,
                        size_t ws_bytes, dpz_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* DPZ_CODEC_H */
