// Batched enqueue of many node codecs (the gossip-round engine, decentralizepy_amd/gossip.py).
//
// A simulated round encodes every node's model and folds every node's neighbourhood
// (reference: each node process calls sharing/PartialModel.py:188-255 get_data_to_send, then
// sharing/Sharing.py:156-190 _averaging).  With 12-96 nodes per GPU the per-call host cost of a
// Python enqueue (~30-50 us) exceeds the kernels' device time, so the loop over nodes lives here:
// node j goes to stream j % n_streams (one workspace per stream), and its sampled-path status
// word is copied to status[j] (device) on the same stream so the caller reads all of them once.
#include <cstdlib>
#include <hip/hip_runtime.h>

#include "../../include/dpz_codec.h"
#include "dpz_topk.h"

extern "C" int dpz_topk_encode_batch_ex(int m, const float* const* x, const float* const* x0,
                                        int64_t n, int64_t k, int32_t* const* counter,
                                        int32_t* const* idx_out, float* const* val_out,
                                        void* const* ws, size_t ws_bytes, int n_streams,
                                        const dpz_stream_t* streams, int32_t* status, int flags) {
  if (m < 0 || n_streams < 1 || !x || !idx_out || !val_out || !ws || !streams) return DPZ_ERR_ARG;
  if (flags & ~(DPZ_BATCH_HINT | DPZ_BATCH_HINT_ALL)) return DPZ_ERR_ARG;
  for (int j = 0; j < m; ++j) {
    const int q = j % n_streams;
    // the prior window: every encode with HINT_ALL, all but each stream's first with HINT
    const bool hint = (flags & DPZ_BATCH_HINT_ALL) || ((flags & DPZ_BATCH_HINT) && j >= n_streams);
    // the sampled path's compact writes node j's final status word to status[j] itself (a
    // separate 4-byte device copy per node cost a blit launch of ~8 us on its stream)
    int rc = dpz::topk_encode_status(x[j], x0 ? x0[j] : nullptr, nullptr, DPZ_ACC_NONE, x[j],
                                     n, k, idx_out[j],
                                     val_out[j], counter ? counter[j] : nullptr, ws[q], ws_bytes,
                                     static_cast<hipStream_t>(streams[q]),
                                     status ? status + j : nullptr, n_streams > 1, false, hint);
    if (rc != DPZ_OK) return rc;
  }
  return DPZ_OK;
}

extern "C" int dpz_topk_encode_batch(int m, const float* const* x, const float* const* x0,
                                     int64_t n, int64_t k, int32_t* const* counter,
                                     int32_t* const* idx_out, float* const* val_out,
                                     void* const* ws, size_t ws_bytes, int n_streams,
                                     const dpz_stream_t* streams, int32_t* status) {
  return dpz_topk_encode_batch_ex(m, x, x0, n, k, counter, idx_out, val_out, ws, ws_bytes,
                                  n_streams, streams, status, 0);
}

namespace dpz {
// dpz_fold.hip: every node's fold in one launch per FW_BATCH nodes (1 = the batch does not qualify)
int fold_batch_walk(int m, const float* const* local, float* const* out, int64_t n,
                    const int* n_payloads, const int32_t* const* idx, const float* const* vals,
                    const int64_t* k, const float* w, const float* w_self, int flags,
                    hipStream_t st, const int32_t* guard, int64_t guard_n);
}  // namespace dpz

extern "C" int dpz_decode_average_batch(int m, const float* const* local, float* const* out,
                                        int64_t n, const int* n_payloads,
                                        const int32_t* const* idx, const float* const* vals,
                                        const int64_t* k, const float* w, const float* w_self,
                                        int flags, void* const* ws, size_t ws_bytes,
                                        int n_streams, const dpz_stream_t* streams) {
  if (m < 0 || n_streams < 1 || !local || !out || !n_payloads || !ws || !streams) return DPZ_ERR_ARG;
  for (int j = 0; j < m; ++j)
    if (n_payloads[j] < 0) return DPZ_ERR_ARG;
  // a round of plain few-payload folds (the C4 gossip round): one walk launch per 22 nodes on
  // streams[0] instead of one per node (dpz_fold.hip fold_batch_walk)
  {
    const int rc = dpz::fold_batch_walk(m, local, out, n, n_payloads, idx, vals, k, w, w_self,
                                        flags, static_cast<hipStream_t>(streams[0]), nullptr, 0);
    if (rc != 1) return rc;
  }
  int64_t off = 0;
  for (int j = 0; j < m; ++j) {
    const int q = j % n_streams;
    const int np = n_payloads[j];
    if (np < 0) return DPZ_ERR_ARG;
    int rc = dpz_decode_average(local[j], n, np, idx + off, vals + off, k + off, w + off,
                                w_self ? w_self[j] : 0.0f, flags, out[j], ws[q], ws_bytes,
                                streams[q]);
    if (rc != DPZ_OK) return rc;
    off += np;
  }
  return DPZ_OK;
}

// The round's folds with no host check of the round's encodes in between (gossip.py): the
// one-launch walk path of dpz_decode_average_batch, each launch reading guard[0, guard_n) (DEVICE
// int32: the encodes' status words) first and writing nothing if any is nonzero.  DPZ_ERR_
// UNSUPPORTED, nothing enqueued, when the batch does not take the one-launch path.
extern "C" int dpz_decode_average_batch_guarded(int m, const float* const* local,
                                                float* const* out, int64_t n,
                                                const int* n_payloads, const int32_t* const* idx,
                                                const float* const* vals, const int64_t* k,
                                                const float* w, const float* w_self, int flags,
                                                const int32_t* guard, int64_t guard_n,
                                                dpz_stream_t stream) {
  if (m < 0 || !local || !out || !n_payloads || !guard || guard_n < 1) return DPZ_ERR_ARG;
  for (int j = 0; j < m; ++j)
    if (n_payloads[j] < 0) return DPZ_ERR_ARG;
  const int rc = dpz::fold_batch_walk(m, local, out, n, n_payloads, idx, vals, k, w, w_self,
                                      flags, static_cast<hipStream_t>(stream), guard, guard_n);
  return rc == 1 ? DPZ_ERR_UNSUPPORTED : rc;
}

// One codec step per node: encode node j's model (as dpz_topk_encode_batch) and/or replace-decode
// the payload (r_idx[j], r_val[j]) into r_out[j] from r_local[j] (dpz_decode_average with
// DPZ_FOLD_REPLACE_ONLY), node j on streams[j % n_streams].  Host cost: the launches only.
extern "C" int dpz_encode_replace_batch(int m, int what, const float* const* x,
                                        const float* const* x0, int64_t n, int64_t k,
                                        int32_t* const* counter, int32_t* const* idx_out,
                                        float* const* val_out, const float* const* r_local,
                                        const int32_t* const* r_idx, const float* const* r_val,
                                        int64_t r_k, float* const* r_out, void* const* ws,
                                        size_t ws_bytes, void* const* dws, size_t dws_bytes,
                                        int n_streams, const dpz_stream_t* streams) {
  if (m < 0 || n_streams < 1 || !streams || !(what & (DPZ_BATCH_ENCODE | DPZ_BATCH_DECODE)) ||
      (what & ~(DPZ_BATCH_ENCODE | DPZ_BATCH_DECODE | DPZ_BATCH_HINT | DPZ_BATCH_HINT_ALL)))
    return DPZ_ERR_ARG;
  if ((what & DPZ_BATCH_ENCODE) && (!x || !idx_out || !val_out || !ws)) return DPZ_ERR_ARG;
  if ((what & DPZ_BATCH_DECODE) && (!r_local || !r_idx || !r_val || !r_out || !dws))
    return DPZ_ERR_ARG;
  // On ONE stream, a node whose decoded payload is not the one it is encoding (a neighbour's)
  // runs its encode and decode as one co-scheduled call (dpz_topk_encode_replace: the decode's
  // chunks ride in the encoder's latency-bound launches; C2 serial step 61.8 -> 59.4 us on
  // MI355X).  On several streams the other nodes' streaming already fills the tails, and the
  // plain launches measured faster (C2 3 streams: 41.9 vs 42.7 us).  DPZ_BATCH_COSCHED=0 / 1
  // forces the stream rule (never the independence rule).
  // A node decoding over the model it encodes (r_local[j] == x[j], the reference's
  // deserialized_model base) takes the fused call on any stream count: the encoder's filter
  // writes the decode's copy of x as it streams x (dpz_topk_encode_replace).
  // DPZ_BATCH_COSCHED=0 / 1 forces the plain / co-scheduled enqueue (diagnostic build, A/B)
  const int cs_env = (int)DPZ_KNOB_INT(BATCH_COSCHED, -1);
  const bool cosched = cs_env >= 0 ? cs_env != 0 : n_streams == 1;
  for (int j = 0; j < m; ++j) {
    const int q = j % n_streams;
    // the prior window: every encode with HINT_ALL, all but each stream's first with HINT
    const int hint = ((what & DPZ_BATCH_HINT_ALL) || ((what & DPZ_BATCH_HINT) && j >= n_streams))
                         ? DPZ_TOPK_HINT : 0;
    const bool both = (what & DPZ_BATCH_ENCODE) && (what & DPZ_BATCH_DECODE) &&
                      r_idx[j] != idx_out[j] && r_val[j] != val_out[j];
    const bool fused = both && r_local[j] == x[j] && cs_env != 0;
    if (both && (cosched || fused)) {
      const int fl = DPZ_TOPK_ASYNC | (n_streams > 1 ? DPZ_TOPK_SHARED : 0) | hint;
      int rc = dpz_topk_encode_replace(x[j], x0 ? x0[j] : nullptr, nullptr, DPZ_ACC_NONE, x[j], n,
                                       k, idx_out[j], val_out[j], counter ? counter[j] : nullptr,
                                       ws[q], ws_bytes, fl, r_local[j], r_idx[j],
                                       r_val[j], r_k, n, r_out[j], dws[q], dws_bytes, streams[q]);
      if (rc != DPZ_OK) return rc;
      continue;
    }
    if (what & DPZ_BATCH_ENCODE) {
      // several streams: several codecs share the GPU, the smaller filter grid (DPZ_TOPK_SHARED)
      const int fl = DPZ_TOPK_ASYNC | (n_streams > 1 ? DPZ_TOPK_SHARED : 0) | hint;
      int rc = dpz_topk_encode(x[j], x0 ? x0[j] : nullptr, nullptr, DPZ_ACC_NONE, x[j], n, k,
                               idx_out[j], val_out[j], counter ? counter[j] : nullptr, ws[q],
                               ws_bytes, fl, streams[q]);
      if (rc != DPZ_OK) return rc;
    }
    if (what & DPZ_BATCH_DECODE) {
      const int32_t* ip = r_idx[j];
      const float* vp = r_val[j];
      const int64_t kk = r_k;
      int rc = dpz_decode_average(r_local[j], n, 1, &ip, &vp, &kk, nullptr, 0.0f,
                                  DPZ_FOLD_REPLACE_ONLY, r_out[j], dws[q], dws_bytes, streams[q]);
      if (rc != DPZ_OK) return rc;
    }
  }
  return DPZ_OK;
}
