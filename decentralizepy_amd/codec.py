"""Device-tensor front end of the HIP codec (libdpzcodec.so).

Every function takes and returns torch tensors that live on a ROCm device; PyTorch is used only
for allocation, streams and tensor handles — the arithmetic runs in the hand-written HIP kernels
behind the C ABI (``include/dpz_codec.h``).  Calls are enqueued on the current torch stream.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import (DPZ_ACC_ACCUMULATE, DPZ_ACC_ADD, DPZ_ACC_NONE, DPZ_EW_ADD, DPZ_EW_CHOCO,
                   DPZ_EW_SUB, DPZ_FOLD_REPLACE_ONLY,
                   DPZ_FOLD_SELF, DPZ_TOPK_ASYNC, DPZ_TOPK_EXACT, DPZ_TOPK_STREAM,
                   DPZ_TOPK_TAIL, check)

__all__ = ["DPZ_ACC_NONE", "DPZ_ACC_ACCUMULATE", "DPZ_ACC_ADD", "DPZ_EW_SUB", "DPZ_EW_ADD",
           "DPZ_EW_CHOCO", "Workspace", "topk_encode",
           "topk_threshold", "mask_below_threshold", "elementwise",
           "topk_complete", "decode_average", "replace", "wavedec_len", "wavedec", "waverec",
           "pack_fp16", "unpack_fp16", "elias_encode", "elias_decode", "elias_decode_async",
           "KernelTimer", "NodeStepBatch", "topk_sticky_status", "rfft", "irfft", "fft_native", "cplx_key",
           "cplx_gather", "cplx_pair_indices", "lz4_compress", "lz4_decompress", "lz4_frame_info",
           "delta_i32", "running_sum_i32", "mask_words", "topk_encode_sliced", "counter_unslice",
           "counter_slice", "rewind_apply", "counter_flush"]


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _require(t, dtype, name):
    if t is None:
        return
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor (got {t.device}); no CPU path exists")
    if t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


class Workspace:
    """Caller-owned device scratch for the encoder and the decoder, reused across calls.

    The top-k workspace must be zero-filled before its first use (the library keeps it so
    afterwards), hence ``torch.zeros``.
    """

    def __init__(self, device):
        self.device = torch.device(device)
        self.buf = None
        self._nk = None
        self.dbuf = None
        self.ebuf = None
        self.hint_key = None  # signature of the last sampled-path encode enqueued on buf

    def get(self, n, k):
        if self.buf is not None and self._nk == (n, k):
            return self.buf
        need = int(_lib.lib().dpz_topk_workspace_bytes(int(n), int(k)))
        if self.buf is None or self.buf.numel() < need:
            self.buf = torch.zeros(max(need, 256), dtype=torch.uint8, device=self.device)
            self.hint_key = None
        self._nk = (n, k)
        return self.buf

    def get_decode(self, n, n_payloads):
        need = int(_lib.lib().dpz_decode_workspace_bytes(int(n), int(n_payloads)))
        if self.dbuf is None or self.dbuf.numel() < need:
            self.dbuf = torch.empty(max(need, 256), dtype=torch.uint8, device=self.device)
        return self.dbuf

    def get_elias(self, k, nbytes):
        need = int(_lib.lib().dpz_elias_workspace_bytes(int(k), int(nbytes)))
        if self.ebuf is None or self.ebuf.numel() < need:
            self.ebuf = torch.empty(max(need, 256), dtype=torch.uint8, device=self.device)
        return self.ebuf


def topk_encode(x, k, x0=None, acc=None, acc_mode=DPZ_ACC_NONE, vals_src=None, counter=None,
                idx_out=None, val_out=None, workspace=None, exact=False, asynchronous=False,
                phase=None, co_replace=None, status_out=None, shared=False, fold_base=None,
                val_fp16=False, hint=False, keep_x=False):
    """Top-k magnitude encode (reference PartialModel.py:164-255 / Wavelet.py:142-197).

    Returns ``(idx int32[k], val fp32[k])`` in ascending index order.  Mutates ``acc`` and
    ``counter`` in place like the reference mutates ``model.accumulated_changes`` and
    ``model.shared_parameters_counter``.  With ``asynchronous=True`` the call only enqueues
    work; call :func:`topk_complete` with the same arguments before reading the result.
    ``phase="stream"`` / ``"tail"`` split the enqueue in two (both asynchronous; see
    DPZ_TOPK_STREAM in dpz_codec.h) so independent work can overlap the latency-bound tail.
    ``co_replace=(local, idx, vals, out)`` also performs the independent decode
    ``replace(local, idx, vals, out=out)`` of a received payload inside the encoder's
    latency-bound selection launches (dpz_topk_encode_replace); it is complete when the encode's
    stream work is.  ``status_out`` (a 1-element int32 device tensor or view): asynchronous
    encode whose final status word (0 = final, else re-run with ``exact=True``) is written there
    on the device (dpz_topk_encode_status).  ``shared``: several codecs run concurrently on the
    GPU (DPZ_TOPK_SHARED: the smaller filter grid); identical results.
    ``fold_base=(base_out, weights, w_self)``: also write the no-hit base of the coming
    Metro-Hastings fold over x with those weights into ``base_out`` (dpz_topk_encode_foldbase;
    the filter writes it as it streams x), for a later ``decode_average(x, payloads, weights,
    w_self, out=base_out, base_ready=True)``.
    ``val_fp16``: the values are written as fp16 (round to nearest even, ``torch.half``), by the
    encode itself (DPZ_TOPK_VAL_FP16: the C5 payload's value packing); ``val`` is float16[k].
    ``hint``: a node's next round — take the key window from the previous encode's exact
    threshold on this ``workspace`` when that encode had the same n, k and key source, skipping
    the sample launch (DPZ_TOPK_HINT; a window that no longer brackets the k-th key misses and a
    blocking call re-runs the sampled path).  ``keep_x``: x is read again right after (the node's
    fold over its own model): stream it with the default cache policy (DPZ_TOPK_KEEP_X).  Both
    leave the result unchanged.
    """
    _require(x, torch.float32, "x")
    _require(x0, torch.float32, "x0")
    _require(acc, torch.float32, "acc")
    _require(counter, torch.int32, "counter")
    n = x.numel()
    k = int(k)
    if vals_src is None:
        vals_src = x
    _require(vals_src, torch.float32, "vals_src")
    if idx_out is None:
        idx_out = torch.empty(k, dtype=torch.int32, device=x.device)
    vdt = torch.float16 if val_fp16 else torch.float32
    if val_out is None:
        val_out = torch.empty(k, dtype=vdt, device=x.device)
    _require(val_out, vdt, "val_out")
    if val_fp16 and (co_replace is not None or fold_base is not None):
        raise ValueError("val_fp16: a plain encode (no co_replace / fold_base)")
    wso = workspace or Workspace(x.device)
    ws = wso.get(n, k)
    flags = ((DPZ_TOPK_EXACT if exact else 0) | (DPZ_TOPK_ASYNC if asynchronous else 0)
             | (_lib.DPZ_TOPK_SHARED if shared else 0)
             | (_lib.DPZ_TOPK_VAL_FP16 if val_fp16 else 0)
             | (_lib.DPZ_TOPK_KEEP_X if keep_x else 0))
    # the device checks the prior's signature itself; this only avoids a predictable miss
    hkey = (n, k, bool(shared), int(acc_mode), x0 is not None)
    if hint and not exact and wso.hint_key == hkey:
        flags |= _lib.DPZ_TOPK_HINT
    wso.hint_key = None if exact else hkey
    if phase is not None:
        flags |= {"stream": DPZ_TOPK_STREAM, "tail": DPZ_TOPK_TAIL}[phase]
    if fold_base is not None:
        base_out, fw, fws = fold_base
        _require(base_out, torch.float32, "base_out")
        if base_out.numel() != n:
            raise ValueError("fold base: base_out must hold n values")
        if co_replace is not None or phase is not None or status_out is not None:
            raise ValueError("fold_base: a whole encode without co_replace / phase / status_out")
        nw = len(fw)
        w_arr = (ctypes.c_float * max(nw, 1))(*[float(v) for v in fw])
        rc = _lib.lib().dpz_topk_encode_foldbase(
            _ptr(x), _ptr(x0), _ptr(acc), int(acc_mode), _ptr(vals_src), n, k, _ptr(idx_out),
            _ptr(val_out), _ptr(counter), _ptr(ws), ws.numel(), flags, nw, w_arr, float(fws),
            _ptr(base_out), _stream(x.device))
        check(rc, "dpz_topk_encode_foldbase")
        return idx_out, val_out
    if status_out is not None:
        _require(status_out, torch.int32, "status_out")
        if co_replace is not None or phase is not None or exact:
            raise ValueError("status_out: a plain sampled-path encode only")
        rc = _lib.lib().dpz_topk_encode_status(_ptr(x), _ptr(x0), _ptr(acc), int(acc_mode),
                                               _ptr(vals_src), n, k, _ptr(idx_out), _ptr(val_out),
                                               _ptr(counter), _ptr(ws), ws.numel(),
                                               _ptr(status_out),
                                               (_lib.DPZ_TOPK_SHARED if shared else 0)
                                               | (_lib.DPZ_TOPK_VAL_FP16 if val_fp16 else 0),
                                               _stream(x.device))
        check(rc, "dpz_topk_encode_status")
        return idx_out, val_out
    if co_replace is None:
        rc = _lib.lib().dpz_topk_encode(_ptr(x), _ptr(x0), _ptr(acc), int(acc_mode),
                                        _ptr(vals_src), n, k, _ptr(idx_out), _ptr(val_out),
                                        _ptr(counter), _ptr(ws), ws.numel(), flags,
                                        _stream(x.device))
        check(rc, "dpz_topk_encode")
        return idx_out, val_out
    if phase is not None:
        raise ValueError("co_replace cannot be combined with a phase split")
    r_local, r_idx, r_val, r_out = co_replace
    _require(r_local, torch.float32, "co_replace local")
    _require(r_idx, torch.int32, "co_replace idx")
    _require(r_val, torch.float32, "co_replace vals")
    _require(r_out, torch.float32, "co_replace out")
    if r_idx.numel() != r_val.numel() or r_out.numel() != r_local.numel():
        raise ValueError("co_replace: idx/vals or local/out sizes differ")
    r_n = r_local.numel()
    dws = (workspace or Workspace(x.device)).get_decode(r_n, 1)
    rc = _lib.lib().dpz_topk_encode_replace(
        _ptr(x), _ptr(x0), _ptr(acc), int(acc_mode), _ptr(vals_src), n, k, _ptr(idx_out),
        _ptr(val_out), _ptr(counter), _ptr(ws), ws.numel(), flags, _ptr(r_local), _ptr(r_idx),
        _ptr(r_val), r_idx.numel(), r_n, _ptr(r_out), _ptr(dws), dws.numel(), _stream(x.device))
    check(rc, "dpz_topk_encode_replace")
    return idx_out, val_out


def mask_words(n):
    """uint32 words of a selection mask over n elements (ceil(n / 32)); held as int32 tensors."""
    return int(_lib.lib().dpz_mask_words(int(n)))


def topk_encode_sliced(x, k, sel_mask, planes=None, x0=None, acc=None, acc_mode=DPZ_ACC_NONE,
                       vals_src=None, idx_out=None, val_out=None, workspace=None, exact=False,
                       status_out=None, shared=False, val_fp16=False, hint=False):
    """The selection of :func:`topk_encode` with its bookkeeping in coalesced form
    (dpz_topk_encode_sliced; reference Wavelet.py:194-197): ``planes`` (int32[32 * mask_words(n)],
    the bit-sliced shared_parameters_counter, or None) += 1 at the selected indices, and
    ``sel_mask`` (int32[mask_words(n)]) gets the selected bits — the accumulator rewind is left
    to the caller's next accumulating pass (``wavedec(..., rewind_mask=sel_mask)``) or
    :func:`rewind_apply`.  ``acc`` (DPZ_ACC_ADD) is only read.  Blocking unless ``status_out``
    (then asynchronous: a nonzero status means re-run with ``exact=True``).  ``hint``: the key
    window from the previous encode on ``workspace`` (as :func:`topk_encode`; a blocking call
    that misses re-runs the sampled path, then the exact one)."""
    _require(x, torch.float32, "x")
    _require(x0, torch.float32, "x0")
    _require(acc, torch.float32, "acc")
    _require(sel_mask, torch.int32, "sel_mask")
    _require(planes, torch.int32, "planes")
    n = x.numel()
    k = int(k)
    nw = mask_words(n)
    if sel_mask.numel() < nw or (planes is not None and planes.numel() < 32 * nw):
        raise ValueError("sel_mask / planes too small for n")
    if vals_src is None:
        vals_src = x
    _require(vals_src, torch.float32, "vals_src")
    if idx_out is None:
        idx_out = torch.empty(k, dtype=torch.int32, device=x.device)
    vdt = torch.float16 if val_fp16 else torch.float32
    if val_out is None:
        val_out = torch.empty(k, dtype=vdt, device=x.device)
    _require(val_out, vdt, "val_out")
    _require(status_out, torch.int32, "status_out")
    wso = workspace or Workspace(x.device)
    ws = wso.get(n, k)
    flags = ((DPZ_TOPK_EXACT if exact else 0) | (_lib.DPZ_TOPK_SHARED if shared else 0)
             | (_lib.DPZ_TOPK_VAL_FP16 if val_fp16 else 0))
    # the device checks the prior's signature itself; this only avoids a predictable miss
    hkey = (n, k, bool(shared), int(acc_mode), x0 is not None)
    if hint and not exact and wso.hint_key == hkey:
        flags |= _lib.DPZ_TOPK_HINT
    wso.hint_key = None if exact else hkey
    rc = _lib.lib().dpz_topk_encode_sliced(
        _ptr(x), _ptr(x0), _ptr(acc), int(acc_mode), _ptr(vals_src), n, k, _ptr(idx_out),
        _ptr(val_out), _ptr(planes), _ptr(sel_mask), _ptr(ws), ws.numel(), _ptr(status_out),
        flags, _stream(x.device))
    check(rc, "dpz_topk_encode_sliced")
    return idx_out, val_out


def counter_unslice(planes, n, out=None):
    """int32[n] counter from its bit planes (dpz_counter_unslice)."""
    _require(planes, torch.int32, "planes")
    if out is None:
        out = torch.empty(int(n), dtype=torch.int32, device=planes.device)
    _require(out, torch.int32, "out")
    if planes.numel() < 32 * mask_words(n) or out.numel() < int(n):
        raise ValueError("counter_unslice: size mismatch")
    check(_lib.lib().dpz_counter_unslice(_ptr(planes), int(n), _ptr(out), _stream(out.device)),
          "dpz_counter_unslice")
    return out


def counter_slice(counter, planes=None):
    """Bit planes (int32[32 * mask_words(n)]) of an int32 counter (dpz_counter_slice)."""
    _require(counter, torch.int32, "counter")
    n = counter.numel()
    if planes is None:
        planes = torch.empty(32 * mask_words(n), dtype=torch.int32, device=counter.device)
    _require(planes, torch.int32, "planes")
    if planes.numel() < 32 * mask_words(n):
        raise ValueError("counter_slice: planes too small")
    check(_lib.lib().dpz_counter_slice(_ptr(counter), n, _ptr(planes), _stream(counter.device)),
          "dpz_counter_slice")
    return planes


def counter_flush(counter, ring, seg_off, mode=_lib.DPZ_COUNTER_AUTO, workspace=None):
    """``counter[ring[j]] += 1`` for every entry of the ring's segments (dpz_counter_flush):
    ``seg_off`` (host ints, seg_off[0] = 0) delimits segments of strictly ascending indices, one
    per round's payload (reference PartialModel.py:205-207, applied on read).  ``workspace``: a
    device uint8 tensor kept by the caller (grown here when too small)."""
    _require(counter, torch.int32, "counter")
    _require(ring, torch.int32, "ring")
    m = len(seg_off) - 1
    if m < 1:
        return counter
    if int(seg_off[-1]) > ring.numel():
        raise ValueError("counter_flush: segments past the ring")
    need = int(_lib.lib().dpz_counter_flush_workspace_bytes(counter.numel()))
    if workspace is None or workspace.numel() < need:
        workspace = torch.empty(need, dtype=torch.uint8, device=counter.device)
    offs = (ctypes.c_int64 * (m + 1))(*[int(v) for v in seg_off])
    check(_lib.lib().dpz_counter_flush(_ptr(counter), counter.numel(), _ptr(ring), offs, m,
                                       int(mode), _ptr(workspace), workspace.numel(),
                                       _stream(counter.device)), "dpz_counter_flush")
    return counter


def rewind_apply(acc, sel_mask):
    """acc[i] = 0 where sel_mask has bit i (the deferred rewind on its own, dpz_rewind_apply)."""
    _require(acc, torch.float32, "acc")
    _require(sel_mask, torch.int32, "sel_mask")
    if sel_mask.numel() < mask_words(acc.numel()):
        raise ValueError("rewind_apply: mask too small")
    check(_lib.lib().dpz_rewind_apply(_ptr(acc), _ptr(sel_mask), acc.numel(), _stream(acc.device)),
          "dpz_rewind_apply")
    return acc


def topk_complete(x, k, idx_out, val_out, workspace, x0=None, acc=None, acc_mode=DPZ_ACC_NONE,
                  vals_src=None, counter=None):
    """Finish an asynchronous encode; returns True if the exact fallback had to run."""
    n = x.numel()
    if vals_src is None:
        vals_src = x
    ws = workspace.get(n, k)
    fb = ctypes.c_int(0)
    rc = _lib.lib().dpz_topk_complete(_ptr(x), _ptr(x0), _ptr(acc), int(acc_mode), _ptr(vals_src),
                                      n, int(k), _ptr(idx_out), _ptr(val_out), _ptr(counter),
                                      _ptr(ws), ws.numel(), ctypes.byref(fb), _stream(x.device))
    check(rc, "dpz_topk_complete")
    return bool(fb.value)


def topk_status(workspace):
    """Status word of the last sampled encode in ``workspace`` (0 = ok, else the exact path ran or
    must run).  Synchronises with the device."""
    if workspace.buf is None:
        return 0
    return int(workspace.buf[8:12].view(torch.int32).item())


def topk_sticky_status(workspace, clear=False):
    """OR of the final status of every sampled-path encode on ``workspace`` since the last clear
    (0 = all final).  Synchronises the current stream (dpz_topk_sticky_status)."""
    if workspace.buf is None:
        return 0
    torch.cuda.synchronize(workspace.device)  # encodes may be pending on other streams
    v = ctypes.c_int32(0)
    rc = _lib.lib().dpz_topk_sticky_status(_ptr(workspace.buf), workspace.buf.numel(),
                                           1 if clear else 0, ctypes.byref(v),
                                           _stream(workspace.device))
    check(rc, "dpz_topk_sticky_status")
    return int(v.value)


class NodeStepBatch:
    """A prepared native enqueue of m node codec steps (dpz_encode_replace_batch): node j encodes
    ``nodes[j]["x"]`` (change vs ``x0``, counter update) into its payload ``idx``/``val`` and
    replace-decodes ``decode_src(j)``'s payload over its current model ``x`` into ``out`` (the
    reference's deserialized_model starts from the receiver's state_dict, PartialModel.py:278-295;
    with ``decode_src(j) != j`` the encoder's filter writes the copy of ``x``), on
    ``streams[j % len(streams)]`` with that stream's workspace.  The pointer arrays are built
    once; :meth:`run` is one ctypes call whatever m is (the host loop is native)."""

    def __init__(self, nodes, n, k, streams, workspaces, decode_src=None, rings=None):
        """``rings``: one :class:`~decentralizepy_amd._device.RingCounter` per node (over its
        ``counter``): the encodes then update no counter and write their payload indices into
        the node's ring slot, as the PartialModel plugin does; the rings are flushed when full
        and by :meth:`flush_rings` (ordered on each node's stream)."""
        m = len(nodes)
        self.m, self.n, self.k = m, int(n), int(k)
        for d in nodes:
            for key in ("x", "x0", "out"):
                _require(d[key], torch.float32, key)
                if d[key].numel() != n:
                    raise ValueError(f"node tensor {key} must hold n elements")
            _require(d["idx"], torch.int32, "idx")
            _require(d["val"], torch.float32, "val")
            _require(d.get("counter"), torch.int32, "counter")
            if d["idx"].numel() != k or d["val"].numel() != k:
                raise ValueError("payload buffers must hold k entries")
        src = decode_src or (lambda j: j)
        P = ctypes.c_void_p * max(m, 1)
        self._x = P(*[d["x"].data_ptr() for d in nodes])
        self._x0 = P(*[d["x0"].data_ptr() for d in nodes])
        self._cnt = P(*[(d["counter"].data_ptr() if d.get("counter") is not None else 0)
                        for d in nodes])
        self._idx = P(*[d["idx"].data_ptr() for d in nodes])
        self._val = P(*[d["val"].data_ptr() for d in nodes])
        self._rl = P(*[d["x"].data_ptr() for d in nodes])
        self._ri = P(*[nodes[src(j)]["idx"].data_ptr() for j in range(m)])
        self._rv = P(*[nodes[src(j)]["val"].data_ptr() for j in range(m)])
        self._ro = P(*[d["out"].data_ptr() for d in nodes])
        S = len(streams)
        if len(workspaces) != S:
            raise ValueError("one workspace per stream")
        wbufs = [w.get(n, k) for w in workspaces]
        dbufs = [w.get_decode(n, 1) for w in workspaces]
        Q = ctypes.c_void_p * S
        self._ws = Q(*[b.data_ptr() for b in wbufs])
        self._dws = Q(*[b.data_ptr() for b in dbufs])
        self._ws_bytes = min(b.numel() for b in wbufs)
        self._dws_bytes = min(b.numel() for b in dbufs)
        self._streams = Q(*[s.cuda_stream for s in streams])
        self._S = S
        self.workspaces = workspaces
        self._keep = (nodes, wbufs, dbufs, streams)
        self._rings = rings
        if rings is not None:
            if len(rings) != m:
                raise ValueError("one ring per node")
            self._src = [src(j) for j in range(m)]
            self._tstreams = list(streams)
            self._cnt = P(*([0] * m))  # no counter update in the encodes
            # the last committed payload of every node (its own buffer until the first encode)
            self._last = [d["idx"].data_ptr() for d in nodes]

    def _ring_slot(self, j):
        """Node j's next ring slot; a full ring is flushed first, on node j's stream."""
        r = self._rings[j]
        if r.ring is None or r.segs[-1] + self.k > r.ring.numel() or len(r.segs) > r.MAX_SEGS:
            with torch.cuda.stream(self._tstreams[j % self._S]):
                return r.slot(self.k)
        return r.slot(self.k)

    def flush_rings(self):
        """Every node's deferred counter updates into its counter, on its stream."""
        if self._rings is None:
            return
        for j, r in enumerate(self._rings):
            if r.pending_rounds():
                with torch.cuda.stream(self._tstreams[j % self._S]):
                    r.flush()

    def run(self, what=_lib.DPZ_BATCH_ENCODE | _lib.DPZ_BATCH_DECODE, m=None):
        """``what`` with DPZ_BATCH_HINT: the encodes take the prior window (DPZ_TOPK_HINT) —
        after this batch's first encoding run every encode, the first on each stream too."""
        m = self.m if m is None else int(m)
        if what & _lib.DPZ_BATCH_HINT and what & _lib.DPZ_BATCH_ENCODE:
            if getattr(self, "_primed", False):
                what = (what & ~_lib.DPZ_BATCH_HINT) | _lib.DPZ_BATCH_HINT_ALL
            self._primed = True
        idx, ri = self._idx, self._ri
        enc = bool(what & _lib.DPZ_BATCH_ENCODE)
        if self._rings is not None:
            P = ctypes.c_void_p * max(self.m, 1)
            new = [self._ring_slot(j).data_ptr() if enc else self._last[j] for j in range(m)]
            idx = P(*(new + [0] * (self.m - m)))
            # a payload encoded earlier in this run (src < j, same stream) is the new slot
            ri = P(*([(new[q] if (enc and q < j) else self._last[q])
                      for j, q in ((j, self._src[j]) for j in range(m))] + [0] * (self.m - m)))
        rc = _lib.lib().dpz_encode_replace_batch(
            m, int(what), self._x, self._x0, self.n, self.k, self._cnt, idx, self._val,
            self._rl, ri, self._rv, self.k, self._ro, self._ws, self._ws_bytes, self._dws,
            self._dws_bytes, self._S, self._streams)
        check(rc, "dpz_encode_replace_batch")
        if self._rings is not None and enc:
            for j in range(m):
                self._rings[j].commit(self.k)
                self._last[j] = new[j]

    def sticky_status(self, clear=False):
        """OR of every encode's final status on these workspaces since the last clear."""
        v = 0
        for w in self.workspaces:
            v |= topk_sticky_status(w, clear)
        return v


def decode_average(local, payloads, weights=None, w_self=None, out=None, replace_only=False,
                   workspace=None, zero_base=False, add_only=False, accumulate=False,
                   also_local=False, base_ready=False):
    """Batched replace + Metro-Hastings fold (reference Sharing.py:156-229, PartialModel.py:257-303).

    payloads : list of ``(idx int32 device tensor or None, vals fp32 device tensor)``
    weights  : per-payload weights (Python floats, rounded to fp32 like torch does)
    w_self   : weight of the local term, or None for no self term (server variant)
    zero_base: sparse payloads are zero off their indices (STC's ``T = zeros; T[idx] = params``)
               and the fold starts from +0.0 (DPZ_FOLD_ZERO_BASE)
    add_only : one payload, ``out = local + T`` with T zero-based (DPZ_FOLD_ADD_ONLY)
    accumulate: ``out`` holds a running total the fold continues (DPZ_FOLD_ACCUMULATE)
    also_local: the result is also written over ``local`` in place (DPZ_FOLD_ALSO_LOCAL)
    base_ready: ``out`` already holds this fold's no-hit base over ``local`` (written by
               ``topk_encode(..., fold_base=(out, weights, w_self))``): only the elements the
               payloads hit are rewritten (DPZ_FOLD_BASE_READY)
    """
    _require(local, torch.float32, "local")
    n = local.numel()
    if out is None:
        out = torch.empty_like(local)
    _require(out, torch.float32, "out")
    npay = len(payloads)
    idx_arr = (ctypes.c_void_p * max(npay, 1))()
    val_arr = (ctypes.c_void_p * max(npay, 1))()
    k_arr = (ctypes.c_int64 * max(npay, 1))()
    w_arr = (ctypes.c_float * max(npay, 1))()
    for i, (idx, vals) in enumerate(payloads):
        _require(idx, torch.int32, "idx")
        _require(vals, torch.float32, "vals")
        if idx is not None and idx.numel() != vals.numel():
            raise ValueError("payload idx and vals differ in length")
        if idx is None and vals.numel() != n:
            raise ValueError("a dense payload (idx=None) must hold n values")
        idx_arr[i] = idx.data_ptr() if idx is not None else None
        val_arr[i] = vals.data_ptr()
        k_arr[i] = vals.numel()
        w_arr[i] = float(weights[i]) if weights is not None else 1.0
    flags = ((DPZ_FOLD_SELF if w_self is not None else 0)
             | (DPZ_FOLD_REPLACE_ONLY if replace_only else 0)
             | (_lib.DPZ_FOLD_ZERO_BASE if zero_base else 0)
             | (_lib.DPZ_FOLD_ADD_ONLY if add_only else 0)
             | (_lib.DPZ_FOLD_ACCUMULATE if accumulate else 0)
             | (_lib.DPZ_FOLD_ALSO_LOCAL if also_local else 0)
             | (_lib.DPZ_FOLD_BASE_READY if base_ready else 0))
    ws = (workspace or Workspace(local.device)).get_decode(n, npay)
    rc = _lib.lib().dpz_decode_average(_ptr(local), n, npay, idx_arr, val_arr, k_arr, w_arr,
                                       float(w_self) if w_self is not None else 0.0, flags,
                                       _ptr(out), _ptr(ws), ws.numel(), _stream(local.device))
    check(rc, "dpz_decode_average")
    return out


def topk_threshold(x, k, workspace=None, cap=None):
    """Choco's threshold selection (reference sharing/Choco.py:117-161): every element with
    ``|x| >= T`` (T = the k-th largest |x|, all ties kept; 0 when k == 0) that is nonzero, in
    ascending index order.  Returns ``(idx int32[c], vals fp32[c])`` (blocks for the count)."""
    _require(x, torch.float32, "x")
    n = x.numel()
    cap = n if cap is None else int(cap)
    idx = torch.empty(max(cap, 1), dtype=torch.int32, device=x.device)
    val = torch.empty(max(cap, 1), dtype=torch.float32, device=x.device)
    ws = (workspace or Workspace(x.device)).get(n, int(k))
    cnt = ctypes.c_int64(0)
    rc = _lib.lib().dpz_topk_threshold(_ptr(x), n, int(k), _ptr(idx), _ptr(val), cap, _ptr(ws),
                                       ws.numel(), ctypes.byref(cnt), _stream(x.device))
    check(rc, "dpz_topk_threshold")
    c = int(cnt.value)
    return idx[:c], val[:c]


def mask_below_threshold(x, workspace, out=None):
    """``x[|x| < T] = 0`` with T of the last :func:`topk_threshold` on ``workspace``."""
    _require(x, torch.float32, "x")
    out = x if out is None else out
    rc = _lib.lib().dpz_mask_below_threshold(_ptr(x), x.numel(), _ptr(workspace.buf), _ptr(out),
                                             _stream(x.device))
    check(rc, "dpz_mask_below_threshold")
    return out


def elementwise(op, a, b, d=None, c=0.0, out=None):
    """fp32 elementwise helpers of the Choco update (DPZ_EW_SUB / ADD / CHOCO)."""
    for t, nm in ((a, "a"), (b, "b"), (d, "d")):
        _require(t, torch.float32, nm)
    if out is None:
        out = torch.empty_like(a)
    rc = _lib.lib().dpz_elementwise(int(op), _ptr(a), _ptr(b), _ptr(d), float(c), a.numel(),
                                    _ptr(out), _stream(a.device))
    check(rc, "dpz_elementwise")
    return out


def replace(local, idx, vals, out=None, workspace=None):
    """``T = local.clone(); T[idx] = vals`` (reference PartialModel.py:292-295)."""
    return decode_average(local, [(idx, vals)], out=out, replace_only=True, workspace=workspace)


WAVELETS = ("sym2", "haar")  # the fused kernels (dpz_dwt.hip, dpz_haar.hip)
_BANKS = None
_BANK_DEV = {}


def _bank_table():
    """pywt's fp32 filter banks (decentralizepy_amd/wavelet_filters.json, generated from
    PyWavelets 1.1.1 by tools/gen_wavelet_filters.py)."""
    global _BANKS
    if _BANKS is None:
        import json
        import os
        with open(os.path.join(os.path.dirname(os.path.abspath(__file__)),
                               "wavelet_filters.json")) as f:
            _BANKS = json.load(f)["wavelets"]
    return _BANKS


def wavelet_names():
    """Every wavelet the device kernels implement: sym2 / haar (fused kernels) and every other
    pywt discrete wavelet with an even filter length <= 64 (dpz_dwt_generic)."""
    return sorted(set(WAVELETS) | set(_bank_table()))


def filter_len(wavelet):
    _check_wavelet(wavelet)
    return {"sym2": 4, "haar": 2}.get(wavelet) or len(_bank_table()[wavelet][0])


def _check_wavelet(wavelet):
    if wavelet not in WAVELETS and wavelet not in _bank_table():
        raise NotImplementedError(
            f"wavelet '{wavelet}': the device kernels implement sym2, haar and the pywt discrete "
            f"wavelets with filter length <= 64 ({len(_bank_table())} names, wavelet_names())")


def _fused(wavelet, level):
    """sym2 to level 4 and haar to level 8 run the fused kernels; every other (wavelet, level)
    the generic-filter path."""
    return (wavelet == "sym2" and int(level) <= 4) or (wavelet == "haar" and int(level) <= 8)


def _bank(wavelet, device):
    """The filter bank in device memory: dec_lo, dec_hi, rec_lo, rec_hi (4F fp32)."""
    key = (wavelet, str(device))
    t = _BANK_DEV.get(key)
    if t is None:
        b = np.concatenate([np.array(v, dtype=np.uint32) for v in _bank_table()[wavelet]])
        t = torch.from_numpy(b.view(np.float32).copy()).to(device)
        _BANK_DEV[key] = t
    return t


def _generic_ws(n, level, wavelet, device):
    nb = int(_lib.lib().dpz_wavelet_generic_workspace_bytes(int(n), int(level),
                                                            filter_len(wavelet)))
    return torch.empty(max(1, (nb + 3) // 4), dtype=torch.float32, device=device), nb


def wavedec_len(n, level=4, wavelet="sym2"):
    _check_wavelet(wavelet)
    if _fused(wavelet, level):
        fn = _lib.lib().dpz_wavedec_len if wavelet == "sym2" else _lib.lib().dpz_haar_wavedec_len
        m = int(fn(int(n), int(level)))
    else:
        m = int(_lib.lib().dpz_wavedec_len_generic(int(n), int(level), filter_len(wavelet)))
    if m < 0:
        # a level whose input is shorter than the filter (pywt's multi-reflection branch) or a
        # level past the kernels' 8: not implemented on the device (Wavelet's documented error)
        raise NotImplementedError(f"{wavelet} level-{level} wavedec unsupported for n={n}")
    return m


def wavedec(x, level=4, x0=None, want_x=True, coeffs_x=None, coeffs_diff=None, accumulate=False,
            wavelet="sym2", rewind_mask=None):
    """Multilevel DWT (mode "symmetric"; ``wavelet`` "sym2" / "haar" on the fused kernels, any
    other name of :func:`wavelet_names` on dpz_dwt_generic) as one ``coeffs_to_array`` vector
    (reference Wavelet.py:12-32).

    Returns ``(W(x) or None, W(x - x0) or None)``; with ``accumulate=True`` adds W(x - x0) into
    ``coeffs_diff`` instead of overwriting it.  ``rewind_mask`` (with ``accumulate``, no W(x)): the
    selection mask of :func:`topk_encode_sliced` — the deferred rewind is applied first,
    ``acc = (selected ? 0 : acc) + W(x - x0)`` (dpz_dwt_sym2_rewind / dpz_dwt_haar_rewind).
    """
    if rewind_mask is not None:
        if not accumulate or want_x or coeffs_diff is None or x0 is None:
            raise ValueError("rewind_mask: an accumulating W(x - x0) pass into coeffs_diff only")
        _require(x, torch.float32, "x")
        _require(x0, torch.float32, "x0")
        _require(coeffs_diff, torch.float32, "coeffs_diff")
        _require(rewind_mask, torch.int32, "rewind_mask")
        n = x.numel()
        m = wavedec_len(n, level, wavelet)
        if coeffs_diff.numel() != m or x0.numel() != n or rewind_mask.numel() < mask_words(m):
            raise ValueError("rewind_mask: size mismatch")
        if not _fused(wavelet, level):
            ws, nb = _generic_ws(n, level, wavelet, x.device)
            rc = _lib.lib().dpz_dwt_generic(
                _ptr(x), _ptr(x0), n, int(level), _ptr(_bank(wavelet, x.device)),
                filter_len(wavelet), None, _ptr(coeffs_diff), 1, _ptr(rewind_mask), _ptr(ws), nb,
                _stream(x.device))
            check(rc, f"dpz_dwt_generic({wavelet})")
            return None, coeffs_diff
        fn = (_lib.lib().dpz_dwt_sym2_rewind if wavelet == "sym2"
              else _lib.lib().dpz_dwt_haar_rewind)
        rc = fn(_ptr(x), _ptr(x0), n, int(level), _ptr(coeffs_diff), _ptr(rewind_mask),
                _stream(x.device))
        check(rc, f"dpz_dwt_{wavelet}_rewind")
        return None, coeffs_diff
    _require(x, torch.float32, "x")
    _require(x0, torch.float32, "x0")
    n = x.numel()
    m = wavedec_len(n, level, wavelet)
    if want_x and coeffs_x is None:
        coeffs_x = torch.empty(m, dtype=torch.float32, device=x.device)
    if x0 is not None and coeffs_diff is None:
        if accumulate:
            raise ValueError("accumulate needs coeffs_diff")
        coeffs_diff = torch.empty(m, dtype=torch.float32, device=x.device)
    for t, nm in ((coeffs_x if want_x else None, "coeffs_x"),
                  (coeffs_diff if x0 is not None else None, "coeffs_diff")):
        _require(t, torch.float32, nm)
        if t is not None and t.numel() != m:
            raise ValueError(f"{nm} must hold wavedec_len(n, level) = {m} values")
    if x0 is not None and x0.numel() != n:
        raise ValueError("x0 must match x")
    if not _fused(wavelet, level):
        ws, nb = _generic_ws(n, level, wavelet, x.device)
        rc = _lib.lib().dpz_dwt_generic(
            _ptr(x), _ptr(x0), n, int(level), _ptr(_bank(wavelet, x.device)), filter_len(wavelet),
            _ptr(coeffs_x if want_x else None), _ptr(coeffs_diff if x0 is not None else None),
            1 if accumulate else 0, None, _ptr(ws), nb, _stream(x.device))
        check(rc, f"dpz_dwt_generic({wavelet})")
    else:
        fn = _lib.lib().dpz_dwt_sym2 if wavelet == "sym2" else _lib.lib().dpz_dwt_haar
        rc = fn(_ptr(x), _ptr(x0), n, int(level), _ptr(coeffs_x if want_x else None),
                _ptr(coeffs_diff if x0 is not None else None), 1 if accumulate else 0,
                _stream(x.device))
        check(rc, f"dpz_dwt_{wavelet}")
    return (coeffs_x if want_x else None), (coeffs_diff if x0 is not None else None)


def waverec(coeffs, n, level=4, out=None, wavelet="sym2"):
    """Multilevel IDWT (any wavelet of :func:`wavelet_names`), first n outputs (reference
    Wavelet.py:311-316)."""
    _require(coeffs, torch.float32, "coeffs")
    if coeffs.numel() != wavedec_len(n, level, wavelet):
        raise ValueError("coeffs must hold wavedec_len(n, level) values")
    if out is None:
        out = torch.empty(int(n), dtype=torch.float32, device=coeffs.device)
    _require(out, torch.float32, "out")
    if out.numel() < int(n):
        raise ValueError("out must hold n values")
    if not _fused(wavelet, level):
        ws, nb = _generic_ws(n, level, wavelet, coeffs.device)
        rc = _lib.lib().dpz_idwt_generic(_ptr(coeffs), int(n), int(level),
                                         _ptr(_bank(wavelet, coeffs.device)), filter_len(wavelet),
                                         _ptr(out), _ptr(ws), nb, _stream(coeffs.device))
        check(rc, f"dpz_idwt_generic({wavelet})")
        return out
    fn = _lib.lib().dpz_idwt_sym2 if wavelet == "sym2" else _lib.lib().dpz_idwt_haar
    rc = fn(_ptr(coeffs), int(n), int(level), _ptr(out), _stream(coeffs.device))
    check(rc, f"dpz_idwt_{wavelet}")
    return out


def scatter_fill(dst, idx, value):
    """``dst[idx] = value`` (reference models/Model.py:53-64 rewind_accumulation)."""
    _require(dst, torch.float32, "dst")
    _require(idx, torch.int32, "idx")
    rc = _lib.lib().dpz_scatter_fill(_ptr(dst), dst.numel(), _ptr(idx), idx.numel(), float(value),
                                     _stream(dst.device))
    check(rc, "dpz_scatter_fill")
    return dst


def pack_fp16(x, out=None):
    _require(x, torch.float32, "x")
    if out is None:
        out = torch.empty(x.numel(), dtype=torch.float16, device=x.device)
    rc = _lib.lib().dpz_pack_fp16(_ptr(x), x.numel(), _ptr(out), _stream(x.device))
    check(rc, "dpz_pack_fp16")
    return out


def unpack_fp16(h, out=None):
    _require(h, torch.float16, "h")
    if out is None:
        out = torch.empty(h.numel(), dtype=torch.float32, device=h.device)
    rc = _lib.lib().dpz_unpack_fp16(_ptr(h), h.numel(), _ptr(out), _stream(h.device))
    check(rc, "dpz_unpack_fp16")
    return out


def elias_encode(idx, out=None, workspace=None):
    """Elias-gamma stream of a strictly increasing device int32 index array (k >= 2).

    Returns a device uint8 view of exactly the reference's byte count (compression/Elias.py:20-52).
    """
    _require(idx, torch.int32, "idx")
    k = idx.numel()
    if k < 2:
        raise IndexError("Elias coding needs at least two indices (reference Elias.py:38-46)")
    cap = int(_lib.lib().dpz_elias_max_bytes(k))
    if out is None or out.numel() < cap:
        out = torch.empty(cap, dtype=torch.uint8, device=idx.device)
    workspace = workspace or Workspace(idx.device)
    ws = workspace.get_elias(k, 0)
    nbytes = ctypes.c_int64(0)
    rc = _lib.lib().dpz_elias_encode(_ptr(idx), k, _ptr(out), out.numel(), ctypes.byref(nbytes),
                                     _ptr(ws), ws.numel(), _stream(idx.device))
    if rc == _lib.DPZ_ERR_ARG:
        raise ValueError("Elias coding needs strictly increasing indices")
    check(rc, "dpz_elias_encode")
    return out[:nbytes.value]


def elias_decode(buf, nbytes, nbits, first, count, dtype=torch.int64, workspace=None):
    """Values of an Elias-gamma stream held on the device (compression/Elias.py:54-97).

    ``buf`` is a device uint8 tensor with at least round_up(nbytes, 4) + 16 bytes; ``nbits`` and
    ``first`` come from the stream's trailer; ``count`` bounds the output (the stream encodes at
    most (nbits - 128) + 1 values).
    """
    _require(buf, torch.uint8, "buf")
    if buf.numel() < ((nbytes + 3) // 4) * 4 + 16:
        raise ValueError("buf must be padded to round_up(nbytes, 4) + 16 bytes")
    out = torch.empty(max(count, 1), dtype=dtype, device=buf.device)
    workspace = workspace or Workspace(buf.device)
    ws = workspace.get_elias(2, nbytes)
    n = ctypes.c_int64(0)
    o64 = out if dtype == torch.int64 else None
    o32 = out if dtype == torch.int32 else None
    if o64 is None and o32 is None:
        raise ValueError("dtype must be torch.int64 or torch.int32")
    rc = _lib.lib().dpz_elias_decode(_ptr(buf), nbytes, nbits, first, _ptr(o64), _ptr(o32),
                                     out.numel(), ctypes.byref(n), _ptr(ws), ws.numel(),
                                     _stream(buf.device))
    if rc == _lib.DPZ_ERR_ARG:
        raise ValueError("malformed Elias stream")
    check(rc, "dpz_elias_decode")
    return out[:n.value]


def elias_decode_async(buf, nbytes, nbits, first, count, status, dtype=torch.int32,
                       workspace=None):
    """``elias_decode`` with no host synchronisation: the caller knows the value count (the
    payload's other leg) and passes a device int32 status word, OR-ed nonzero on the stream when
    the stream is malformed or holds a different count (the values are then unspecified).  Read
    the status once, after the round's folds (PartialModel.decompress_data's device path)."""
    _require(buf, torch.uint8, "buf")
    _require(status, torch.int32, "status")
    if buf.numel() < ((nbytes + 3) // 4) * 4 + 16:
        raise ValueError("buf must be padded to round_up(nbytes, 4) + 16 bytes")
    if count < 1:
        raise ValueError("count must be >= 1")
    if dtype not in (torch.int64, torch.int32):
        raise ValueError("dtype must be torch.int64 or torch.int32")
    out = torch.empty(count, dtype=dtype, device=buf.device)
    workspace = workspace or Workspace(buf.device)
    ws = workspace.get_elias(2, nbytes)
    o64 = out if dtype == torch.int64 else None
    o32 = out if dtype == torch.int32 else None
    rc = _lib.lib().dpz_elias_decode_async(_ptr(buf), nbytes, nbits, first, _ptr(o64), _ptr(o32),
                                           count, _ptr(status), _ptr(ws), ws.numel(),
                                           _stream(buf.device))
    if rc == _lib.DPZ_ERR_ARG:
        raise ValueError("malformed Elias stream")
    check(rc, "dpz_elias_decode_async")
    return out


def fpz_encode(x, precision=0, out=None, workspace=None):
    """Block-floating stream of a device fp32 vector (csrc/dpz_fpz.hip; the float leg of
    compression/EliasFpzip.py:19-51 at precision 0 and EliasFpzipLossy.py:14-58 at precision p).
    Returns a device uint8 view of exactly the stream's bytes."""
    _require(x, torch.float32, "x")
    n = x.numel()
    cap = int(_lib.lib().dpz_fpz_max_bytes(n))
    if out is None or out.numel() < cap:
        out = torch.empty(cap, dtype=torch.uint8, device=x.device)
    need = int(_lib.lib().dpz_fpz_workspace_bytes(n))
    workspace = workspace or Workspace(x.device)
    if workspace.ebuf is None or workspace.ebuf.numel() < need:
        workspace.ebuf = torch.empty(max(need, 256), dtype=torch.uint8, device=x.device)
    ws = workspace.ebuf
    nbytes = ctypes.c_int64(0)
    rc = _lib.lib().dpz_fpz_encode(_ptr(x), n, int(precision), _ptr(out), out.numel(),
                                   ctypes.byref(nbytes), _ptr(ws), ws.numel(), _stream(x.device))
    if rc == _lib.DPZ_ERR_UNSUPPORTED:
        raise ValueError("float precision must be 0 (lossless) or 10..32")
    check(rc, "dpz_fpz_encode")
    return out[:nbytes.value]


def fpz_decode(buf, n, precision, out=None, check_status=True, status=None):
    """Values of a block-floating stream held on the device (a uint8 tensor of the whole stream,
    4-byte aligned); ``n`` and ``precision`` come from its header.  With ``check_status`` the
    call synchronises and raises ValueError on a malformed stream; a caller's ``status`` (device
    int32 word) is OR-ed instead, with no synchronisation."""
    _require(buf, torch.uint8, "buf")
    if out is None:
        out = torch.empty(max(n, 1), dtype=torch.float32, device=buf.device)
    _require(out, torch.float32, "out")
    if out.numel() < n:
        raise ValueError("out holds fewer than n values")
    if status is None:
        status = torch.zeros(1, dtype=torch.int32, device=buf.device)
    else:
        _require(status, torch.int32, "status")
        check_status = False
    rc = _lib.lib().dpz_fpz_decode(_ptr(buf), buf.numel(), n, int(precision), _ptr(out),
                                   _ptr(status), _stream(buf.device))
    if rc == _lib.DPZ_ERR_ARG:
        raise ValueError("malformed float stream")
    if rc == _lib.DPZ_ERR_UNSUPPORTED:
        raise ValueError("float precision must be 0 (lossless) or 10..32")
    check(rc, "dpz_fpz_decode")
    if check_status and int(status.item()) != 0:
        raise ValueError("malformed float stream")
    return out[:n]


def _fft_ws(n, workspace, device):
    need = int(_lib.lib().dpz_fft_workspace_bytes(int(n)))
    if need < 0:
        raise ValueError(f"real FFT of n={n} unsupported (2 <= n < 2**31)")
    workspace = workspace or Workspace(device)
    buf = getattr(workspace, "fbuf", None)
    if buf is None or buf.numel() < max(need, 256):
        buf = workspace.fbuf = torch.empty(max(need, 256), dtype=torch.uint8, device=device)
    return buf


def rfft(x, out=None, workspace=None):
    """``torch.fft.rfft(x)`` of a device fp32 vector (reference sharing/JWINS/FFT.py:12-25):
    the native mixed-radix kernels, or hipFFT for a size with a prime factor above 4096
    (``fft_native(n)``); returns complex64[n // 2 + 1]."""
    _require(x, torch.float32, "x")
    n = x.numel()
    if out is None:
        out = torch.empty(n // 2 + 1, dtype=torch.complex64, device=x.device)
    _require(out, torch.complex64, "out")
    if out.numel() != n // 2 + 1:
        raise ValueError("out must hold n // 2 + 1 complex values")
    ws = _fft_ws(n, workspace, x.device)
    rc = _lib.lib().dpz_rfft(_ptr(x), n, _ptr(out), _ptr(ws), ws.numel(), _stream(x.device))
    check(rc, "dpz_rfft")
    return out


def fft_native(n):
    """True when rfft / irfft of n reals run this build's kernels (else hipFFT)."""
    return bool(_lib.lib().dpz_fft_native(int(n)))


def irfft(coeffs, n, out=None, workspace=None):
    """``torch.fft.irfft(coeffs, n)`` (1/n normalisation; reference sharing/JWINS/FFT.py:301).
    ``coeffs`` (complex64[n // 2 + 1]) is overwritten."""
    _require(coeffs, torch.complex64, "coeffs")
    n = int(n)
    if coeffs.numel() != n // 2 + 1:
        raise ValueError("coeffs must hold n // 2 + 1 complex values")
    if out is None:
        out = torch.empty(n, dtype=torch.float32, device=coeffs.device)
    _require(out, torch.float32, "out")
    ws = _fft_ws(n, workspace, coeffs.device)
    rc = _lib.lib().dpz_irfft(_ptr(coeffs), n, _ptr(out), _ptr(ws), ws.numel(),
                              _stream(coeffs.device))
    check(rc, "dpz_irfft")
    return out


def cplx_key(change, acc=None, acc_mode=DPZ_ACC_NONE, out=None):
    """fp32 |change| of a complex64 change vector after the DPZ_ACC_* accumulation step
    (reference PartialModel.py:315-329 + FFT.py:143-149)."""
    _require(change, torch.complex64, "change")
    _require(acc, torch.complex64, "acc")
    m = change.numel()
    if acc is not None and acc.numel() != m:
        raise ValueError("acc must match the change length")
    if out is None:
        out = torch.empty(m, dtype=torch.float32, device=change.device)
    _require(out, torch.float32, "out")
    rc = _lib.lib().dpz_cplx_key(_ptr(change), _ptr(acc), int(acc_mode), m, _ptr(out),
                                 _stream(change.device))
    check(rc, "dpz_cplx_key")
    return out


def cplx_gather(src, idx, acc=None, out=None):
    """``src[idx]`` of a complex64 vector; zeroes ``acc[idx]`` when given (Model.py:53-64)."""
    _require(src, torch.complex64, "src")
    _require(idx, torch.int32, "idx")
    _require(acc, torch.complex64, "acc")
    if out is None:
        out = torch.empty(idx.numel(), dtype=torch.complex64, device=src.device)
    _require(out, torch.complex64, "out")
    rc = _lib.lib().dpz_cplx_gather(_ptr(src), src.numel(), _ptr(idx), idx.numel(), _ptr(out),
                                    _ptr(acc), _stream(src.device))
    check(rc, "dpz_cplx_gather")
    return out


def cplx_pair_indices(idx, out=None):
    """int32[2k] ``(2 i, 2 i + 1)`` per index: a complex payload as a payload of the float view."""
    _require(idx, torch.int32, "idx")
    k = idx.numel()
    if out is None:
        out = torch.empty(2 * k, dtype=torch.int32, device=idx.device)
    _require(out, torch.int32, "out")
    rc = _lib.lib().dpz_cplx_pair_indices(_ptr(idx), k, _ptr(out), _stream(idx.device))
    check(rc, "dpz_cplx_pair_indices")
    return out


def _lz4_ws(workspace, device, need):
    workspace = workspace or Workspace(device)
    buf = getattr(workspace, "lbuf", None)
    if buf is None or buf.numel() < max(need, 256):
        buf = workspace.lbuf = torch.empty(max(need, 256), dtype=torch.uint8, device=device)
    return buf


def lz4_compress(data, out=None, workspace=None):
    """LZ4 frame of a device byte tensor (csrc/dpz_lz4.hip: independent 4 KB blocks, one wave
    each); returns a device uint8 view of exactly the frame (reference Lz4Wrapper.py:20-98)."""
    _require(data, torch.uint8, "data")
    n = data.numel()
    cap = int(_lib.lib().dpz_lz4_max_bytes(n))
    if out is None or out.numel() < cap:
        out = torch.empty(cap, dtype=torch.uint8, device=data.device)
    ws = _lz4_ws(workspace, data.device, int(_lib.lib().dpz_lz4_workspace_bytes(n, 0, 0)))
    nbytes = ctypes.c_int64(0)
    rc = _lib.lib().dpz_lz4_compress(_ptr(data), n, _ptr(out), out.numel(), ctypes.byref(nbytes),
                                     _ptr(ws), ws.numel(), _stream(data.device))
    check(rc, "dpz_lz4_compress")
    return out[:nbytes.value]


def lz4_frame_info(frame):
    """(content_size or -1, blocks, linked, block_max) of a host frame (bytes-like)."""
    b = bytes(frame)
    cs, nb, ln, bm = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int(0), ctypes.c_int64(0)
    rc = _lib.lib().dpz_lz4_frame_info(b, len(b), ctypes.byref(cs), ctypes.byref(nb),
                                       ctypes.byref(ln), ctypes.byref(bm))
    if rc == _lib.DPZ_ERR_ARG:
        raise ValueError("malformed LZ4 frame")
    check(rc, "dpz_lz4_frame_info")
    return int(cs.value), int(nb.value), bool(ln.value), int(bm.value)


def lz4_decompress(frame, device, out=None, workspace=None, max_size=None):
    """Content of an LZ4 frame (host bytes-like) decoded on ``device``; returns a device uint8
    tensor.  Linked frames (python-lz4's default) and independent frames with blocks of at most
    64 KB are supported.  The frame comes from a peer, so its header is untrusted: a stored
    content size is checked against what the blocks can hold (each decodes to at most bmax
    bytes) and against ``max_size`` BEFORE anything is allocated.  Block / content xxh32
    checksums, when the frame carries them, are skipped, not verified (the transport —
    ZeroMQ over TCP — already guarantees integrity; every decoder read and write is
    bounds-checked, so a corrupt frame cannot fault or overrun)."""
    b = frame if isinstance(frame, bytes) else bytes(frame)
    cs, nb, linked, bmax = lz4_frame_info(b)
    bound = nb * bmax
    if cs > bound or (max_size is not None and cs > int(max_size)):
        raise ValueError(f"malformed LZ4 frame: content size {cs} exceeds what its {nb} "
                         f"blocks can hold ({bound} bytes) or max_size")
    # without a stored content size the blocks bound it
    size = cs if cs >= 0 else (min(bound, int(max_size)) if max_size is not None else bound)
    if out is None or out.numel() < size:
        out = torch.empty(max(size, 1), dtype=torch.uint8, device=device)
    _require(out, torch.uint8, "out")
    # the frame goes up through a pinned buffer kept with the workspace (the call synchronizes
    # its stream before returning, so the buffer is free again when the next call starts)
    wsp = workspace or Workspace(out.device)
    pin = getattr(wsp, "lz4_pin", None)
    if pin is None or pin.numel() < max(len(b), 1):
        pin = wsp.lz4_pin = torch.empty(max(len(b), 4096), dtype=torch.uint8, pin_memory=True)
    if b:
        pin.numpy()[:len(b)] = np.frombuffer(b, dtype=np.uint8)
    # and into a device buffer kept with it (no allocation per call)
    dbuf = getattr(wsp, "lz4_dev", None)
    if dbuf is None or dbuf.numel() < max(len(b), 1) or dbuf.device != out.device:
        dbuf = wsp.lz4_dev = torch.empty(max(len(b), 4096), dtype=torch.uint8, device=out.device)
    dframe = dbuf[:max(len(b), 1)]
    dframe.copy_(pin[:max(len(b), 1)], non_blocking=True)
    workspace = wsp
    need = int(_lib.lib().dpz_lz4_workspace_bytes(0, nb, 0 if linked else bmax))
    ws = _lz4_ws(workspace, out.device, need)
    n = ctypes.c_int64(0)
    rc = _lib.lib().dpz_lz4_decompress(_ptr(dframe), b, len(b), _ptr(out), out.numel(),
                                       ctypes.byref(n), _ptr(ws), ws.numel(), _stream(out.device))
    if rc == _lib.DPZ_ERR_ARG:
        raise ValueError("malformed LZ4 frame")
    check(rc, "dpz_lz4_decompress")
    return out[:n.value]


def delta_i32(idx, out=None):
    """``np.diff(idx, prepend=0).astype(np.int32)`` of a device int32 vector."""
    _require(idx, torch.int32, "idx")
    if out is None:
        out = torch.empty_like(idx)
    rc = _lib.lib().dpz_delta_i32(_ptr(idx), idx.numel(), _ptr(out), _stream(idx.device))
    check(rc, "dpz_delta_i32")
    return out


def running_sum_i32(d, dtype=torch.int64, workspace=None):
    """``np.cumsum`` of a device int32 vector as int64 (or truncated to int32)."""
    _require(d, torch.int32, "d")
    k = d.numel()
    out = torch.empty(max(k, 1), dtype=dtype, device=d.device)
    ws = _lz4_ws(workspace, d.device, int(_lib.lib().dpz_running_sum_workspace_bytes(k)))
    rc = _lib.lib().dpz_running_sum_i32(_ptr(d), k, _ptr(out if dtype == torch.int64 else None),
                                        _ptr(out if dtype == torch.int32 else None), _ptr(ws),
                                        ws.numel(), _stream(d.device))
    check(rc, "dpz_running_sum_i32")
    return out[:k]


class KernelTimer:
    """Per-kernel device time measured by the library with HIP event pairs on each launch's own
    stream (``dpz_timing_*``).  Launches into a capturing stream are not timed.

    >>> with KernelTimer() as t:
    ...     topk_encode(...)
    >>> t.result  # {"topk_filter": (ms_total, launches), ...}
    """

    N_MAX = 64

    def __enter__(self):
        _lib.lib().dpz_timing_enable(1)
        self.result = {}
        return self

    def __exit__(self, *exc):
        self.result = self.read()
        _lib.lib().dpz_timing_enable(0)
        return False

    @classmethod
    def read(cls):
        ms = (ctypes.c_double * cls.N_MAX)()
        cnt = (ctypes.c_int64 * cls.N_MAX)()
        nk = _lib.lib().dpz_timing_read(ms, cnt, cls.N_MAX)
        out = {}
        for i in range(min(nk, cls.N_MAX)):
            if cnt[i]:
                out[_lib.lib().dpz_kernel_name(i).decode()] = (ms[i], int(cnt[i]))
        return out
