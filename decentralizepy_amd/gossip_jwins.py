"""One synchronous JWINS gossip round of a whole topology on the GPU (SURVEY.md §8d "JWINS C3
shape (b)": the topology-faithful 16 x 3 round of tutorial/JWINS/regular_16.txt).

In the reference every node is a process running ``node/DPSGDNode.py:72-115``: train, then
``sharing.get_data_to_send`` — JWINS draws ``alpha = random.choice(alpha_list)`` from a generator
seeded with the node's uid (``sharing/JWINS/JWINS.py:87-97``), ``_pre_step`` takes the wavelet
transform of the model and of its change since ``init_model`` plus the accumulated changes
(``sharing/PartialModel.py:305-331`` with T = ``Wavelet.change_transformer_wavelet``,
``Wavelet.py:12-32``), and ``serialized_model`` sends either the top-``round(alpha*M)``
coefficients of |change| with their W(x) values (counter += 1, accumulator rewound,
``Wavelet.py:142-231``) or, for ``alpha >= metadata_cap``, all of W(x) with the accumulator zeroed.
Every neighbour's payload then enters ``Wavelet._averaging`` (``Wavelet.py:269-329``): a
Metro-Hastings fold in the wavelet domain over the local W(x), in the order the node iterates its
neighbour SET, ``waverec`` back to N parameters, and ``_post_step`` (``PartialModel.py:333-353``:
``acc += W(x_new - prev)``; ``init_model = prev = x_new``).

This engine keeps every node's state resident in HBM (model, init_model, W(x), W(change),
accumulator, counter), shards the nodes over the ranks (one process per GPU) and replaces the
per-edge sends by ONE all-gather of the round's variable-size payloads: every rank draws every
node's alpha from the same uid-seeded generators, so every rank knows every payload's size and
position without exchanging them.  The per-node work is the HIP codec (DWT pair, sampled top-k
with ADD accumulation, batched coefficient-domain fold, IDWT, accumulating DWT); ``ops`` is
injectable so the round logic is tested against the numpy oracle on the CPU (gloo, world 2).
"""
import contextlib
import ctypes
import random

import torch

from .gossip import mh_weights, shard

ALIGN = 64  # payload slots start on 256-byte boundaries (the fold's 16-byte index loads)


def _al(v):
    return -(-v // ALIGN) * ALIGN


class HipJwinsOps:
    """The HIP codec behind the round (no CPU path).  The rank's nodes run as ``streams``
    concurrent codecs (node j on stream j % S, one top-k workspace each), as decentralizepy runs
    several node processes per GPU: one node's latency-bound selection tail overlaps another's
    streaming kernels.  ``fork`` / ``join`` order the streams against the caller's stream around
    each phase of the round (the fold needs every neighbour's payload)."""

    def __init__(self, device, wavelet, level, streams=3):
        from . import codec
        self.codec = codec
        self.device = device
        self.wavelet, self.level = wavelet, level
        self.streams = [torch.cuda.Stream(device) for _ in range(max(1, streams))]
        self.wss = [codec.Workspace(device) for _ in self.streams]
        self.ws = self.wss[0]

    def reserve(self, m_len, ks):
        """Size every top-k workspace for every k a round can draw, once (a workspace that grows
        mid-round would be reallocated between asynchronous encodes)."""
        for ws in self.wss:
            for k in ks:
                ws.get(m_len, k)

    def fork(self):
        cur = torch.cuda.current_stream(self.device)
        for st in self.streams:
            st.wait_stream(cur)

    def join(self):
        cur = torch.cuda.current_stream(self.device)
        for st in self.streams:
            cur.wait_stream(st)

    def on(self, j):
        """Context: node j's work goes to its stream."""
        return torch.cuda.stream(self.streams[j % len(self.streams)])

    def transform_pair(self, x, x0, wx, wc):
        self.codec.wavedec(x, self.level, x0=x0, coeffs_x=wx, coeffs_diff=wc,
                           wavelet=self.wavelet)

    def encode(self, wc, k, acc, wx, counter, idx_out, val_out, status, j=0):
        """Asynchronous: the final status word goes to ``status`` on the device."""
        self.codec.topk_encode(wc, k, acc=acc, acc_mode=self.codec.DPZ_ACC_ADD, vals_src=wx,
                               counter=counter, idx_out=idx_out, val_out=val_out,
                               workspace=self.wss[j % len(self.wss)], status_out=status,
                               shared=len(self.streams) > 1)

    # the bookkeeping in coalesced form (dpz_topk_encode_sliced): counter as bit planes, the
    # accumulator rewind deferred to the post-step's accumulating DWT (dpz_dwt_sym2_rewind)
    sliced = True

    def encode_sliced(self, wc, k, acc, wx, planes, mask, idx_out, val_out, status, j=0):
        self.codec.topk_encode_sliced(wc, k, mask, planes, acc=acc,
                                      acc_mode=self.codec.DPZ_ACC_ADD, vals_src=wx,
                                      idx_out=idx_out, val_out=val_out,
                                      workspace=self.wss[j % len(self.wss)], status_out=status,
                                      shared=len(self.streams) > 1)

    def encode_sliced_exact(self, wc, k, acc, wx, planes, mask, idx_out, val_out):
        self.codec.topk_encode_sliced(wc, k, mask, planes, acc=acc,
                                      acc_mode=self.codec.DPZ_ACC_ADD, vals_src=wx,
                                      idx_out=idx_out, val_out=val_out, workspace=self.ws,
                                      exact=True)

    def accumulate_rewind(self, acc, new, prev, mask):
        self.codec.wavedec(new, self.level, x0=prev, want_x=False, coeffs_diff=acc,
                           accumulate=True, wavelet=self.wavelet, rewind_mask=mask)

    def unslice(self, planes, m_len):
        return self.codec.counter_unslice(planes, m_len)

    def encode_exact(self, wc, k, acc, wx, counter, idx_out, val_out):
        self.codec.topk_encode(wc, k, acc=acc, acc_mode=self.codec.DPZ_ACC_ADD, vals_src=wx,
                               counter=counter, idx_out=idx_out, val_out=val_out,
                               workspace=self.ws, exact=True)

    def missed(self, status):
        """Nodes whose sampled encode missed (one host read for the whole round)."""
        return torch.nonzero(status).flatten().tolist()

    def fold_all(self, jobs, m_len):
        """jobs: (local W(x), [(idx or None, vals)], weights, w_self, out) per node; ONE batched
        native enqueue (dpz_decode_average_batch) of every node's Metro-Hastings fold."""
        from . import _lib
        from ._lib import DPZ_FOLD_SELF
        locs, outs, counts, idx, val, kk, w, ws_ = [], [], [], [], [], [], [], []
        for local, pays, wts, w_self, out in jobs:
            locs.append(local.data_ptr())
            outs.append(out.data_ptr())
            counts.append(len(pays))
            for (pi, pv), wq in zip(pays, wts):
                idx.append(pi.data_ptr() if pi is not None else None)
                val.append(pv.data_ptr())
                kk.append(pv.numel())
                w.append(wq)
            ws_.append(w_self)
        m, tot = len(jobs), max(1, len(idx))
        dws = [w_.get_decode(m_len, max(counts) if counts else 1) for w_ in self.wss]
        S = len(self.streams)
        rc = _lib.lib().dpz_decode_average_batch(  # node j on stream j % S (the streams' order)
            m, (ctypes.c_void_p * max(1, m))(*locs), (ctypes.c_void_p * max(1, m))(*outs),
            m_len, (ctypes.c_int * max(1, m))(*counts), (ctypes.c_void_p * tot)(*idx),
            (ctypes.c_void_p * tot)(*val), (ctypes.c_int64 * tot)(*kk),
            (ctypes.c_float * tot)(*w), (ctypes.c_float * max(1, m))(*ws_), DPZ_FOLD_SELF,
            (ctypes.c_void_p * S)(*[d.data_ptr() for d in dws]), min(d.numel() for d in dws), S,
            (ctypes.c_void_p * S)(*[st.cuda_stream for st in self.streams]))
        _lib.check(rc, "dpz_decode_average_batch")

    def inverse(self, tot, n, out):
        self.codec.waverec(tot, n, self.level, out=out, wavelet=self.wavelet)

    def accumulate(self, acc, new, prev):
        self.codec.wavedec(new, self.level, x0=prev, want_x=False, coeffs_diff=acc,
                           accumulate=True, wavelet=self.wavelet)


class JwinsRound:
    """Nodes [lo, hi) of a topology on this rank; ``step()`` runs one JWINS round of every node.

    Node i is uid i (the reference's Linear mapping of one process per node).  Per-node state,
    rows of (hi - lo, ·) tensors: ``x`` (the model after the round), ``x0`` (init_model == prev),
    ``acc`` (accumulated_changes, M), ``counter`` (shared_parameters_counter, M; with the HIP ops
    kept as bit planes and materialised on read, and the encode's rewind applied by the round's
    accumulating post-step — exact after every ``step()``)."""

    def __init__(self, adj, x_init, alpha_list="[0.1, 0.2, 0.3, 0.4, 1.0]", rank=0, world=1,
                 group=None, wavelet="sym2", level=4, metadata_cap=0.5, ops=None, device=None,
                 m_len=None):
        self.adj, self.n_nodes = adj, len(adj)
        self.rank, self.world, self.group = rank, world, group
        self.coll = world > 1 or group is not None  # as GossipRound.coll
        self.lo, self.hi, self.per = shard(self.n_nodes, world, rank)
        assert x_init.shape[0] == self.hi - self.lo
        self.N = x_init.shape[1]
        self.device = device or x_init.device
        self.alpha_list = eval(alpha_list) if isinstance(alpha_list, str) else list(alpha_list)
        self.metadata_cap = metadata_cap
        if m_len is None:
            from . import codec
            m_len = codec.wavedec_len(self.N, level, wavelet)
        self.M = M = int(m_len)
        self.ops = ops or HipJwinsOps(self.device, wavelet, level)
        # JWINS.__init__: random.seed(uid) in every node process; every rank replays every node's
        # draws so all payload sizes are known everywhere
        self.rngs = [random.Random(uid) for uid in range(self.n_nodes)]
        m = self.hi - self.lo

        def rows(length, dtype=torch.float32, init=None):
            # one row per node, every row starting on a 256-byte boundary (the kernels' vector
            # paths need 16-byte aligned operands; M = N + 9 is odd for sym2)
            buf = torch.zeros(m, _al(length), dtype=dtype, device=self.device)
            v = buf[:, :length]
            if init is not None:
                v.copy_(init)
            return v

        self.x = rows(self.N, init=x_init)
        self.x0 = rows(self.N, init=x_init)
        self.acc = rows(M)
        self.sliced = bool(getattr(self.ops, "sliced", False))
        if self.sliced:  # counter as bit planes + selection masks (HipJwinsOps.encode_sliced)
            from . import codec
            nw = codec.mask_words(M)
            self.planes = rows(32 * nw, torch.int32)
            self.mask = rows(nw, torch.int32)
            self.pending = [False] * m
        else:
            self._counter = rows(M, torch.int32)
        self.wx = rows(M)   # pre_share_model_transformed
        self.wc = rows(M)   # W(x - x0); the fold total reuses it
        f32 = dict(dtype=torch.float32, device=self.device)
        self.status = torch.zeros(max(1, m), dtype=torch.int32, device=self.device)
        partial = [a for a in self.alpha_list if a < metadata_cap]
        kmax = max([round(a * M) for a in partial], default=0)
        self.slot_idx = _al(kmax)
        self.slot_val = _al(max(kmax, M if any(a >= metadata_cap for a in self.alpha_list) else 0))
        self.send_idx = torch.zeros(self.per * self.slot_idx, dtype=torch.int32,
                                    device=self.device)
        self.send_val = torch.zeros(self.per * self.slot_val, **f32)
        if self.coll:
            self.recv_idx = torch.empty(world * self.per * self.slot_idx, dtype=torch.int32,
                                        device=self.device)
            self.recv_val = torch.empty(world * self.per * self.slot_val, **f32)
        self.weights = [mh_weights(adj, i) for i in range(self.n_nodes)]
        if hasattr(self.ops, "reserve"):
            self.ops.reserve(M, sorted({round(a * M) for a in partial}))
        self.alphas = None
        self.round = 0

    @property
    def counter(self):
        """shared_parameters_counter rows (materialised from the bit planes when sliced)."""
        if not self.sliced:
            return self._counter
        return torch.stack([self.ops.unslice(self.planes[j], self.M)
                            for j in range(self.hi - self.lo)]) if self.hi > self.lo else \
            torch.zeros(0, self.M, dtype=torch.int32, device=self.device)

    # ---- layout of one round's payloads ------------------------------------------------------
    def _layout(self, alphas):
        """Per node: (partial, k, idx offset, val offset) inside its rank's block, and the padded
        per-rank block sizes (identical on every rank)."""
        lay, s_idx, s_val = [None] * self.n_nodes, 0, 0
        for r in range(self.world):
            lo, hi, _ = shard(self.n_nodes, self.world, r)
            oi = ov = 0
            for q in range(lo, hi):
                partial = alphas[q] < self.metadata_cap
                k = round(alphas[q] * self.M) if partial else 0
                lay[q] = (partial, k, oi, ov)
                oi += _al(k)
                ov += _al(k if partial else self.M)
            s_idx, s_val = max(s_idx, oi), max(s_val, ov)
        return lay, max(ALIGN, s_idx), max(ALIGN, s_val)

    def _payload(self, q, lay, s_idx, s_val):
        partial, k, oi, ov = lay[q]
        r = q // self.per
        if self.coll:
            bi, bv = self.recv_idx[r * s_idx:], self.recv_val[r * s_val:]
        else:
            bi, bv = self.send_idx, self.send_val
        if partial:
            return bi[oi:oi + k], bv[ov:ov + k]
        if not self.coll:
            return None, self.wx[q - self.lo]  # the full W(x), no copy on one rank
        return None, bv[ov:ov + self.M]

    # ---- one round ---------------------------------------------------------------------------
    def _on(self, j):
        on = getattr(self.ops, "on", None)
        return on(j) if on is not None else contextlib.nullcontext()

    def _fork(self):
        if hasattr(self.ops, "fork"):
            self.ops.fork()

    def _join(self):
        if hasattr(self.ops, "join"):
            self.ops.join()

    def encode_all(self, lay):
        m = self.hi - self.lo
        self._fork()
        for j in range(m):
            q = self.lo + j
            with self._on(j):
                self.ops.transform_pair(self.x[j], self.x0[j], self.wx[j], self.wc[j])
                partial, k, oi, ov = lay[q]
                if partial and self.sliced:
                    self.ops.encode_sliced(self.wc[j], k, self.acc[j], self.wx[j], self.planes[j],
                                           self.mask[j], self.send_idx[oi:oi + k],
                                           self.send_val[ov:ov + k], self.status[j:j + 1], j=j)
                    self.pending[j] = True
                elif partial:
                    kw = {"j": j} if hasattr(self.ops, "on") else {}
                    self.ops.encode(self.wc[j], k, self.acc[j], self.wx[j], self._counter[j],
                                    self.send_idx[oi:oi + k], self.send_val[ov:ov + k],
                                    self.status[j:j + 1], **kw)
                else:  # Wavelet.py:185-192: all of W(x), accumulated changes zeroed
                    if self.sliced:
                        self.pending[j] = False
                    self.acc[j].zero_()
                    self.status[j:j + 1].zero_()
                    if self.coll:
                        self.send_val[ov:ov + self.M].copy_(self.wx[j])
        self._join()
        # a sampled-path miss (rare) left that node's payload and bookkeeping untouched: redo it
        for j in self.ops.missed(self.status[:m]):
            partial, k, oi, ov = lay[self.lo + j]
            if self.sliced:
                self.ops.encode_sliced_exact(self.wc[j], k, self.acc[j], self.wx[j],
                                             self.planes[j], self.mask[j],
                                             self.send_idx[oi:oi + k], self.send_val[ov:ov + k])
            else:
                self.ops.encode_exact(self.wc[j], k, self.acc[j], self.wx[j], self._counter[j],
                                      self.send_idx[oi:oi + k], self.send_val[ov:ov + k])

    def exchange(self, s_idx, s_val):
        if not self.coll:
            return
        import torch.distributed as dist
        dist.all_gather_into_tensor(self.recv_idx[:self.world * s_idx], self.send_idx[:s_idx],
                                    group=self.group)
        dist.all_gather_into_tensor(self.recv_val[:self.world * s_val], self.send_val[:s_val],
                                    group=self.group)

    def fold_all(self, lay, s_idx, s_val):
        jobs = []
        for j in range(self.hi - self.lo):
            nbrs, w, w_self = self.weights[self.lo + j]
            pays = [self._payload(q, lay, s_idx, s_val) for q in nbrs]
            jobs.append((self.wx[j], pays, w, w_self, self.wc[j]))
        self._fork()
        self.ops.fold_all(jobs, self.M)  # node j on stream j % S
        for j in range(self.hi - self.lo):
            with self._on(j):
                self.ops.inverse(self.wc[j], self.N, self.x[j])        # model <- waverec(total)
                if self.sliced and self.pending[j]:  # acc = (rewound ? 0 : acc) + W(x_new - prev)
                    self.ops.accumulate_rewind(self.acc[j], self.x[j], self.x0[j], self.mask[j])
                    self.pending[j] = False
                else:
                    self.ops.accumulate(self.acc[j], self.x[j], self.x0[j])  # acc += W(x_new - prev)
                self.x0[j].copy_(self.x[j])                              # init = prev = x_new
        self._join()

    def step(self):
        alphas = [rng.choice(self.alpha_list) for rng in self.rngs]
        self.alphas = alphas
        lay, s_idx, s_val = self._layout(alphas)
        self.encode_all(lay)
        self.exchange(s_idx, s_val)
        self.fold_all(lay, s_idx, s_val)
        self.round += 1
