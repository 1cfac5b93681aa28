"""One synchronous gossip round of a whole topology, nodes sharded over GPUs.

In the reference every node is its own process: ``Node`` calls ``sharing.get_data_to_send`` (top-k
encode, ``sharing/PartialModel.py:188-255``), sends the dict to each neighbour over ZeroMQ, then
``sharing._averaging`` folds the neighbours' payloads with Metro-Hastings weights
(``sharing/Sharing.py:156-190``, weight ``1 / (max(len(peer_deques), degree) + 1)``).  Simulating a
96-node round on one node of 8 MI355X, this engine keeps every node's flat model resident in HBM,
shards the nodes over the ranks (one process per GPU), and replaces the per-edge sends by ONE
all-gather of the fixed-size payloads (every node sends the same k): each rank encodes its own
nodes, ``all_gather_into_tensor`` over RCCL gives every rank every payload (96 x 8k bytes: 84 MB
at N = 11M), and each rank folds its own nodes' neighbourhoods locally — bit-exact with the
reference's per-node fold.

Over-HBM regime (BASELINE.json C4: "RCCL reduce-scatter ... only when a simulated topology's
payloads exceed one GPU's HBM"): when the all-gathered payload buffers would not fit the rank's
budget, the payloads are never replicated.  The fold is split by linearity,
``x_d' = x_d * (w_self + sum_s w_s - B_d) + A_d`` with ``A_d = sum_s w_s * v_s`` and
``B_d = sum_s w_s`` over the entries of each neighbour payload (zero elsewhere): every rank folds
the contributions of the payloads it owns into dense (A, B) rows for every destination node
(batched HIP fold, zero base), one ``reduce_scatter_tensor`` per destination group sums them on
the owning rank, which combines them with its model (``DPZ_EW_MHCOMBINE``).  Destination groups
are sized to the budget.  This path reassociates the fp32 sums (RCCL's reduction order), so it
matches the reference within fp32 tolerance, not bit for bit.

Peer exchange (``exchange="peer"``): each rank sends every other rank exactly the payloads of
its nodes that have a neighbour there — one ``all_to_all_single`` with uneven splits (grouped
point-to-point writes over xGMI on RCCL) — and folds bit-exactly as in the all-gather mode, the
local neighbours' payloads read in place.  A rank holds only the remote payloads its own
nodes' neighbourhoods name (96_regular.edges over 8 ranks: about 41 of 84 remote payloads), so
"auto" takes it over the reduce-scatter whenever those fit the budget and the all-gather does
not.

The encode / fold callables are injectable so the sharding and exchange logic can be tested with
the CPU gloo backend; the defaults are the HIP codec (no CPU fallback).
"""
import ctypes
import math

import torch


def read_edges(path):
    """Adjacency sets from a reference ``.edges`` file (``graphs/Graph.py:57-103``, type "edges":
    first line = node count, then one undirected edge "a b" per line)."""
    with open(path) as f:
        n = int(f.readline().strip())
        adj = [set() for _ in range(n)]
        for line in f:
            line = line.strip()
            if not line:
                continue
            a, b = map(int, line.split())
            adj[a].add(b)
            adj[b].add(a)
    return adj


def mh_weights(adj, i):
    """Metro-Hastings weights of node i's neighbours and the self weight, rounded exactly like
    the reference (Python doubles, ``Sharing.py:165-185``), in the reference's FOLD ORDER: the
    node folds ``peer_deques`` in the iteration order of its neighbour set
    (``node/DPSGDNode.py:111-115`` builds the averaging dict from ``graph.neighbors(uid)``, a
    ``set`` filled by ``graphs/Graph.py:57-103``).  ``read_edges`` fills the same sets in the same
    insertion order, so ``list(adj[i])`` is that order; it is NOT ascending for most nodes of
    96_regular.edges, and the fp32 fold is order-sensitive."""
    nbrs = list(adj[i])
    w = [1 / (max(len(nbrs), len(adj[j])) + 1) for j in nbrs]
    total = 0
    for v in w:
        total += v
    return nbrs, w, 1 - total


def shard(n_nodes, world, rank):
    """Contiguous node block of `rank` and the padded per-rank count for the all-gather."""
    per = math.ceil(n_nodes / world)
    lo = min(rank * per, n_nodes)
    hi = min(lo + per, n_nodes)
    return lo, hi, per


class GossipRound:
    """Nodes [lo, hi) of a topology on this rank; ``step()`` runs one full round."""

    def __init__(self, adj, x_init, alpha, rank=0, world=1, group=None, encode=None, fold=None,
                 device=None, streams=3, exchange="auto", hbm_budget=None, partial=None,
                 combine=None, node_batch=True, node_group=4, guarded=True, sliced_counter=True,
                 ring_counter=None, ring_slots=None):
        """adj: adjacency sets of all nodes; x_init: (hi - lo, N) fp32 tensor with this rank's
        nodes' flat models (device tensor for the HIP codec).

        exchange: "allgather" (bit-exact), "peer" (bit-exact; only the payloads this rank's
        neighbourhoods name), "reduce_scatter" (over-HBM) or "auto" (when world > 1 and the
        all-gathered payloads exceed ``hbm_budget`` bytes: "peer" if its payloads fit, else
        reduce-scatter; default budget: half of the device's free memory at construction).  ``partial(payloads, weights, out)``
        (zero-based weighted sum of sparse payloads) and ``combine(x, B, A, c, out)`` are
        injectable like encode / fold (CPU tests); the defaults are the HIP codec."""
        self.adj = adj
        # node_batch: the HIP encodes of this rank's nodes in groups of `node_group` nodes, one
        # launch per phase and group (dpz_topk_encode_nodes), the groups round-robin over
        # `streams`; False: node after node on the streams.  Measured on MI355X (96_regular x
        # 11M, tools/diag/c4_group_ab.sh): groups of 4 5.21 ms per round, 16: 5.24, 1: 5.36,
        # node after node 5.50-5.61; with the sliced counters (tools/diag/c4_group_sliced_ab.sh,
        # group:streams) 4:3 4.90-4.92, 8:3 4.92, 4:2 4.92-4.93, 2:3 4.97-4.99, 4:4 5.02
        self.node_batch = node_batch
        self.node_group = max(1, int(node_group))
        # guarded: (HIP, all-gather exchange) the folds follow the encodes with no host wait in
        # between, guarded on the device by the encodes' status words (_step_guarded)
        self.guarded = guarded
        self.n_nodes = len(adj)
        self.rank, self.world, self.group = rank, world, group
        # the exchange runs through the collectives with more than one rank, or whenever the
        # caller hands over a process group (one rank too: the RCCL path then runs as a loopback,
        # tests/test_gpu_rccl.py); one rank without a group exchanges in place
        self.coll = world > 1 or group is not None
        self.lo, self.hi, self.per = shard(self.n_nodes, world, rank)
        assert x_init.shape[0] == self.hi - self.lo
        self.N = x_init.shape[1]
        self.k = round(alpha * self.N)
        self.device = device or x_init.device
        self.x = x_init.contiguous().clone()
        self.x0 = x_init.contiguous().clone()  # init_model of every owned node
        # sliced_counter (HIP, node-batched encodes): every node's shared_parameters_counter as 32
        # bit planes plus a selection mask per round (DPZ_TOPK_SLICED: compact writes the mask
        # and ripple-adds it to the planes instead of k scattered counter atomics); ``counter``
        # materialises the int32 counters on read (the reference reads them once, at the end).
        # Measured on MI355X (C4, 96_regular x 11M, tools/diag/slpf_ab.sh): 4.90-4.92 ms per
        # round against 5.03-5.05 with the int32 counter.  One node per rank (no node batch) or a
        # segment geometry the sliced compact does not take (n > 2^26) falls back to the int32
        # counter (_unslice)
        self.sliced_counter = (bool(sliced_counter) and encode is None and fold is None
                               and node_batch and self.hi - self.lo > 1)
        # ring_counter (HIP, node-batched encodes; round 6, as PartialModel's RingCounter): the
        # encodes write each round's payload indices into a slot of a per-node ring of rounds and
        # update no counter at all; the int32 counters take the ring's rounds (dpz_counter_flush)
        # when read (``counter``: the reference's end-of-run dump, node/DPSGDNode.py:186-194) or
        # when the ring is full.  None: on whenever the node-batched HIP encode runs
        self.ring_counter = (encode is None and fold is None and node_batch and
                             self.hi - self.lo > 1 and (ring_counter is None or bool(ring_counter)))
        if self.ring_counter:
            self.sliced_counter = False
        self._ring = None
        if self.sliced_counter:
            from . import codec
            nw = codec.mask_words(self.N)
            self._planes = torch.zeros(self.hi - self.lo, 32 * nw, dtype=torch.int32,
                                       device=self.device)
            self._selmask = torch.zeros(self.hi - self.lo, nw, dtype=torch.int32,
                                        device=self.device)
            self._counter = None
        else:
            self._counter = torch.zeros_like(self.x, dtype=torch.int32)
        self.send_idx = torch.zeros(self.per, self.k, dtype=torch.int32, device=self.device)
        self.send_val = torch.zeros(self.per, self.k, dtype=torch.float32, device=self.device)
        gathered = self.per * world * self.k * 8
        if hbm_budget is None:
            if self.device.type == "cuda":
                hbm_budget = torch.cuda.mem_get_info(self.device)[0] // 2
            else:
                hbm_budget = float("inf")
        if self.ring_counter:
            # (per, slots, k): a node's rounds adjacent (one flush segment list per node); the
            # round's send_idx is the slot's (per, k) view.  At most an eighth of the budget.
            row = self.per * self.k * 4
            cap = 64 if hbm_budget == float("inf") else int(hbm_budget // 8 // max(1, row))
            self.ring_slots = max(2, min(64, cap)) if ring_slots is None else max(1, int(ring_slots))
            self._ring = torch.zeros(self.per, self.ring_slots, self.k, dtype=torch.int32,
                                     device=self.device)
            self._ring_used = 0
            self._flush_ws = None
            self.send_idx = self._ring[:, 0, :]
        if self.coll:
            # the exchange mode and the reduce-scatter group size decide which collectives every
            # rank issues: all ranks must derive them from ONE budget (the smallest), or ranks
            # with slightly different free memory issue mismatched collectives and hang
            import torch.distributed as dist
            dev = self.device if dist.get_backend(group) == "nccl" else torch.device("cpu")
            b = torch.tensor([float(hbm_budget)], dtype=torch.float64, device=dev)
            dist.all_reduce(b, op=dist.ReduceOp.MIN, group=group)
            hbm_budget = float(b.item())
        self.hbm_budget = hbm_budget
        self._peer_plan()
        if exchange == "auto":
            exchange = "allgather"
            if world > 1 and gathered > hbm_budget:
                exchange = "peer" if self._peer_bytes <= hbm_budget else "reduce_scatter"
        if exchange not in ("allgather", "peer", "reduce_scatter"):
            raise ValueError(f"unknown exchange {exchange!r}")
        self.exchange_mode = exchange
        if exchange == "reduce_scatter" and self.ring_counter:
            # the over-HBM legs keep their payload pointer tables across rounds: the ring's
            # moving send rows would leave them stale, so this mode keeps the int32 counters
            self.ring_counter = False
            self._ring = None
            self.send_idx = torch.zeros(self.per, self.k, dtype=torch.int32, device=self.device)
        if exchange == "peer":
            k = self.k
            n_recv = max(1, self._peer_n_recv)
            self._peer_recv = torch.empty(n_recv, 2, k, dtype=torch.int32, device=self.device)
            self._peer_send = torch.empty(max(1, len(self._peer_rows)), 2, k, dtype=torch.int32,
                                          device=self.device)
            self._peer_rows_t = torch.tensor(self._peer_rows, dtype=torch.long,
                                             device=self.device)
            self.recv_idx = self.recv_val = None
        elif exchange == "allgather":
            self.recv_idx = torch.empty(self.per * world, self.k, dtype=torch.int32,
                                        device=self.device)
            self.recv_val = torch.empty(self.per * world, self.k, dtype=torch.float32,
                                        device=self.device)
        else:
            self.recv_idx = self.recv_val = None
            self._partial = partial or self._hip_partial
            self._combine = combine or self._hip_combine
            self._ones = torch.ones(self.k, dtype=torch.float32, device=self.device)
            self._zero_local = torch.zeros(self.N, dtype=torch.float32, device=self.device)
            # destination nodes per reduce-scatter: send (A, B) rows for `world` ranks plus the
            # received pair, within the budget
            row = 4 * self.N
            g = int(hbm_budget // (2 * row * (world + 1))) if hbm_budget != float("inf") else self.per
            self.rs_group = max(1, min(self.per, g))
        self.out = torch.empty_like(self.x)
        self.leg_times = None
        # the encodes' sampled-path status words (padded to `per`: the all-gathered guard of the
        # folds, _step_guarded); the injected CPU encodes never miss and leave them 0
        self.status = torch.zeros(max(1, self.per), dtype=torch.int32, device=self.device)
        self.weights = [mh_weights(adj, i) for i in range(self.lo, self.hi)]
        self._encode = encode or self._hip_encode
        self._fold = fold or self._hip_fold
        self._hip = encode is None and fold is None
        if self._hip:
            # the nodes of this rank run as `streams` concurrent codecs (one workspace each):
            # one node's latency-bound selection tail overlaps another's streaming kernels
            from . import codec
            self.streams = [torch.cuda.Stream(self.device) for _ in range(max(1, streams))]
            self.wss = [codec.Workspace(self.device) for _ in self.streams]


    def _peer_plan(self):
        """The peer exchange's static plan (topology and sharding are fixed): for every rank the
        remote nodes its neighbourhoods name; this rank's send rows (its nodes, grouped by
        destination rank, ascending) and receive rows (the remote nodes it needs, grouped by
        source rank, ascending — the order all_to_all_single lands them in)."""
        W, per, me = self.world, self.per, self.rank
        need = [set() for _ in range(W)]
        for d in range(self.n_nodes):
            r = d // per
            for q in self.adj[d]:
                if q // per != r:
                    need[r].add(q)
        send = [sorted(q for q in need[r] if q // per == me) if r != me else [] for r in range(W)]
        recv = [sorted(q for q in need[me] if q // per == s) if s != me else [] for s in range(W)]
        self._peer_rows = [q - self.lo for r in range(W) for q in send[r]]
        flat = [q for s in range(W) for q in recv[s]]
        self._peer_row = {q: i for i, q in enumerate(flat)}
        self._peer_n_recv = len(flat)
        self._peer_in_splits = [2 * self.k * len(send[r]) for r in range(W)]
        self._peer_out_splits = [2 * self.k * len(recv[s]) for s in range(W)]
        self._peer_bytes = 8 * self.k * (len(flat) + len(self._peer_rows))

    def _payload(self, q):
        """(idx int32[k], val fp32[k]) device rows of node q's payload as this rank holds it."""
        if self.exchange_mode == "peer":
            if self.lo <= q < self.hi:
                return self.send_idx[q - self.lo], self.send_val[q - self.lo]
            row = self._peer_recv[self._peer_row[q]]
            return row[0], row[1].view(torch.float32)
        return self.recv_idx[self._slot(q)], self.recv_val[self._slot(q)]

    def _recv_key(self):
        """Identity of the buffers the fold tables point into (rebuilt when they move)."""
        if self.exchange_mode == "peer":
            return (self._peer_recv.data_ptr(), self.send_idx.data_ptr(),
                    self.send_val.data_ptr())
        return (self.recv_idx.data_ptr(), self.recv_val.data_ptr())

    @property
    def counter(self):
        """Every owned node's int32 shared_parameters_counter (m, N): the tensor itself, or with
        the sliced counter its materialised copy (dpz_counter_unslice per node) — a snapshot:
        writes into it do not reach the engine (construct with sliced_counter=False for a live
        int32 tensor)."""
        if self._ring is not None:
            self._flush_ring()
        if self._counter is not None:
            return self._counter
        from . import codec
        return torch.stack([codec.counter_unslice(self._planes[j], self.N)
                            for j in range(self.hi - self.lo)])

    def counter_row(self, j, out=None):
        """Owned node j's int32 counter alone (N values: the reference node's own
        shared_parameters_counter, node/DPSGDNode.py:186-194) — without the (m, N) stack that
        ``counter`` materialises for the sliced form; ``out`` (int32[N], device) is reused."""
        if self._ring is not None:
            self._flush_ring()
        if self._counter is not None:
            return self._counter[j] if out is None else out.copy_(self._counter[j])
        from . import codec
        return codec.counter_unslice(self._planes[j], self.N, out=out)

    def _flush_ring(self):
        """The ring's committed rounds into every owned node's int32 counter (dpz_counter_flush,
        one call per node: its rounds are adjacent in the ring), the ring emptied."""
        u = self._ring_used
        if u == 0:
            return
        from . import _lib, codec
        if self._flush_ws is None:
            need = max(256, int(_lib.lib().dpz_counter_flush_workspace_bytes(self.N)))
            self._flush_ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        offs = [i * self.k for i in range(u + 1)]
        for j in range(self.hi - self.lo):
            codec.counter_flush(self._counter[j], self._ring[j].view(-1), offs,
                                workspace=self._flush_ws)
        self._ring_used = 0

    def _ring_next(self):
        """The round's payload index buffer: the next free slot of the ring (flushed first when
        full); the slot is committed once the round's encodes are final (_ring_commit)."""
        if self._ring_used == self.ring_slots:
            self._flush_ring()
        self.send_idx = self._ring[:, self._ring_used, :]

    def _ring_commit(self):
        self._ring_used += 1

    def _unslice(self):
        """Back to the int32 counter (the node-batched sliced encode does not take this
        geometry): the planes materialised once, the node tables rebuilt."""
        m = self.hi - self.lo
        cnt = torch.empty(m, self.N, dtype=torch.int32, device=self.device)
        for j in range(m):  # row by row: no (m, N) stack beside the result
            self.counter_row(j, out=cnt[j])
        self._counter = cnt
        self._planes = self._selmask = None
        self.sliced_counter = False
        self.__dict__.pop("_node_tabs", None)

    # ---- default device implementations ---------------------------------------------------
    def _hip_encode(self, x, x0, k, counter, idx_out, val_out):
        from . import codec
        codec.topk_encode(x, k, x0=x0, counter=counter, idx_out=idx_out, val_out=val_out,
                          workspace=self.wss[0], asynchronous=True)

    def _hip_fold(self, local, payloads, weights, w_self, out):
        from . import codec
        codec.decode_average(local, payloads, weights, w_self, out=out, workspace=self.wss[0])

    # ---- one round ----------------------------------------------------------------------------
    @staticmethod
    def _ptrs(rows):
        """Host array of device pointers: the rows of a 2-D tensor (computed, no views) or the
        tensors of a list."""
        if isinstance(rows, torch.Tensor):
            base, step = rows.data_ptr(), rows.stride(0) * rows.element_size()
            return (ctypes.c_void_p * max(1, rows.shape[0]))(
                *[base + j * step for j in range(rows.shape[0])])
        return (ctypes.c_void_p * max(1, len(rows)))(*[t.data_ptr() for t in rows])

    def _stream_args(self):
        m = self.hi - self.lo
        streams = (ctypes.c_void_p * len(self.streams))(*[s.cuda_stream for s in self.streams])
        n = self.N
        k = self.k
        ws_bytes = min(w.get(n, k).numel() for w in self.wss)
        wsp = self._ptrs([w.buf for w in self.wss])
        return m, streams, ws_bytes, wsp

    def _node_table(self, m):
        """Device table of dpz_topk_encode_nodes (8 x 64-bit words per node: x, x0, counter,
        idx_out, val_out, ws, status_out, 0), one per x0 buffer (init_model swaps with the fold
        output every round, so two tables alternate)."""
        import numpy as np
        key = self.x0.data_ptr()
        tabs = self.__dict__.setdefault("_node_tabs", {})
        if key not in tabs:
            rows = []
            for j in range(m):
                sl = self.sliced_counter
                cnt = 0 if self.ring_counter else (self._planes if sl else self._counter)[j].data_ptr()
                rows.append([self.x[j].data_ptr(), self.x0[j].data_ptr(), cnt,
                             self.send_idx[j].data_ptr(),
                             self.send_val[j].data_ptr(), self.node_ws[j].buf.data_ptr(),
                             self.status.data_ptr() + 4 * j,
                             self._selmask[j].data_ptr() if sl else 0])
            tabs[key] = torch.from_numpy(np.array(rows, dtype=np.uint64).view(np.int64)).to(
                self.device)
        tab = tabs[key]
        if self.ring_counter:
            # the idx_out column at this round's slot: slot s of node j lies s * k * 4 bytes past
            # slot 0 (one small device add on the current stream, ordered before the encodes)
            if getattr(self, "_ring_col0", None) is None:
                base = self._ring[:m, 0, :]
                step = base.stride(0) * base.element_size()
                self._ring_col0 = torch.tensor([base.data_ptr() + j * step for j in range(m)],
                                               dtype=torch.int64, device=self.device)
            off = self.send_idx.data_ptr() - self._ring.data_ptr()
            torch.add(self._ring_col0, off, out=tab[:m, 3])
        return tab

    def _encode_nodes(self, m, check=True):
        """Every node's encode with one launch per phase (dpz_topk_encode_nodes): each node its
        own workspace; from the second round on every window is the node's previous one
        (DPZ_TOPK_HINT).  Returns False when (N, k) is not on the sampled path."""
        from . import _lib, codec
        if not (self.N >= (1 << 18) and 1 <= self.k <= self.N // 2):
            return False
        G = self.node_group or m
        if getattr(self, "node_ws", None) is None:
            # groups of G nodes round-robin over the S streams; a group's nodes run together, so
            # each needs its own workspace, but consecutive groups on one stream reuse the same G
            # (workspaces hot in the caches; the prior window from the node before in the slot)
            S = len(self.streams)
            slots = [[codec.Workspace(self.device) for _ in range(G)] for _ in range(S)]
            self.node_ws = [slots[(j // G) % S][j % G] for j in range(m)]
        ws_bytes = min(w.get(self.N, self.k).numel() for w in self.node_ws)
        tab = self._node_table(m)
        flags = _lib.DPZ_TOPK_HINT if getattr(self, "_primed", False) else 0
        if self.sliced_counter:
            flags |= _lib.DPZ_TOPK_SLICED
        # groups of G nodes, round-robin over the streams: one group's latency-bound selection
        # launches (and their scattered counter updates) overlap another group's filter
        cur = torch.cuda.current_stream(self.device)
        for st in self.streams:
            st.wait_stream(cur)
        for i, g0 in enumerate(range(0, m, G)):
            st = self.streams[i % len(self.streams)]
            rc = _lib.lib().dpz_topk_encode_nodes(min(G, m - g0), tab.data_ptr() + 64 * g0,
                                                  self.N, self.k, ws_bytes, flags,
                                                  ctypes.c_void_p(st.cuda_stream))
            if rc == _lib.DPZ_ERR_UNSUPPORTED and g0 == 0 and self.sliced_counter:
                # the sliced geometry check precedes every launch: nothing was enqueued
                self._unslice()
                flags &= ~_lib.DPZ_TOPK_SLICED
                tab = self._node_table(m)
                rc = _lib.lib().dpz_topk_encode_nodes(min(G, m - g0), tab.data_ptr(), self.N,
                                                      self.k, ws_bytes, flags,
                                                      ctypes.c_void_p(st.cuda_stream))
            _lib.check(rc, "dpz_topk_encode_nodes")
        for st in self.streams:
            cur.wait_stream(st)
        self._primed = True
        if check:
            self._rerun_missed(torch.nonzero(self.status[:m]).flatten().tolist())
        return True

    def _rerun_missed(self, bad):
        """A missed sampled encode wrote nothing (no counter update either): re-run those nodes'
        selections exactly (local node numbers).  Their status words are cleared after: the
        payloads are final, so a re-exchange and its folds must not see the stale miss."""
        self._rerun_encodes(bad)
        if bad:
            self.status[torch.as_tensor(list(bad), dtype=torch.long, device=self.status.device)] = 0

    def _rerun_encodes(self, bad):
        if not self._hip:
            for j in bad:
                self._encode(self.x[j], self.x0[j], self.k, self.counter[j], self.send_idx[j],
                             self.send_val[j])
            return
        from . import codec
        for j in bad:
            ws = self.node_ws[j] if getattr(self, "node_ws", None) is not None else self.wss[0]
            if self.sliced_counter:
                codec.topk_encode_sliced(self.x[j], self.k, self._selmask[j], self._planes[j],
                                         x0=self.x0[j], idx_out=self.send_idx[j],
                                         val_out=self.send_val[j], workspace=ws, exact=True)
            elif self.ring_counter:  # the round's slot: counted when the ring is flushed
                codec.topk_encode(self.x[j], self.k, x0=self.x0[j], idx_out=self.send_idx[j],
                                  val_out=self.send_val[j], workspace=ws, exact=True)
            else:
                codec.topk_encode(self.x[j], self.k, x0=self.x0[j], counter=self._counter[j],
                                  idx_out=self.send_idx[j], val_out=self.send_val[j],
                                  workspace=ws, exact=True)

    def encode_all(self, check=True):
        """Every owned node's encode.  check=False (HIP): the status words stay on the device
        for the guarded fold (step); nothing here waits for the encodes."""
        if not self._hip:
            for j in range(self.hi - self.lo):
                self._encode(self.x[j], self.x0[j], self.k, self.counter[j], self.send_idx[j],
                             self.send_val[j])
            return
        from . import _lib, codec
        m = self.hi - self.lo
        if self.ring_counter:
            self._ring_next()
            if self._encode_nodes(m, check):
                self._ring_commit()
                return
            # (n, k) off the sampled path: exact encodes into the slot, no counter update
            self._rerun_encodes(list(range(m)))
            self._ring_commit()
            return
        if self.node_batch and m > 1 and self._encode_nodes(m, check):
            return
        if self.sliced_counter:  # (n, k) off the sampled path: exact sliced encodes
            self._rerun_missed(list(range(m)))
            return
        m, streams, ws_bytes, wsp = self._stream_args()
        cur = torch.cuda.current_stream(self.device)
        for st in self.streams:
            st.wait_stream(cur)
        # one native call enqueues every node's encode (node j on stream j % S) and copies each
        # node's sampled-path status word to self.status[j]; every encode takes its key window
        # from the previous encode on its stream's workspace (DPZ_BATCH_HINT: the nodes' change
        # distributions are alike; a miss is re-run below), from the second round on the first
        # one on each stream too (HINT_ALL)
        hint = _lib.DPZ_BATCH_HINT_ALL if getattr(self, "_primed", False) else _lib.DPZ_BATCH_HINT
        self._primed = True
        rc = _lib.lib().dpz_topk_encode_batch_ex(
            m, self._ptrs(self.x[:m]), self._ptrs(self.x0[:m]), self.N, self.k,
            self._ptrs(self._counter[:m]), self._ptrs(self.send_idx[:m]),
            self._ptrs(self.send_val[:m]), wsp, ws_bytes, len(self.streams), streams,
            self.status.data_ptr(), hint)
        _lib.check(rc, "dpz_topk_encode_batch_ex")
        for st in self.streams:
            cur.wait_stream(st)
        # a sampled-path miss (rare) re-runs that node's selection exactly
        if check:
            self._rerun_missed(torch.nonzero(self.status[:m]).flatten().tolist())

    def _hip_partial(self, payloads, weights, out):
        from . import codec
        # zero base: the local operand only shapes the call (its values never enter the sum)
        codec.decode_average(self._zero_local, payloads, weights, None, out=out,
                             workspace=self.wss[0], zero_base=True)

    def _hip_combine(self, x, b, a, c, out):
        from . import codec
        from ._lib import DPZ_EW_MHCOMBINE
        codec.elementwise(DPZ_EW_MHCOMBINE, x, b, a, c, out=out)

    def _rs_tables(self):
        """Per destination group [g0, g0 + gsz): the (A, B) contribution rows this rank owns.
        Row layout of the packed send buffer (W, gsz, 2, N): destination node d = r*per + g0 + j
        of rank r is block r, row j; plane 0 = A_d, plane 1 = B_d.  Each job is (r, j, own
        payloads as (local node, weight)); rows without a job stay zero.  Built once: the
        topology and the node sharding do not change between rounds."""
        per, G = self.per, self.rs_group
        mine = set(range(self.lo, self.hi))
        groups = []
        for g0 in range(0, per, G):
            gsz = min(G, per - g0)
            jobs, empty = [], []
            for r in range(self.world):
                for j in range(gsz):
                    d = r * per + g0 + j
                    own = []
                    if d < self.n_nodes:
                        nbrs, w, _ = mh_weights(self.adj, d)
                        own = [(q - self.lo, wq) for q, wq in zip(nbrs, w) if q in mine]
                    (jobs.append((r, j, own)) if own else empty.append((r, j)))
            groups.append((g0, gsz, jobs, empty))
        return groups

    def _rs_batch_args(self, send, jobs):
        """Host tables of ONE dpz_decode_average_batch call that writes every A and B row of a
        group (zero base: A_d = sum_s w_s * v_s, B_d = sum_s w_s * 1 on the payload entries)."""
        outs, counts, idx, val, kk, w = [], [], [], [], [], []
        for plane in (0, 1):
            for r, j, own in jobs:
                outs.append(send[r, j, plane].data_ptr())
                counts.append(len(own))
                for q, wq in own:
                    idx.append(self.send_idx[q].data_ptr())
                    val.append(self.send_val[q].data_ptr() if plane == 0 else self._ones.data_ptr())
                    kk.append(self.k)
                    w.append(wq)
        m, tot = len(outs), max(1, len(idx))
        loc = (ctypes.c_void_p * max(1, m))(*([self._zero_local.data_ptr()] * m))
        return dict(m=m, local=loc, out=(ctypes.c_void_p * max(1, m))(*outs),
                    np=(ctypes.c_int * max(1, m))(*counts), idx=(ctypes.c_void_p * tot)(*idx),
                    val=(ctypes.c_void_p * tot)(*val), k=(ctypes.c_int64 * tot)(*kk),
                    w=(ctypes.c_float * tot)(*w))

    def fold_reduce_scatter(self):
        """Over-HBM exchange + fold: see the module docstring.  Per destination group: ONE batched
        zero-base fold writes this rank's (A, B) rows into one packed send buffer, ONE
        reduce-scatter sums them on the owning ranks, and each owner combines its nodes."""
        import torch.distributed as dist
        W, N = self.world, self.N
        if getattr(self, "_rs", None) is None:
            G = self.rs_group
            self._rs = self._rs_tables()
            # persistent packed buffers sized for the largest group (within the budget)
            self._rs_send = torch.zeros(W, G, 2, N, dtype=torch.float32, device=self.device)
            self._rs_recv = (torch.empty(G, 2, N, dtype=torch.float32, device=self.device)
                             if self.coll else None)
            self._rs_args = {}
        t_mark = self._leg_mark(None)  # per-leg timing (bench only, self.leg_times)
        for g0, gsz, jobs, empty in self._rs:
            send = self._rs_send[:, :gsz]
            if self._hip and jobs:
                from . import _lib
                from ._lib import DPZ_FOLD_ZERO_BASE
                key = (g0, send.data_ptr())
                a = self._rs_args.get(key)
                if a is None:
                    a = self._rs_args[key] = self._rs_batch_args(send, jobs)
                streams = (ctypes.c_void_p * len(self.streams))(
                    *[s.cuda_stream for s in self.streams])
                maxp = max(len(own) for _, _, own in jobs)
                dws = [w_.get_decode(N, maxp) for w_ in self.wss]
                cur = torch.cuda.current_stream(self.device)
                for st in self.streams:
                    st.wait_stream(cur)
                rc = _lib.lib().dpz_decode_average_batch(
                    a["m"], a["local"], a["out"], N, a["np"], a["idx"], a["val"], a["k"], a["w"],
                    None, DPZ_FOLD_ZERO_BASE, self._ptrs(dws), min(d.numel() for d in dws),
                    len(self.streams), streams)
                _lib.check(rc, "dpz_decode_average_batch")
                for st in self.streams:
                    cur.wait_stream(st)
            else:
                for r, j, own in jobs:
                    pays = [(self.send_idx[q], self.send_val[q]) for q, _ in own]
                    ones = [(self.send_idx[q], self._ones) for q, _ in own]
                    ws_ = [wq for _, wq in own]
                    self._partial(pays, ws_, send[r, j, 0])
                    self._partial(ones, ws_, send[r, j, 1])
            for r, j in empty:  # rows of destinations with no neighbour on this rank
                send[r, j].zero_()
            t_mark = self._leg_mark(t_mark, "rs_partial")
            if self.coll:
                # the slice [:, :gsz] of a (W, G, 2, N) buffer is contiguous only when gsz == G
                src = send if send.is_contiguous() else send.contiguous()
                recv = self._rs_recv[:gsz]
                dist.reduce_scatter_tensor(recv.view(-1), src.view(-1), group=self.group)
            else:
                recv = send[0]
            t_mark = self._leg_mark(t_mark, "rs_collective")
            for j in range(gsz):
                d = self.lo + g0 + j
                if d >= self.hi:
                    continue
                nbrs, w, w_self = self.weights[d - self.lo]
                c = w_self + sum(w)
                self._combine(self.x[d - self.lo], recv[j, 1], recv[j, 0], c,
                              self.out[d - self.lo])
            t_mark = self._leg_mark(t_mark, "rs_combine")
        self.x0, self.out = self.out, self.x0
        self.x.copy_(self.x0)

    def _leg_mark(self, t_prev, name=None):
        """With ``self.leg_times`` a dict: synchronize, add the time since t_prev to leg `name`
        and return the new mark (bench only; a no-op otherwise)."""
        if self.leg_times is None:
            return None
        import time
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        now = time.perf_counter()
        if name is not None and t_prev is not None:
            self.leg_times[name] = self.leg_times.get(name, 0.0) + (now - t_prev)
        return now

    def exchange(self):
        if self.exchange_mode == "reduce_scatter":
            return  # folded into fold_reduce_scatter
        if self.exchange_mode == "peer":
            if not self.coll or not (sum(self._peer_in_splits) or sum(self._peer_out_splits)):
                return  # no remote neighbour anywhere (one rank): the folds read in place
            import torch.distributed as dist
            ns = len(self._peer_rows)
            if ns:  # this rank's payloads that other ranks fold, packed (idx, val) per row
                self._peer_send[:ns, 0].copy_(self.send_idx.index_select(0, self._peer_rows_t))
                self._peer_send[:ns, 1].copy_(
                    self.send_val.index_select(0, self._peer_rows_t).view(torch.int32))
            dist.all_to_all_single(self._peer_recv.view(-1)[:sum(self._peer_out_splits)],
                                   self._peer_send.view(-1)[:sum(self._peer_in_splits)],
                                   output_split_sizes=self._peer_out_splits,
                                   input_split_sizes=self._peer_in_splits, group=self.group)
            return
        if not self.coll:
            self.recv_idx, self.recv_val = self.send_idx, self.send_val  # no copy on one rank
            return
        import torch.distributed as dist
        dist.all_gather_into_tensor(self.recv_idx, self.send_idx.contiguous(), group=self.group)
        dist.all_gather_into_tensor(self.recv_val, self.send_val, group=self.group)

    def _fold_tables(self):
        """Host tables of the batched fold (payload pointers, sizes, weights), built once: the
        receive buffers and the neighbourhoods do not change between rounds."""
        m = self.hi - self.lo
        counts, idx, val, kk, w, ws_ = [], [], [], [], [], []
        for j in range(m):
            nbrs, wj, w_self = self.weights[j]
            counts.append(len(nbrs))
            for q in nbrs:
                pi, pv = self._payload(q)
                idx.append(pi.data_ptr())
                val.append(pv.data_ptr())
                kk.append(self.k)
            w.extend(wj)
            ws_.append(w_self)
        tot = max(1, len(idx))
        return dict(np=(ctypes.c_int * max(1, m))(*counts), idx=(ctypes.c_void_p * tot)(*idx),
                    val=(ctypes.c_void_p * tot)(*val), k=(ctypes.c_int64 * tot)(*kk),
                    w=(ctypes.c_float * tot)(*w), w_self=(ctypes.c_float * max(1, m))(*ws_),
                    key=self._recv_key())

    def _fold_tab(self):
        """The fold tables of the current receive buffers, built once.  With the ring of rounds
        the payloads read in place are slot views: the table is built at one slot and its index
        pointers into the ring moved to the current slot (a numpy add, no rebuild)."""
        if not self.ring_counter:
            tab = getattr(self, "_tab", None)
            if tab is None or tab["key"] != self._recv_key():
                tab = self._tab = self._fold_tables()
            return tab
        import numpy as np
        off = self.send_idx.data_ptr() - self._ring.data_ptr()  # this slot's byte offset
        cur = self.send_idx.data_ptr()
        kn = tuple(v - off if v == cur else v for v in self._recv_key())  # slot-independent
        tab = getattr(self, "_tab", None)
        if tab is None or tab["key_ring"] != kn:
            tab = self._tab = self._fold_tables()
            idx0 = np.array([int(v or 0) for v in tab["idx"]], dtype=np.int64)
            lo, hi = self._ring.data_ptr(), self._ring.data_ptr() + self._ring.numel() * 4
            tab["ring_mask"] = ((idx0 >= lo) & (idx0 < hi)).astype(np.int64)
            tab["idx0"] = idx0 - tab["ring_mask"] * off
            tab["idx_now"] = np.empty_like(idx0)
            tab["idx"] = (ctypes.c_void_p * len(idx0)).from_buffer(tab["idx_now"])
            tab["key_ring"] = kn
        np.add(tab["idx0"], tab["ring_mask"] * off, out=tab["idx_now"])
        return tab

    def fold_all(self, guard=None):
        """Every owned node's Metro-Hastings fold.  guard (HIP, DEVICE int32): the round's
        encode status words; the one-launch fold then writes nothing if any is nonzero
        (dpz_decode_average_batch_guarded).  Returns False, with nothing enqueued, when the
        guarded launch does not apply to this round (the caller checks the encodes first)."""
        nodes = range(self.hi - self.lo)
        if guard is not None and not self._hip:  # the injected folds: the guard read on the host
            if bool(guard.any()):
                self.x0, self.out = self.out, self.x0
            else:
                self.fold_all()
            return True
        if guard is not None:
            from . import _lib
            from ._lib import DPZ_FOLD_ALSO_LOCAL, DPZ_FOLD_SELF
            m = self.hi - self.lo
            tab = self._fold_tab()
            ptrs = getattr(self, "_fold_ptrs", None)
            key = (self.x.data_ptr(), self.out.data_ptr())
            if ptrs is None or ptrs[0] != key:
                ptrs = self._fold_ptrs = (key, self._ptrs(self.x[:m]), self._ptrs(self.out[:m]))
            rc = _lib.lib().dpz_decode_average_batch_guarded(
                m, ptrs[1], ptrs[2], self.N, tab["np"], tab["idx"], tab["val"], tab["k"],
                tab["w"], tab["w_self"], DPZ_FOLD_SELF | DPZ_FOLD_ALSO_LOCAL, guard.data_ptr(),
                guard.numel(), ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream))
            if rc == _lib.DPZ_ERR_UNSUPPORTED:
                return False
            _lib.check(rc, "dpz_decode_average_batch_guarded")
            self.x0, self.out = self.out, self.x0
            return True
        if self._hip:
            from . import _lib
            from ._lib import DPZ_FOLD_ALSO_LOCAL, DPZ_FOLD_SELF
            tab = self._fold_tab()
            m = self.hi - self.lo
            streams = (ctypes.c_void_p * len(self.streams))(*[s.cuda_stream for s in self.streams])
            maxp = max((len(self.weights[j][0]) for j in nodes), default=1)
            dws = [w.get_decode(self.N, maxp) for w in self.wss]
            cur = torch.cuda.current_stream(self.device)
            for st in self.streams:
                st.wait_stream(cur)
            rc = _lib.lib().dpz_decode_average_batch(
                m, self._ptrs(self.x[:m]), self._ptrs(self.out[:m]), self.N, tab["np"],
                tab["idx"], tab["val"], tab["k"], tab["w"], tab["w_self"],
                DPZ_FOLD_SELF | DPZ_FOLD_ALSO_LOCAL,
                self._ptrs(dws), min(d.numel() for d in dws), len(self.streams), streams)
            _lib.check(rc, "dpz_decode_average_batch")
            for st in self.streams:
                cur.wait_stream(st)
        else:
            for j in nodes:
                nbrs, w, w_self = self.weights[j]
                payloads = [self._payload(q) for q in nbrs]
                self._fold(self.x[j], payloads, w, w_self, self.out[j])
        # post step: the averaged model becomes both the model and init_model (reference
        # Sharing._averaging load_state_dict + PartialModel._post_step): init_model takes the
        # fold output buffer (swap, no copy); the HIP fold also wrote the result over the model
        # in place (DPZ_FOLD_ALSO_LOCAL), the injected CPU fold gets one copy
        self.x0, self.out = self.out, self.x0
        if not self._hip:
            self.x.copy_(self.x0)

    def _slot(self, node):
        r = node // self.per
        return r * self.per + (node - r * self.per)

    def step(self):
        t = self._leg_mark(None)
        if self.exchange_mode in ("allgather", "peer") and self.guarded:
            return self._step_guarded(t)
        self.encode_all()
        t = self._leg_mark(t, "encode")
        if self.exchange_mode == "reduce_scatter":
            self.fold_reduce_scatter()
            return
        self.exchange()
        t = self._leg_mark(t, "exchange")
        self.fold_all()
        self._leg_mark(t, "fold")

    def _step_guarded(self, t):
        """A round with no host wait between the encodes and the folds: the encodes' status words
        (all-gathered with the payloads over the ranks) guard the one-launch folds on the device,
        and the host reads them back once the encodes (and the exchange) are done — while the
        folds run.  A miss (rare) left every fold unwritten: the missed nodes re-encode exactly,
        the payloads are exchanged again and the round's folds re-run (every rank sees the same
        gathered words, so all ranks take the same collectives)."""
        m = self.hi - self.lo
        self.encode_all(check=False)
        t = self._leg_mark(t, "encode")
        self.exchange()
        if self.coll:
            import torch.distributed as dist
            if getattr(self, "status_all", None) is None:
                self.status_all = torch.zeros(self.per * self.world, dtype=torch.int32,
                                              device=self.device)
            dist.all_gather_into_tensor(self.status_all, self.status[:self.per], group=self.group)
            words = self.status_all
        else:
            words = self.status[:m]
        cuda = self.device.type == "cuda"
        host = getattr(self, "_status_host", None)
        if host is None or host.numel() != words.numel():
            host = self._status_host = torch.zeros(words.numel(), dtype=torch.int32,
                                                   pin_memory=cuda)
        host.copy_(words, non_blocking=cuda)
        ev = None
        if cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
        t = self._leg_mark(t, "exchange")
        if not self.fold_all(guard=words):
            if ev is not None:
                ev.synchronize()
            bad = [j for j in range(m) if int(host[self._slot(self.lo + j)]) != 0]
            self._rerun_missed(bad)
            if self.coll and bool(host.any()):
                self.exchange()
            self.fold_all()
            self._leg_mark(t, "fold")
            return
        if ev is not None:
            ev.synchronize()  # the encodes and the exchange only: the folds keep running
        if bool(host.any()):
            if cuda:
                torch.cuda.synchronize(self.device)
            self.x0, self.out = self.out, self.x0  # the guarded folds wrote nothing
            self._rerun_missed([j for j in range(m) if int(host[self._slot(self.lo + j)]) != 0])
            self.exchange()
            self.fold_all()
        self._leg_mark(t, "fold")
