"""One synchronous gossip round of a whole topology, nodes sharded over GPUs.

In the reference every node is its own process: ``Node`` calls ``sharing.get_data_to_send`` (top-k
encode, ``sharing/PartialModel.py:188-255``), sends the dict to each neighbour over ZeroMQ, then
``sharing._averaging`` folds the neighbours' payloads with Metro-Hastings weights
(``sharing/Sharing.py:156-190``, weight ``1 / (max(len(peer_deques), degree) + 1)``).  Simulating a
96-node round on one node of 8 MI355X, this engine keeps every node's flat model resident in HBM,
shards the nodes over the ranks (one process per GPU), and replaces the per-edge sends by ONE
all-gather of the fixed-size payloads (every node sends the same k): each rank encodes its own
nodes, ``all_gather_into_tensor`` over RCCL gives every rank every payload (96 x 8k bytes: 84 MB
at N = 11M), and each rank folds its own nodes' neighbourhoods locally.  No reduce-scatter: the
96 models fit one GPU's HBM.

The encode / fold callables are injectable so the sharding and exchange logic can be tested with
the CPU gloo backend; the defaults are the HIP codec (no CPU fallback).
"""
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
    """Metro-Hastings weights of node i's neighbours, in ascending neighbour order, and the self
    weight, rounded exactly like the reference (Python doubles, ``Sharing.py:165-185``)."""
    nbrs = sorted(adj[i])
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
                 device=None):
        """adj: adjacency sets of all nodes; x_init: (hi - lo, N) fp32 tensor with this rank's
        nodes' flat models (device tensor for the HIP codec)."""
        self.adj = adj
        self.n_nodes = len(adj)
        self.rank, self.world, self.group = rank, world, group
        self.lo, self.hi, self.per = shard(self.n_nodes, world, rank)
        assert x_init.shape[0] == self.hi - self.lo
        self.N = x_init.shape[1]
        self.k = round(alpha * self.N)
        self.device = device or x_init.device
        self.x = x_init.contiguous().clone()
        self.x0 = x_init.contiguous().clone()  # init_model of every owned node
        self.counter = torch.zeros_like(self.x, dtype=torch.int32)
        self.send_idx = torch.zeros(self.per, self.k, dtype=torch.int32, device=self.device)
        self.send_val = torch.zeros(self.per, self.k, dtype=torch.float32, device=self.device)
        self.recv_idx = torch.empty(self.per * world, self.k, dtype=torch.int32,
                                    device=self.device)
        self.recv_val = torch.empty(self.per * world, self.k, dtype=torch.float32,
                                    device=self.device)
        self.out = torch.empty_like(self.x)
        self.weights = [mh_weights(adj, i) for i in range(self.lo, self.hi)]
        if encode is None or fold is None:
            from . import codec
            self.ws = codec.Workspace(self.device)
        self._encode = encode or self._hip_encode
        self._fold = fold or self._hip_fold

    # ---- default device implementations ---------------------------------------------------
    def _hip_encode(self, x, x0, k, counter, idx_out, val_out):
        from . import codec
        codec.topk_encode(x, k, x0=x0, counter=counter, idx_out=idx_out, val_out=val_out,
                          workspace=self.ws, asynchronous=True)

    def _hip_fold(self, local, payloads, weights, w_self, out):
        from . import codec
        codec.decode_average(local, payloads, weights, w_self, out=out, workspace=self.ws)

    def _complete(self):
        """Finish the asynchronous encodes (a sampled-path miss re-runs exactly, rarely)."""
        if self._encode != self._hip_encode:
            return
        from . import codec
        for j in range(self.hi - self.lo):
            codec.topk_complete(self.x[j], self.k, self.send_idx[j], self.send_val[j], self.ws,
                                x0=self.x0[j], counter=self.counter[j])

    # ---- one round ----------------------------------------------------------------------------
    def encode_all(self):
        for j in range(self.hi - self.lo):
            self._encode(self.x[j], self.x0[j], self.k, self.counter[j], self.send_idx[j],
                         self.send_val[j])
        self._complete()

    def exchange(self):
        if self.world == 1:
            self.recv_idx[: self.per].copy_(self.send_idx)
            self.recv_val[: self.per].copy_(self.send_val)
            return
        import torch.distributed as dist
        dist.all_gather_into_tensor(self.recv_idx, self.send_idx, group=self.group)
        dist.all_gather_into_tensor(self.recv_val, self.send_val, group=self.group)

    def fold_all(self):
        for j in range(self.hi - self.lo):
            nbrs, w, w_self = self.weights[j]
            payloads = [(self.recv_idx[self._slot(q)], self.recv_val[self._slot(q)]) for q in nbrs]
            self._fold(self.x[j], payloads, w, w_self, self.out[j])
        # post step: the averaged model becomes both the model and init_model
        self.x.copy_(self.out)
        self.x0.copy_(self.out)

    def _slot(self, node):
        r = node // self.per
        return r * self.per + (node - r * self.per)

    def step(self):
        self.encode_all()
        self.exchange()
        self.fold_all()
