"""CPU (gloo, world_size 2): the gossip-round engine's node sharding, payload all-gather and
Metro-Hastings neighbourhoods, with the oracle standing in for the HIP codec (the device path is
covered by tests/test_gpu_gossip.py).  Topologies are the reference's own data files
(eval/96_regular.edges, tutorial/JWINS/regular_16.txt) copied under tests/golden/."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import fold as ofold
from oracle import topk as otopk
from tests import scenario

EDGES96 = os.path.join(scenario.GOLDEN, "96_regular.edges")
EDGES16 = os.path.join(scenario.GOLDEN, "regular_16.edges")


def _oracle_encode(x, x0, k, counter, idx_out, val_out):
    c = counter.numpy()
    idx, val = otopk.encode(x.numpy(), x0.numpy(), None, otopk.ACC_NONE, k, counter=c)
    idx_out.copy_(torch.from_numpy(idx))
    val_out.copy_(torch.from_numpy(val))


def _oracle_fold(local, payloads, weights, w_self, out):
    pays = [(i.numpy(), v.numpy()) for i, v in payloads]
    out.copy_(torch.from_numpy(ofold.fold(local.numpy(), pays, weights, w_self)))


def _models(n_nodes, n, seed=5):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n_nodes, n, generator=g)


def _train(eng, r):
    g = torch.Generator().manual_seed(100 + r)
    noise = 0.01 * torch.randn(eng.n_nodes, eng.N, generator=g)
    eng.x += noise[eng.lo:eng.hi]


def _direct_round(adj, x, x0, k):
    """The reference semantics written out node by node (no sharding, no all-gather)."""
    from decentralizepy_amd.gossip import mh_weights
    pays = [otopk.encode(x[i], x0[i], None, otopk.ACC_NONE, k) for i in range(len(adj))]
    out = np.empty_like(x)
    for i in range(len(adj)):
        nbrs, w, w_self = mh_weights(adj, i)
        out[i] = ofold.fold(x[i], [pays[j] for j in nbrs], w, w_self)
    return out


def test_read_edges_and_weights():
    from decentralizepy_amd.gossip import mh_weights, read_edges, shard
    adj = read_edges(EDGES96)
    assert len(adj) == 96
    assert sum(len(a) for a in adj) == 380          # sum of degrees
    assert {len(a) for a in adj} <= {3, 4}
    nbrs, w, w_self = mh_weights(adj, 0)
    assert nbrs == list(adj[0]) and abs(sum(w) + w_self - 1) < 1e-12
    # the reference folds in neighbour-SET iteration order, which differs from ascending order
    # for most nodes of this topology (e.g. a neighbour set {5, 9, 12} iterates 9, 12, 5)
    assert sum(1 for i in range(96) if mh_weights(adj, i)[0] != sorted(adj[i])) > 48
    adj16 = read_edges(EDGES16)
    assert len(adj16) == 16 and {len(a) for a in adj16} == {3}
    lo, hi, per = shard(96, 8, 7)
    assert (lo, hi, per) == (84, 96, 12)
    assert shard(10, 4, 3) == (9, 10, 3)


def test_single_rank_round_matches_direct_simulation():
    from decentralizepy_amd.gossip import GossipRound, read_edges
    adj = read_edges(EDGES16)
    n = 2000
    x = _models(16, n)
    eng = GossipRound(adj, x, 0.05, encode=_oracle_encode, fold=_oracle_fold)
    ref_x, ref_x0 = x.numpy().copy(), x.numpy().copy()
    for r in range(2):
        _train(eng, r)
        g = torch.Generator().manual_seed(100 + r)
        ref_x = ref_x + (0.01 * torch.randn(16, n, generator=g)).numpy()
        eng.step()
        ref_x = _direct_round(adj, ref_x, ref_x0, eng.k)
        ref_x0 = ref_x.copy()
        np.testing.assert_array_equal(eng.x.numpy().view(np.uint32), ref_x.view(np.uint32))


def _worker(rank, world, port, n, path, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from decentralizepy_amd.gossip import GossipRound, read_edges, shard
        adj = read_edges(path)
        x = _models(len(adj), n)
        lo, hi, _ = shard(len(adj), world, rank)
        eng = GossipRound(adj, x[lo:hi], 0.05, rank=rank, world=world, encode=_oracle_encode,
                          fold=_oracle_fold)
        for r in range(2):
            _train(eng, r)
            eng.step()
        q.put((rank, lo, eng.x.numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("path,n", [(EDGES16, 1500), (EDGES96, 600)])
def test_two_rank_round_equals_single_rank(path, n):
    from decentralizepy_amd.gossip import GossipRound, read_edges
    adj = read_edges(path)
    x = _models(len(adj), n)
    single = GossipRound(adj, x, 0.05, encode=_oracle_encode, fold=_oracle_fold)
    for r in range(2):
        _train(single, r)
        single.step()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, path, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, lo, xs in got:
        np.testing.assert_array_equal(xs.view(np.uint32),
                                      single.x.numpy()[lo:lo + xs.shape[0]].view(np.uint32))


def _torch_partial(payloads, weights, out):
    out.zero_()
    for (idx, val), w in zip(payloads, weights):
        out.index_add_(0, idx.long(), val * torch.tensor(w, dtype=torch.float32))


def _torch_combine(x, b, a, c, out):
    out.copy_(x * (torch.tensor(c, dtype=torch.float32) - b) + a)


def _rs_worker(rank, world, port, n, path, q, skew=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from decentralizepy_amd.gossip import GossipRound, read_edges, shard
        adj = read_edges(path)
        x = _models(len(adj), n)
        lo, hi, per = shard(len(adj), world, rank)
        k = round(0.05 * n)
        # an emulated budget one byte below ONE payload: neither the all-gathered payloads nor
        # the peer exchange's fit, auto picks the reduce-scatter, one destination node per group
        budget = k * 8 - 1
        if skew:  # rank 1 alone would fit the all-gather: the ranks must still agree (MIN)
            budget += rank * 10 ** 12
        eng = GossipRound(adj, x[lo:hi], 0.05, rank=rank, world=world, encode=_oracle_encode,
                          fold=_oracle_fold, hbm_budget=budget, partial=_torch_partial,
                          combine=_torch_combine)
        assert eng.exchange_mode == "reduce_scatter" and eng.recv_idx is None
        assert eng.rs_group == 1
        for r in range(2):
            _train(eng, r)
            eng.step()
        q.put((rank, lo, eng.x.numpy().copy()))
    except Exception as e:  # noqa: BLE001 - reported to the parent instead of a queue timeout
        q.put((rank, None, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("path,n,skew", [(EDGES16, 1500, False), (EDGES96, 600, False),
                                         (EDGES16, 1500, True)])
def test_reduce_scatter_round_matches_within_tolerance(path, n, skew):
    """The over-HBM exchange (payloads never replicated; dense (A, B) contributions
    reduce-scattered to the owning rank) reproduces the bit-exact all-gather round within fp32
    reassociation tolerance, over two rounds (BASELINE.json C4)."""
    from decentralizepy_amd.gossip import GossipRound, read_edges
    adj = read_edges(path)
    x = _models(len(adj), n)
    single = GossipRound(adj, x, 0.05, encode=_oracle_encode, fold=_oracle_fold)
    assert single.exchange_mode == "allgather"
    for r in range(2):
        _train(single, r)
        single.step()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + (os.getpid() % 1000) + (7 if skew else 0)
    procs = [ctx.Process(target=_rs_worker, args=(r, 2, port, n, path, q, skew))
             for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, lo, xs in got:
        assert lo is not None, xs
        ref = single.x.numpy()[lo:lo + xs.shape[0]]
        np.testing.assert_allclose(xs, ref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("miss_round", [0, 1])
def test_guarded_round_reruns_a_missed_encode(miss_round):
    """The guarded round (encodes, exchange and folds with no host check in between; the encodes'
    status words guard the folds): a node whose encode reports a miss — its payload poisoned —
    leaves every fold of the round unwritten, is re-encoded, and the round's folds re-run, so the
    models and counters equal the host-checked engine's (guarded=False) round for round."""
    from decentralizepy_amd.gossip import GossipRound, read_edges
    adj = read_edges(EDGES16)
    n = 1500
    x = _models(16, n)
    a = GossipRound(adj, x, 0.05, encode=_oracle_encode, fold=_oracle_fold, guarded=True)
    b = GossipRound(adj, x, 0.05, encode=_oracle_encode, fold=_oracle_fold, guarded=False)
    orig = a.encode_all
    state = {"r": 0, "reruns": 0}

    def encode_all(check=True):
        c5 = a.counter[5].clone()
        orig(check)
        if state["r"] == miss_round:  # node 5 "missed": no counter update, a garbage payload
            a.counter[5] = c5
            a.send_val[5].fill_(float("nan"))
            a.status[5] = 1

    def rerun(bad, _orig=a._rerun_missed):
        state["reruns"] += len(bad)
        _orig(bad)  # the engine's own re-run clears the missed nodes' status words
        assert not bool(a.status.any())

    a.encode_all = encode_all
    a._rerun_missed = rerun
    for r in range(2):
        state["r"] = r
        for eng in (a, b):
            _train(eng, r)
            eng.step()
        np.testing.assert_array_equal(a.x.numpy().view(np.uint32), b.x.numpy().view(np.uint32))
        np.testing.assert_array_equal(a.x0.numpy().view(np.uint32), b.x0.numpy().view(np.uint32))
        np.testing.assert_array_equal(a.counter.numpy(), b.counter.numpy())
    assert state["reruns"] == 1


def _peer_worker(rank, world, port, n, path, q, budget):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from decentralizepy_amd.gossip import GossipRound, read_edges, shard
        adj = read_edges(path)
        x = _models(len(adj), n)
        lo, hi, _ = shard(len(adj), world, rank)
        kw = dict(exchange="peer") if budget is None else dict(hbm_budget=budget)
        eng = GossipRound(adj, x[lo:hi], 0.05, rank=rank, world=world, encode=_oracle_encode,
                          fold=_oracle_fold, **kw)
        assert eng.exchange_mode == "peer" and eng.recv_idx is None
        for r in range(2):
            _train(eng, r)
            eng.step()
        q.put((rank, lo, eng.x.numpy().copy(), eng._peer_n_recv))
    except Exception as e:  # noqa: BLE001 - reported to the parent instead of a queue timeout
        q.put((rank, None, repr(e), 0))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("path,n,world,auto", [(EDGES16, 1500, 2, False), (EDGES96, 600, 2, False),
                                                (EDGES96, 600, 3, True)])
def test_peer_exchange_round_equals_single_rank(path, n, world, auto):
    """The peer exchange (each rank sends other ranks only the payloads their nodes' neighbours
    name, one all_to_all_single with uneven splits) is bit-exact with the single-rank round;
    "auto" takes it when the all-gathered payloads exceed the budget and its own fit; a rank
    holds fewer remote payloads than the all-gather would give it."""
    from decentralizepy_amd.gossip import GossipRound, read_edges, shard
    adj = read_edges(path)
    x = _models(len(adj), n)
    single = GossipRound(adj, x, 0.05, encode=_oracle_encode, fold=_oracle_fold)
    for r in range(2):
        _train(single, r)
        single.step()
    _, _, per = shard(len(adj), world, 0)
    k = round(0.05 * n)
    budget = per * world * k * 8 - 1 if auto else None  # one byte short of the all-gather
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29300 + (os.getpid() % 1000) + 11 * world + (5 if auto else 0)
    procs = [ctx.Process(target=_peer_worker, args=(r, world, port, n, path, q, budget))
             for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, lo, xs, n_recv in got:
        assert lo is not None, xs
        assert n_recv <= per * (world - 1)
        np.testing.assert_array_equal(xs.view(np.uint32),
                                      single.x.numpy()[lo:lo + xs.shape[0]].view(np.uint32))


def test_peer_plan_counts():
    """The peer plan of 96_regular.edges over 8 ranks: every rank's receive rows are exactly the
    remote neighbours of its nodes, and the send and receive splits of all ranks agree."""
    from decentralizepy_amd.gossip import GossipRound, read_edges, shard

    class _Plan(GossipRound):
        def __init__(self, adj, rank, world, k):  # the plan alone (no engine state)
            self.adj, self.n_nodes, self.world, self.rank, self.k = adj, len(adj), world, rank, k
            self.lo, self.hi, self.per = shard(self.n_nodes, world, rank)
            self._peer_plan()

    adj = read_edges(EDGES96)
    plans = [_Plan(adj, r, 8, 10) for r in range(8)]
    for r, p in enumerate(plans):
        want = {q for d in range(p.lo, p.hi) for q in adj[d] if not p.lo <= q < p.hi}
        assert set(p._peer_row) == want
        assert p._peer_n_recv < 84  # the all-gather gives every rank 84 remote payloads
        for s, ps in enumerate(plans):
            assert p._peer_out_splits[s] == ps._peer_in_splits[r]
