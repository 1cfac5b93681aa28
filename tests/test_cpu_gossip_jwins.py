"""CPU: the JWINS gossip-round engine (decentralizepy_amd/gossip_jwins.py, SURVEY.md §8d C3 shape
(b)) driven by the numpy oracle: equal to the reference semantics written out node by node
(tests/scenario.OracleNode, pinned by the reference's own JWINS / Wavelet fixtures), and the
world-2 gloo round (variable-size payloads all-gathered) equal to the one-rank round."""
import os

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests import scenario
from tests.jwins_ops import OracleJwinsOps, coeff_len, direct_round_nodes

EDGES16 = os.path.join(scenario.GOLDEN, "regular_16.edges")
TUTORIAL_ALPHAS = "[0.1,0.15,0.2,0.25,0.3,0.4,1.0]"  # tutorial/JWINS/config.ini


def _x(n_nodes, n, seed=3):
    return torch.randn(n_nodes, n, generator=torch.Generator().manual_seed(seed))


def _noise(r, i, n):
    g = torch.Generator().manual_seed(1000 * r + i)
    return (0.01 * torch.randn(n, generator=g)).numpy()


def _engine(adj, x, rank=0, world=1):
    from decentralizepy_amd.gossip_jwins import JwinsRound
    return JwinsRound(adj, x, TUTORIAL_ALPHAS, rank=rank, world=world, ops=OracleJwinsOps(),
                      device=torch.device("cpu"), m_len=coeff_len(x.shape[1]))


def _run(eng, rounds, n):
    drawn = []
    for r in range(rounds):
        for j in range(eng.hi - eng.lo):
            eng.x[j] += torch.from_numpy(_noise(r, eng.lo + j, n))
        eng.step()
        drawn += eng.alphas
    return drawn


def test_engine_equals_reference_semantics_node_by_node():
    from decentralizepy_amd.gossip import read_edges
    adj = read_edges(EDGES16)
    n, rounds = 3001, 3
    x = _x(16, n)
    eng = _engine(adj, x)
    drawn = _run(eng, rounds, n)
    assert any(a >= 0.5 for a in drawn) and any(a < 0.5 for a in drawn)  # both payload kinds
    nodes = direct_round_nodes(adj, x.numpy(), eval(TUTORIAL_ALPHAS), rounds,
                               lambda r, i: _noise(r, i, n))
    for i, nd in enumerate(nodes):
        np.testing.assert_array_equal(eng.x[i].numpy().view(np.uint32), nd.model.view(np.uint32))
        np.testing.assert_array_equal(eng.x0[i].numpy().view(np.uint32), nd.init.view(np.uint32))
        np.testing.assert_array_equal(eng.acc[i].numpy().view(np.uint32), nd.acc.view(np.uint32))
        np.testing.assert_array_equal(eng.counter[i].numpy(), nd.counter)


def test_alpha_draws_cover_full_and_partial_shares():
    """Over the rounds the tests run, the uid-seeded draws give both payload kinds."""
    import random
    alphas = eval(TUTORIAL_ALPHAS)
    draws = [random.Random(u).choice(alphas) for u in range(16)]
    rng = [random.Random(u) for u in range(16)]
    seen = [rng[u].choice(alphas) for _ in range(3) for u in range(16)]
    assert draws == seen[:16]
    assert any(a >= 0.5 for a in seen) and any(a < 0.5 for a in seen)


def _worker(rank, world, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from decentralizepy_amd.gossip import read_edges, shard
        adj = read_edges(EDGES16)
        x = _x(16, n)
        lo, hi, _ = shard(16, world, rank)
        eng = _engine(adj, x[lo:hi], rank=rank, world=world)
        _run(eng, 3, n)
        q.put((rank, lo, eng.x.numpy().copy(), eng.acc.numpy().copy()))
    except Exception as e:  # noqa: BLE001 - reported to the parent instead of a queue timeout
        q.put((rank, None, repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


def test_two_rank_round_equals_single_rank():
    from decentralizepy_amd.gossip import read_edges
    adj = read_edges(EDGES16)
    n = 2003
    x = _x(16, n)
    single = _engine(adj, x)
    _run(single, 3, n)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29900 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, lo, xs, acc in got:
        assert lo is not None, xs
        np.testing.assert_array_equal(xs.view(np.uint32),
                                      single.x.numpy()[lo:lo + xs.shape[0]].view(np.uint32))
        np.testing.assert_array_equal(acc.view(np.uint32),
                                      single.acc.numpy()[lo:lo + xs.shape[0]].view(np.uint32))
