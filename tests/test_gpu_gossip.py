"""GPU: one- and multi-round gossip over the reference topologies with the HIP codec, bit-exact
against the same engine driven by the oracle on the CPU."""
import numpy as np
import pytest
import torch

from tests.test_cpu_gossip import EDGES16, EDGES96, _models, _oracle_encode, _oracle_fold, _train

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("path,n,alpha", [(EDGES16, 300_000, 0.01), (EDGES96, 40_000, 0.02)])
def test_gossip_round_device_matches_oracle(dev, path, n, alpha):
    from decentralizepy_amd.gossip import GossipRound, read_edges
    adj = read_edges(path)
    x = _models(len(adj), n)
    ref = GossipRound(adj, x, alpha, encode=_oracle_encode, fold=_oracle_fold)
    eng = GossipRound(adj, x.to(dev), alpha)
    for r in range(2):
        _train(ref, r)
        g = torch.Generator().manual_seed(100 + r)
        eng.x += (0.01 * torch.randn(len(adj), n, generator=g)).to(dev)
        ref.step()
        eng.step()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(eng.x.cpu().numpy().view(np.uint32),
                                      ref.x.numpy().view(np.uint32))
        np.testing.assert_array_equal(eng.counter.cpu().numpy(), ref.counter.numpy())


@pytest.mark.parametrize("path,n,alpha", [(EDGES16, 300_000, 0.01), (EDGES96, 40_000, 0.02)])
def test_peer_exchange_device_matches_oracle(dev, path, n, alpha):
    """The peer exchange's device fold tables (local neighbours' payloads read in place from the
    send rows, the guarded one-launch fold) on one rank, bit-exact with the oracle round (the
    multi-rank all_to_all_single is covered with gloo, tests/test_cpu_gossip.py)."""
    from decentralizepy_amd.gossip import GossipRound, read_edges
    adj = read_edges(path)
    x = _models(len(adj), n)
    ref = GossipRound(adj, x, alpha, encode=_oracle_encode, fold=_oracle_fold)
    eng = GossipRound(adj, x.to(dev), alpha, exchange="peer")
    assert eng.exchange_mode == "peer" and eng._peer_n_recv == 0
    for r in range(2):
        _train(ref, r)
        g = torch.Generator().manual_seed(100 + r)
        eng.x += (0.01 * torch.randn(len(adj), n, generator=g)).to(dev)
        ref.step()
        eng.step()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(eng.x.cpu().numpy().view(np.uint32),
                                      ref.x.numpy().view(np.uint32))
        np.testing.assert_array_equal(eng.counter.cpu().numpy(), ref.counter.numpy())


@pytest.mark.parametrize("path,n,alpha,budget", [(EDGES16, 200_003, 0.01, 1),
                                                  (EDGES96, 30_000, 0.05, 1),
                                                  (EDGES96, 30_000, 0.05, None)])
def test_reduce_scatter_exchange_device_within_tolerance(dev, path, n, alpha, budget):
    """The over-HBM exchange's device legs — the zero-based batched fold of the owned payloads
    into dense (A, B) rows and the DPZ_EW_MHCOMBINE owner combine — on one rank (forced mode,
    budget of one destination node per group), against the bit-exact all-gather round within
    fp32 reassociation tolerance."""
    from decentralizepy_amd.gossip import GossipRound, read_edges
    adj = read_edges(path)
    x = _models(len(adj), n)
    exact = GossipRound(adj, x.to(dev), alpha)
    rs = GossipRound(adj, x.to(dev), alpha, exchange="reduce_scatter", hbm_budget=budget)
    # budget 1: one destination node per group; None: the whole rank in one batched group
    assert rs.exchange_mode == "reduce_scatter" and rs.rs_group == (1 if budget else len(adj))
    for r in range(2):
        g = torch.Generator().manual_seed(100 + r)
        noise = (0.01 * torch.randn(len(adj), n, generator=g)).to(dev)
        exact.x += noise
        rs.x += noise
        exact.step()
        rs.step()
        torch.cuda.synchronize()
        np.testing.assert_allclose(rs.x.cpu().numpy(), exact.x.cpu().numpy(), rtol=1e-5,
                                   atol=1e-6)
        np.testing.assert_array_equal(rs.counter.cpu().numpy(), exact.counter.cpu().numpy())


@pytest.mark.parametrize("wavelet", ["sym2", "haar", "db4"])
def test_jwins_round_device_matches_oracle(dev, wavelet):
    """C3 shape (b): the JWINS round of tutorial/JWINS/regular_16.txt with the tutorial alpha
    list (uid-seeded draws, full shares included) — DWT pair, ADD-accumulation top-k, batched
    coefficient-domain fold, IDWT, accumulating post-step — bit-exact against the same engine
    driven by the oracle, over 2 rounds.  M >= 2^18 keeps the encodes on the sampled path."""
    from decentralizepy_amd.gossip import read_edges
    from decentralizepy_amd.gossip_jwins import JwinsRound
    from tests.jwins_ops import OracleJwinsOps, coeff_len
    from tests.test_cpu_gossip_jwins import EDGES16, TUTORIAL_ALPHAS, _noise
    adj = read_edges(EDGES16)
    n = 300_001
    x = torch.randn(16, n, generator=torch.Generator().manual_seed(11))
    ref = JwinsRound(adj, x, TUTORIAL_ALPHAS, wavelet=wavelet, ops=OracleJwinsOps(wavelet),
                     device=torch.device("cpu"), m_len=coeff_len(n, 4, wavelet))
    eng = JwinsRound(adj, x.to(dev), TUTORIAL_ALPHAS, wavelet=wavelet)
    assert eng.M == ref.M
    kinds = set()
    for r in range(2):
        for j in range(16):
            nz = torch.from_numpy(_noise(r, j, n))
            ref.x[j] += nz
            eng.x[j] += nz.to(dev)
        ref.step()
        eng.step()
        kinds |= {a >= 0.5 for a in eng.alphas}
        torch.cuda.synchronize()
        for name in ("x", "x0", "acc"):
            np.testing.assert_array_equal(getattr(eng, name).cpu().numpy().view(np.uint32),
                                          getattr(ref, name).numpy().view(np.uint32), err_msg=name)
        np.testing.assert_array_equal(eng.counter.cpu().numpy(), ref.counter.numpy())
    assert kinds == {True, False}


def test_node_batched_encodes_equal_stream_encodes(dev):
    """The round's encodes as one launch per phase over all nodes (dpz_topk_encode_nodes, each
    node its own workspace, the prior window from the second round on) against node-after-node
    encodes on three streams: bit-identical models and counters over three rounds — one node's
    change hides its large entries between the sample chunks (tests/layouts.py) in round 0 and
    jumps x4 in scale in round 2, so its encodes miss and are re-run exactly."""
    from decentralizepy_amd.gossip import GossipRound, read_edges
    from tests.layouts import miss_layout
    adj = read_edges(EDGES16)
    n = 1 << 20
    x = _models(len(adj), n)
    a = GossipRound(adj, x.to(dev), 0.01, node_batch=True)
    b = GossipRound(adj, x.to(dev), 0.01, node_batch=False)
    # the host-checked round (a status check between encodes and folds) beside the guarded ones:
    # a missed encode leaves the guarded folds unwritten and the round re-runs them
    c = GossipRound(adj, x.to(dev), 0.01, node_batch=True, guarded=False)
    miss, _ = miss_layout(n, round(0.01 * n))
    reruns = []
    orig = a._rerun_missed

    def rerun(bad):
        reruns.append(list(bad))
        orig(bad)
        assert not bool(a.status.any())  # the re-run's payloads are final: words cleared

    a._rerun_missed = rerun
    for r in range(3):
        g = torch.Generator().manual_seed(300 + r)
        noise = (0.01 * torch.randn(len(adj), n, generator=g)).to(dev)
        if r == 2:
            noise[5] *= 4.0
        for eng in (a, b, c):
            eng.x += noise
            if r == 0:
                eng.x[3] = eng.x0[3] + torch.from_numpy(miss).to(dev)
            eng.step()
        torch.cuda.synchronize()
        if r == 0:
            assert any(3 in bad for bad in reruns)  # the round's encodes did miss (node 3)
        for o in (b, c):
            np.testing.assert_array_equal(a.x.cpu().numpy().view(np.uint32),
                                          o.x.cpu().numpy().view(np.uint32))
            np.testing.assert_array_equal(a.x0.cpu().numpy().view(np.uint32),
                                          o.x0.cpu().numpy().view(np.uint32))
            np.testing.assert_array_equal(a.counter.cpu().numpy(), o.counter.cpu().numpy())
    assert a.node_ws is not None and getattr(b, "node_ws", None) is None


@pytest.mark.parametrize("path,n,alpha", [(EDGES16, 1 << 20, 0.01), (EDGES96, 40_000, 0.02)])
def test_gossip_round_sliced_counter(dev, path, n, alpha):
    """Every node's shared_parameters_counter in bit-sliced form (DPZ_TOPK_SLICED node-batched
    encodes: compact writes the selection mask and ripple-adds it to the planes): models and the
    materialised counters bit-identical to the int32-counter engine over three rounds, a forced
    sampled miss in round 0 included (re-run exactly through dpz_topk_encode_sliced)."""
    from decentralizepy_amd.gossip import GossipRound, read_edges
    from tests.layouts import miss_layout
    adj = read_edges(path)
    x = _models(len(adj), n)
    a = GossipRound(adj, x.to(dev), alpha, sliced_counter=True, ring_counter=False)
    b = GossipRound(adj, x.to(dev), alpha, sliced_counter=False, ring_counter=False)
    assert a.sliced_counter and not b.sliced_counter
    miss = None
    if n >= (1 << 20):
        miss, _ = miss_layout(n, round(alpha * n))
    for r in range(3):
        g = torch.Generator().manual_seed(500 + r)
        noise = (0.01 * torch.randn(len(adj), n, generator=g)).to(dev)
        for eng in (a, b):
            eng.x += noise
            if r == 0 and miss is not None:
                eng.x[3] = eng.x0[3] + torch.from_numpy(miss).to(dev)
            eng.step()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(a.x.cpu().numpy().view(np.uint32),
                                      b.x.cpu().numpy().view(np.uint32))
        np.testing.assert_array_equal(a.counter.cpu().numpy(), b.counter.cpu().numpy())


def test_sliced_counter_falls_back_past_the_sliced_geometry(dev):
    """n = 2^26 + 64: a wave segment exceeds the sliced compact's LDS row (SL_RMAX), so the first
    node-batched sliced encode returns UNSUPPORTED before any launch and the engine continues on
    the int32 counter (GossipRound._unslice) — results bit-identical to an int32 engine; one node
    per rank never takes the sliced form."""
    from decentralizepy_amd.gossip import GossipRound
    n = (1 << 26) + 64
    adj = [{1}, {0}]
    g = torch.Generator().manual_seed(7)
    x = torch.randn(2, n, generator=g).to(dev)
    a = GossipRound(adj, x, 0.01, ring_counter=False)
    b = GossipRound(adj, x, 0.01, sliced_counter=False, ring_counter=False)
    assert a.sliced_counter
    for r in range(2):
        noise = torch.randn(2, n, generator=torch.Generator(device=dev).manual_seed(r), device=dev)
        for eng in (a, b):
            eng.x += 0.01 * noise
            eng.step()
        torch.cuda.synchronize()
        assert not a.sliced_counter
        assert torch.equal(a.x.view(torch.int32), b.x.view(torch.int32))
        assert torch.equal(a.counter, b.counter)
    del a, b
    one = GossipRound([set()], torch.zeros(1, 1 << 18, device=dev), 0.01)
    assert not one.sliced_counter and not one.ring_counter


@pytest.mark.parametrize("path,n,alpha,slots,exchange", [(EDGES16, 1 << 20, 0.01, 2, "auto"),
                                                         (EDGES96, 40_000, 0.02, 3, "auto"),
                                                         (EDGES96, 40_000, 0.02, 3, "peer")])
def test_gossip_round_ring_counter(dev, path, n, alpha, slots, exchange):
    """The counters deferred to a ring of rounds (the node-batched encodes write each round's
    payload indices into a ring slot and update no counter; dpz_counter_flush on read or when the
    ring is full): models and counters bit-identical to the int32-counter engine over five rounds
    with a 2- / 3-slot ring (wraps: flushes inside the run), the counter read mid-run and at the
    end, a forced sampled miss in round 0 (re-run exactly into the slot), and the counter a live
    tensor (a write into it stays)."""
    from decentralizepy_amd.gossip import GossipRound, read_edges
    from tests.layouts import miss_layout
    adj = read_edges(path)
    x = _models(len(adj), n)
    a = GossipRound(adj, x.to(dev), alpha, ring_slots=slots, exchange=exchange)
    b = GossipRound(adj, x.to(dev), alpha, sliced_counter=False, ring_counter=False)
    assert a.ring_counter and not a.sliced_counter and a.ring_slots == slots
    miss = None
    if n >= (1 << 20):
        miss, _ = miss_layout(n, round(alpha * n))
    for r in range(5):
        g = torch.Generator().manual_seed(700 + r)
        noise = (0.01 * torch.randn(len(adj), n, generator=g)).to(dev)
        for eng in (a, b):
            eng.x += noise
            if r == 0 and miss is not None:
                eng.x[3] = eng.x0[3] + torch.from_numpy(miss).to(dev)
            eng.step()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(a.x.cpu().numpy().view(np.uint32),
                                      b.x.cpu().numpy().view(np.uint32))
        if r in (1, 4):
            np.testing.assert_array_equal(a.counter.cpu().numpy(), b.counter.cpu().numpy())
            np.testing.assert_array_equal(a.counter_row(2).cpu().numpy(),
                                          b.counter[2].cpu().numpy())
    a.counter[0, 0] += 5
    assert int(a.counter[0, 0]) == int(b.counter[0, 0]) + 5


def test_reduce_scatter_mode_keeps_int32_counters(dev):
    """The over-HBM legs cache their payload pointers, so the reduce-scatter mode never takes
    the ring of rounds; three rounds with no counter read in between stay within tolerance of the
    all-gather engine and the counters equal."""
    from decentralizepy_amd.gossip import GossipRound, read_edges
    adj = read_edges(EDGES96)
    x = _models(len(adj), 30_000)
    exact = GossipRound(adj, x.to(dev), 0.05)
    rs = GossipRound(adj, x.to(dev), 0.05, exchange="reduce_scatter", hbm_budget=1)
    assert exact.ring_counter and not rs.ring_counter
    for r in range(3):
        g = torch.Generator().manual_seed(300 + r)
        noise = (0.01 * torch.randn(len(adj), 30_000, generator=g)).to(dev)
        exact.x += noise
        rs.x += noise
        exact.step()
        rs.step()
    torch.cuda.synchronize()
    np.testing.assert_allclose(rs.x.cpu().numpy(), exact.x.cpu().numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(rs.counter.cpu().numpy(), exact.counter.cpu().numpy())
