"""GPU tests of the native per-node step enqueue (dpz_encode_replace_batch) and the sticky status
word that makes an asynchronous encode's sampled-path miss visible (bench.py's timed region)."""
import numpy as np
import pytest
import torch

from oracle import fold as ofold
from oracle import topk as otopk

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def _node(dev, n, k, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, generator=g)
    x0 = x - 0.01 * torch.randn(n, generator=g)
    return dict(x=x.to(dev), x0=x0.to(dev), counter=torch.zeros(n, dtype=torch.int32, device=dev),
                idx=torch.empty(k, dtype=torch.int32, device=dev),
                val=torch.empty(k, dtype=torch.float32, device=dev),
                out=torch.empty(n, dtype=torch.float32, device=dev))


def _what(hint):
    from decentralizepy_amd._lib import DPZ_BATCH_DECODE, DPZ_BATCH_ENCODE, DPZ_BATCH_HINT
    return DPZ_BATCH_ENCODE | DPZ_BATCH_DECODE | (DPZ_BATCH_HINT if hint else 0)


@pytest.mark.parametrize("streams,hint", [(1, False), (2, False), (3, False), (1, True),
                                          (3, True)])
def test_node_step_batch_matches_oracle(dev, streams, hint):
    """hint: each encode takes its window from the previous encode on its stream's workspace
    (DPZ_BATCH_HINT), no sample launch after the first; same results."""
    from decentralizepy_amd import codec
    n, k, m = 1_000_003, 10_000, 5
    nodes = [_node(dev, n, k, 40 + j) for j in range(m)]
    ss = [torch.cuda.Stream(dev) for _ in range(streams)]
    ws = [codec.Workspace(dev) for _ in range(streams)]
    # every node decodes its own payload after its encode (not fused: the payload is the
    # encode's own output)
    b = codec.NodeStepBatch(nodes, n, k, ss, ws)
    b.sticky_status(clear=True)
    for _ in range(2):  # twice: counters accumulate, workspaces are reused
        b.run(_what(hint))
    torch.cuda.synchronize()
    assert b.sticky_status() == 0
    if hint:  # the last encode on every workspace ran without a sample launch (ctrl.hinted)
        assert all(int(w.buf[60:64].view(torch.int32).item()) == 1 for w in ws)
    for j, d in enumerate(nodes):
        x = d["x"].cpu().numpy()
        x0 = d["x0"].cpu().numpy()
        cnt = np.zeros(n, dtype=np.int32)
        oi, ov = otopk.encode(x, x0, None, 0, k, counter=cnt)
        otopk.encode(x, x0, None, 0, k, counter=cnt)
        np.testing.assert_array_equal(d["idx"].cpu().numpy(), oi)
        np.testing.assert_array_equal(_bits(d["val"].cpu().numpy()), _bits(ov))
        np.testing.assert_array_equal(d["counter"].cpu().numpy(), cnt)
        ref = ofold.replace(x, oi, ov)
        np.testing.assert_array_equal(_bits(d["out"].cpu().numpy()), _bits(ref))


@pytest.mark.parametrize("streams,hint", [(1, False), (3, False), (1, True), (3, True)])
def test_node_step_batch_neighbour_decode(dev, streams, hint):
    """Node j decoding node j - S's payload over its own x (S streams): the decode is fused
    into the encode (the filter writes the copy of x, select scatters the entries;
    dpz_encode_replace_batch) and still equals encode + replace."""
    from decentralizepy_amd import codec
    n, k, m = 1_000_003, 10_000, 2 * streams if streams > 1 else 4
    S = streams
    nodes = [_node(dev, n, k, 60 + j) for j in range(m)]
    b = codec.NodeStepBatch(nodes, n, k, [torch.cuda.Stream(dev) for _ in range(S)],
                            [codec.Workspace(dev) for _ in range(S)],
                            decode_src=lambda j: (j - S) % m)
    b.sticky_status(clear=True)
    for _ in range(2):  # node 0 reads node m-1's payload of the previous run
        b.run(_what(hint))
    torch.cuda.synchronize()
    assert b.sticky_status() == 0
    ref = []
    for d in nodes:
        oi, ov = otopk.encode(d["x"].cpu().numpy(), d["x0"].cpu().numpy(), None, 0, k)
        ref.append((oi, ov))
    for j, d in enumerate(nodes):
        oi, ov = ref[(j - S) % m]
        np.testing.assert_array_equal(_bits(d["out"].cpu().numpy()),
                                      _bits(ofold.replace(d["x"].cpu().numpy(), oi, ov)))
        np.testing.assert_array_equal(d["idx"].cpu().numpy(), ref[j][0])


def test_node_step_batch_encode_only_and_decode_only(dev):
    from decentralizepy_amd import codec
    from decentralizepy_amd._lib import DPZ_BATCH_DECODE, DPZ_BATCH_ENCODE
    n, k = 600_001, 6000
    nodes = [_node(dev, n, k, 7), _node(dev, n, k, 8)]
    s = [torch.cuda.Stream(dev)]
    b = codec.NodeStepBatch(nodes, n, k, s, [codec.Workspace(dev)])
    for d in nodes:
        d["out"].fill_(7.0)
    torch.cuda.synchronize()
    b.run(DPZ_BATCH_ENCODE)
    torch.cuda.synchronize()
    assert all(float(d["out"][0]) == 7.0 for d in nodes), "encode-only must not decode"
    b.run(DPZ_BATCH_DECODE, m=1)  # first node only
    torch.cuda.synchronize()
    assert float(nodes[1]["out"][0]) == 7.0
    x = nodes[0]["x"].cpu().numpy()
    x0 = nodes[0]["x0"].cpu().numpy()
    oi, ov = otopk.encode(x, x0, None, 0, k)
    np.testing.assert_array_equal(_bits(nodes[0]["out"].cpu().numpy()),
                                  _bits(ofold.replace(x, oi, ov)))


def test_sticky_status_records_an_uncompleted_miss(dev):
    """An ASYNC encode whose sampled window misses (tests/layouts.py, as in
    test_gpu_codec.test_topk_sampled_miss_falls_back) is never completed: the sticky word must
    say so, and a clear must reset it."""
    from decentralizepy_amd import codec
    n = 1 << 20
    k = round(0.01 * n)
    from tests.layouts import miss_layout
    x, _ = miss_layout(n, k)
    tx = torch.from_numpy(x).to(dev)
    tx0 = torch.zeros(n, device=dev)
    ws = codec.Workspace(dev)
    good = _node(dev, n, k, 3)
    codec.topk_encode(good["x"], k, x0=good["x0"], workspace=ws)  # a normal call first
    assert codec.topk_sticky_status(ws, clear=True) == 0
    codec.topk_encode(tx, k, x0=tx0, workspace=ws, asynchronous=True)
    codec.topk_encode(good["x"], k, x0=good["x0"], workspace=ws, asynchronous=True)
    assert codec.topk_sticky_status(ws) != 0, "the missed async encode must stay recorded"
    assert codec.topk_sticky_status(ws, clear=True) != 0
    assert codec.topk_sticky_status(ws) == 0


@pytest.mark.parametrize("streams", [1, 3])
def test_node_step_batch_ring_counters_match(dev, streams):
    """The bench's ring mode (RingCounter per node: encodes write their payload indices into ring
    slots and update no counter; flushed when full and by flush_rings) against the counter-in-the-
    compact batch over the same runs of the same states — neighbour decodes (decode_src = j - S)
    read the right slot across runs, a partial run (m < nodes) included, the ring wrapping
    (2-round rings): identical outputs, payload values and counters."""
    from decentralizepy_amd import codec
    from decentralizepy_amd._device import RingCounter
    n, k = 1_000_003, 10_000
    S = streams
    m = 2 * S if S > 1 else 4
    a_nodes = [_node(dev, n, k, 80 + j) for j in range(m)]
    for d in a_nodes:  # a valid payload before the first run (the first decodes read it)
        d["idx"].copy_(torch.arange(k, dtype=torch.int32, device=dev) * 7)
        d["val"].zero_()
    b_nodes = [{key: v.clone() for key, v in d.items()} for d in a_nodes]
    rings = [RingCounter(d["counter"], cap_bytes=2 * 4 * k) for d in b_nodes]
    mk = lambda nodes, rg: codec.NodeStepBatch(
        nodes, n, k, [torch.cuda.Stream(dev) for _ in range(S)],
        [codec.Workspace(dev) for _ in range(S)], decode_src=lambda j: (j - S) % m, rings=rg)
    a, b = mk(a_nodes, None), mk(b_nodes, rings)
    for r in range(5):
        mm = m if r != 2 else m - 1  # one partial run
        a.run(_what(True), m=mm)
        b.run(_what(True), m=mm)
        torch.cuda.synchronize()
        for da, db in zip(a_nodes, b_nodes):
            np.testing.assert_array_equal(_bits(da["out"].cpu().numpy()),
                                          _bits(db["out"].cpu().numpy()))
            np.testing.assert_array_equal(_bits(da["val"].cpu().numpy()),
                                          _bits(db["val"].cpu().numpy()))
    b.flush_rings()
    torch.cuda.synchronize()
    # no sampled-path miss (a missed asynchronous encode leaves its slot / buffer stale, which
    # the bench reports through the sticky status)
    assert a.sticky_status() == 0 and b.sticky_status() == 0
    for da, db in zip(a_nodes, b_nodes):
        np.testing.assert_array_equal(da["counter"].cpu().numpy(), db["counter"].cpu().numpy())
