"""GPU: the share counter applied on read (dpz_counter_flush, RingCounter) and the lazily formed
model_change (LazyChange).

Reference: sharing/PartialModel.py:205-207 (``shared_parameters_counter[indices] += 1`` each
round; read once, at the end of the run, node/DPSGDNode.py:186-194) and :317-331
(``model.model_change``, read only by extract_top_gradients / save_change).  The counter must equal
the reference's whenever it is read — mid-run or at the end — and model_change must be the
reference's value whenever it is read."""
import numpy as np
import pytest
import torch

from oracle import topk as otopk
from tests import scenario

pytestmark = pytest.mark.gpu


def _lists(n, k, m, seed):
    rng = np.random.default_rng(seed)
    return [np.sort(rng.choice(n, size=k, replace=False)).astype(np.int32) for _ in range(m)]


@pytest.mark.parametrize("mode", ["scatter", "sweep", "auto"])
@pytest.mark.parametrize("m,offset", [(1, 0), (5, 0), (70, 0), (7, 1)])
def test_counter_flush_matches_numpy(dev, mode, m, offset):
    """Every mode adds one per entry of every segment; 70 segments take two sweep launches;
    offset 1: a counter view that is not 16-byte aligned (the sweep's element-wise tile path).
    The last tile is ragged (n not a multiple of the tile)."""
    from decentralizepy_amd import _lib, codec
    n, k = 1_000_003, 9_000
    lists = _lists(n, k, m, 11 + m)
    lists.append(np.array([0, 5, n - 1], dtype=np.int32))  # the edges of the counter
    lists.append(np.zeros(0, dtype=np.int32))               # an empty round (k = 0)
    ring = torch.from_numpy(np.concatenate(lists)).to(dev)
    seg = np.concatenate([[0], np.cumsum([len(a) for a in lists])]).tolist()
    base = np.random.default_rng(3).integers(0, 50, size=n + offset).astype(np.int32)
    store = torch.from_numpy(base).to(dev)
    counter = store[offset:]
    want = base[offset:].copy()
    for a in lists:
        np.add.at(want, a, 1)
    md = {"scatter": _lib.DPZ_COUNTER_SCATTER, "sweep": _lib.DPZ_COUNTER_SWEEP,
          "auto": _lib.DPZ_COUNTER_AUTO}[mode]
    codec.counter_flush(counter, ring, seg, mode=md)
    np.testing.assert_array_equal(counter.cpu().numpy(), want)
    if offset:
        assert store[0].item() == base[0]  # nothing before the view was written


def test_counter_flush_rejects_bad_segments(dev):
    from decentralizepy_amd import codec
    c = torch.zeros(100, dtype=torch.int32, device=dev)
    r = torch.zeros(10, dtype=torch.int32, device=dev)
    with pytest.raises(RuntimeError):
        codec.counter_flush(c, r, [1, 5])       # seg_off[0] != 0
    with pytest.raises(RuntimeError):
        codec.counter_flush(c, r, [0, 6, 4])    # descending offsets
    with pytest.raises(ValueError):
        codec.counter_flush(c, r, [0, 11])      # past the ring


@pytest.mark.parametrize("cap_rounds", [2, 64])
def test_ring_counter_reads_mid_run_and_at_the_end(dev, cap_rounds):
    """PartialModel's rounds with the counter in a ring (the encode writes the payload straight
    into a ring slot, no counter update): reading the counter mid-run and at the end gives the
    oracle's counter; a ring of two rounds fills and flushes by itself."""
    from decentralizepy_amd import codec
    from decentralizepy_amd._device import RingCounter
    n, k = 1_000_003, 10_000
    cnt = torch.zeros(n, dtype=torch.int32, device=dev)
    ring = RingCounter(cnt, cap_bytes=cap_rounds * 4 * k)
    o_cnt = np.zeros(n, dtype=np.int32)
    ws = codec.Workspace(dev)
    g = torch.Generator().manual_seed(21)
    x = torch.randn(n, generator=g)
    for r in range(6):
        x0 = x.clone()
        x = x0 + 0.01 * torch.randn(n, generator=g)
        slot = ring.slot(k)
        idx, val = codec.topk_encode(x.to(dev), k, x0=x0.to(dev), idx_out=slot, workspace=ws,
                                     hint=True)
        ring.commit(k)
        oi, _ = otopk.encode(x.numpy(), x0.numpy(), None, otopk.ACC_NONE, k, counter=o_cnt)
        np.testing.assert_array_equal(idx.cpu().numpy(), oi)
        if r == 2:  # a mid-run read (indexing, then the whole vector)
            sel = np.array([int(oi[0]), int(oi[-1]), 7])
            np.testing.assert_array_equal(ring[sel].numpy(), o_cnt[sel])
            np.testing.assert_array_equal(ring.numpy(), o_cnt)
            assert ring.pending_rounds() == 0
        assert ring.pending_rounds() <= cap_rounds
    assert ring.tolist() == o_cnt.tolist()  # the node's end-of-run dump


def test_plugin_counter_and_lazy_model_change(dev, tmp_path):
    """The PartialModel plugin over three rounds: model.model_change is formed only when read
    (never by the round itself) and is then T(x - init) bit for bit; the counter read mid-run and
    at the end equals the reference scenario's."""
    from decentralizepy_amd._device import LazyChange
    from collections import deque
    meta, arrays = scenario.load("pm_a01_plain")
    model = scenario.make_model(meta["shape"])
    scenario.set_flat(model, arrays["x0"])
    from decentralizepy_amd.sharing.PartialModel import PartialModel
    plugin = PartialModel(0, 0, None, scenario._Mapping(), scenario._Graph([1, 2, 3]), model,
                          None, str(tmp_path), **meta["kwargs"])
    init = arrays["x0"].copy()
    for r, mr in enumerate(meta["rounds"]):
        scenario.set_flat(model, arrays[f"r{r}_x"])
        plugin.get_data_to_send(degree=3)
        mc = model.model_change
        assert isinstance(mc, LazyChange) and not mc.materialized
        if r == 0:  # read it: the reference's T(x - init)
            want = arrays[f"r{r}_x"] - init
            np.testing.assert_array_equal(mc.cpu().numpy().view(np.uint32), want.view(np.uint32))
            np.testing.assert_array_equal(torch.abs(mc).cpu().numpy(), np.abs(want))
        np.testing.assert_array_equal(model.shared_parameters_counter.numpy(),
                                      arrays[f"r{r}_counter_after_encode"])
        peer = {uid: deque([m]) for uid, m in zip([1, 2, 3], scenario.neighbour_msgs(mr, arrays,
                                                                                      r))}
        plugin._averaging(peer)
        assert model.model_change is None
        init = scenario.get_flat(model)
