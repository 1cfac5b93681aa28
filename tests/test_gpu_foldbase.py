"""GPU parity of the fused fold base (dpz_topk_encode_foldbase) and the hit-only patch decode
(DPZ_FOLD_BASE_READY): the encode's results are unchanged, the base is the fold of x alone, and
the patched output is bit-identical to the oracle's Metro-Hastings fold of the payloads over x
(reference sharing/Sharing.py:156-190 with PartialModel payloads, PartialModel.py:257-303)."""
import numpy as np
import pytest
import torch

from decentralizepy_amd import codec
from oracle import fold as ofold
from oracle import topk as otopk

pytestmark = pytest.mark.gpu


def _payloads(rng, n, ks, overlap=0.0, cluster=None):
    """sorted unique int32 index sets (payload p shares ~overlap of payload 0's indices)"""
    out = []
    base = None
    for j, k in enumerate(ks):
        if k == 0:
            out.append((np.zeros(0, np.int32), np.zeros(0, np.float32)))
            continue
        if cluster is not None:
            lo = cluster[j % len(cluster)]
            idx = np.arange(lo, lo + k, dtype=np.int64)
        else:
            idx = rng.choice(n, size=k, replace=False)
            if base is not None and overlap > 0:
                m = min(int(overlap * k), len(base))
                idx = np.unique(np.concatenate([base[:m], idx]))[:k]
                if len(idx) < k:
                    extra = rng.choice(n, size=2 * k, replace=False)
                    idx = np.unique(np.concatenate([idx, extra]))[:k]
            base = idx if base is None else base
        idx = np.sort(idx).astype(np.int32)
        out.append((idx, rng.standard_normal(len(idx)).astype(np.float32)))
    return out


def _bits(a):
    return np.asarray(a, dtype=np.float32).view(np.uint32)


@pytest.mark.parametrize("n,alpha,ks,weights,overlap,cluster", [
    (300_007, 0.01, [3000], [0.5], 0.0, None),
    (1_000_003, 0.01, [10_000, 10_000, 10_000], None, 0.3, None),
    (11_000_000, 0.01, [110_000, 110_000, 110_000], None, 0.1, None),
    (16_777_216, 0.01, [167_772], None, 0.0, None),
    (2_000_000, 0.01, [20_000, 20_000, 0, 20_000], [0.2, 1 / 3, 0.25, 0.125], 0.5, None),
    (4_000_000, 0.02, [80_000] * 16, None, 0.2, None),
    # clustered payloads: a block's runs overflow the LDS stage and are halved
    (1_000_000, 0.01, [60_000, 60_000, 60_000], None, 0.0, [0, 10_000, 30_000]),
    (100_000, 0.01, [1_000, 1_000], None, 0.0, None),  # exact-path encode: separate base pass
    (1_000_003, 0.02, [12_345], [0.3], 0.0, None),  # one payload: the per-entry patch
])
def test_foldbase_encode_and_patch_match_oracle(dev, n, alpha, ks, weights, overlap, cluster):
    rng = np.random.default_rng(n + len(ks))
    x = rng.standard_normal(n).astype(np.float32)
    x0 = (x - 0.01 * rng.standard_normal(n)).astype(np.float32)
    k = round(alpha * n)
    pays = _payloads(rng, n, ks, overlap, cluster)
    if weights is None:
        weights = [1 / (len(ks) + 1)] * len(ks)
    w_total = 0
    for v in weights:
        w_total += v
    w_self = 1 - w_total
    tx, tx0 = torch.from_numpy(x).to(dev), torch.from_numpy(x0).to(dev)
    cnt = torch.zeros(n, dtype=torch.int32, device=dev)
    base = torch.empty(n, dtype=torch.float32, device=dev)
    idx, val = codec.topk_encode(tx, k, x0=tx0, counter=cnt, fold_base=(base, weights, w_self))
    o_cnt = np.zeros(n, dtype=np.int32)
    oi, ov = otopk.encode(x, x0, None, 0, k, counter=o_cnt)
    assert np.array_equal(idx.cpu().numpy(), oi)
    assert np.array_equal(_bits(val.cpu().numpy()), _bits(ov))
    assert np.array_equal(cnt.cpu().numpy(), o_cnt)
    empty = [(np.zeros(0, np.int32), np.zeros(0, np.float32))] * len(ks)
    want_base = ofold.fold(x, empty, weights, w_self)
    assert np.array_equal(_bits(base.cpu().numpy()), _bits(want_base))
    dp = [(torch.from_numpy(i).to(dev), torch.from_numpy(v).to(dev)) for i, v in pays]
    out = codec.decode_average(tx, dp, weights, w_self, out=base, base_ready=True)
    want = ofold.fold(x, pays, weights, w_self)
    got = out.cpu().numpy()
    bad = np.flatnonzero(_bits(got) != _bits(want))
    assert bad.size == 0, (bad[:10], got[bad[:5]], want[bad[:5]])
    # the plain fold agrees too
    plain = codec.decode_average(tx, dp, weights, w_self).cpu().numpy()
    assert np.array_equal(_bits(plain), _bits(want))


def test_foldbase_unaligned_base_takes_separate_pass(dev):
    n, k = 1_000_003, 10_000
    rng = np.random.default_rng(7)
    x = rng.standard_normal(n).astype(np.float32)
    x0 = (x - 0.01 * rng.standard_normal(n)).astype(np.float32)
    tx, tx0 = torch.from_numpy(x).to(dev), torch.from_numpy(x0).to(dev)
    buf = torch.empty(n + 1, dtype=torch.float32, device=dev)
    base = buf[1:]  # 4-byte offset: not 16-byte aligned
    w = [0.25, 0.25, 0.25]
    codec.topk_encode(tx, k, x0=tx0, fold_base=(base, w, 0.25))
    empty = [(np.zeros(0, np.int32), np.zeros(0, np.float32))] * 3
    assert np.array_equal(_bits(base.cpu().numpy()), _bits(ofold.fold(x, empty, w, 0.25)))


def test_foldbase_rejects_bad_arguments(dev):
    n, k = 300_000, 3000
    x = torch.randn(n, device=dev)
    x0 = torch.randn(n, device=dev)
    base = torch.empty(n, device=dev)
    with pytest.raises(Exception):
        codec.topk_encode(x, k, x0=x0, fold_base=(base, [], 0.5))  # no weights
    with pytest.raises(Exception):
        codec.topk_encode(x, k, x0=x0, fold_base=(base, [0.1] * 17, 0.5))  # > 16 weights
    with pytest.raises(Exception):
        codec.topk_encode(x, k, x0=x0, fold_base=(x, [0.5], 0.5))  # base over x
    idx = torch.arange(0, n, 100, dtype=torch.int32, device=dev)
    with pytest.raises(Exception):  # a dense payload cannot be patched
        codec.decode_average(x, [(None, x0)], [0.5], 0.5, out=base, base_ready=True)
    with pytest.raises(Exception):  # the server form (no self term) is not a base-ready fold
        codec.decode_average(x, [(idx, x0[:idx.numel()])], [0.5], None, out=base,
                             base_ready=True)


class _OneNbrGraph:
    """uid 0 has the single neighbour 1, whose degree is `deg` (a star leaf, a 2-node run)."""

    def __init__(self, deg):
        self.deg = deg

    def neighbors(self, uid):
        return {1} if uid == 0 else set(range(10, 10 + self.deg))


@pytest.mark.parametrize("msg_degree", [3, 5])
def test_partialmodel_one_neighbour_folds_on_the_encoded_base(dev, tmp_path, msg_degree):
    """PartialModel with one neighbour: the encode writes the Metro-Hastings fold's no-hit base
    (weights predicted from the graph, Sharing.py:156-190) and _averaging patches the payload's
    elements; with a message whose degree breaks the prediction (5) the plain fold runs.  Both
    give the oracle's averaged model bit for bit, over two rounds."""
    from collections import deque

    from decentralizepy_amd.sharing.PartialModel import PartialModel
    from tests import scenario
    shape = (1000, 1000, 7)
    n = shape[0] * shape[1] + shape[2]
    rng = np.random.default_rng(msg_degree)
    model = scenario.make_model(shape)
    x = rng.standard_normal(n).astype(np.float32)
    scenario.set_flat(model, x)
    plugin = PartialModel(0, 0, None, scenario._Mapping(), _OneNbrGraph(3), model, None,
                          str(tmp_path), alpha=0.01)
    for r in range(2):
        x = (scenario.get_flat(model) + 0.01 * rng.standard_normal(n)).astype(np.float32)
        scenario.set_flat(model, x)
        plugin.get_data_to_send()
        assert plugin._fb is not None  # the encode wrote the predicted base
        k = round(0.01 * n)
        idx = np.sort(rng.choice(n, k, replace=False)).astype(np.int32)
        val = rng.standard_normal(k).astype(np.float32)
        msg = {"alpha": 0.01, "indices": idx, "params": val, "send_partial": True,
               "degree": msg_degree, "iteration": r, "CHANNEL": "DPSGD"}
        w = 1 / (max(1, msg_degree) + 1)
        plugin._averaging({1: deque([msg])})
        got = scenario.get_flat(model)
        want = ofold.fold(x, [(idx, val)], [w], 1 - w)
        np.testing.assert_array_equal(_bits(got), _bits(want))
