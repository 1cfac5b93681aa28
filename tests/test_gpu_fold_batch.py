"""GPU: dpz_decode_average_batch's one-launch path (dpz_fold.hip fold_walk_batch_kernel: the plain
Metro-Hastings folds of many nodes, <= 4 sparse payloads each, in one launch per 22 nodes) is
bit-exact against the oracle's fold of each node (reference sharing/Sharing.py:156-190 over
PartialModel payloads, PartialModel.py:257-303) — across launch boundaries, mixed payload counts
and sizes, tile sizes from the payload density, the in-place copy over the local model
(DPZ_FOLD_ALSO_LOCAL), and against the per-node launches of the diagnostic build."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import fold as ofold

pytestmark = pytest.mark.gpu


def _ptrs(ts):
    return (ctypes.c_void_p * max(1, len(ts)))(*[t.data_ptr() for t in ts])


def _batch(L, locs, outs, pays, weights, w_selfs, flags, dev):
    from decentralizepy_amd import codec
    m, n = len(locs), locs[0].numel()
    counts = [len(p) for p in pays]
    idx = [i for p in pays for i, _ in p]
    val = [v for p in pays for _, v in p]
    kk = (ctypes.c_int64 * len(idx))(*[i.numel() for i in idx])
    w = (ctypes.c_float * len(idx))(*[x for ws in weights for x in ws])
    ws_ = (ctypes.c_float * m)(*w_selfs)
    wss = [codec.Workspace(dev) for _ in range(3)]
    dws = [x.get_decode(n, 4) for x in wss]
    streams = [torch.cuda.current_stream(dev)] * 3
    st = (ctypes.c_void_p * 3)(*[s.cuda_stream for s in streams])
    rc = L.dpz_decode_average_batch(m, _ptrs(locs), _ptrs(outs), n, (ctypes.c_int * m)(*counts),
                                    _ptrs(idx), _ptrs(val), kk, w, ws_, flags, _ptrs(dws),
                                    min(d.numel() for d in dws), 3, st)
    assert rc == 0
    torch.cuda.synchronize()


def _case(dev, m, n, alpha, seed):
    g = torch.Generator().manual_seed(seed)
    rng = np.random.default_rng(seed)
    xs = [torch.randn(n, generator=g) for _ in range(m)]
    pays, weights, w_selfs = [], [], []
    for j in range(m):
        npay = 1 + (j % 4)
        p = []
        for q in range(npay):
            k = max(1, int(alpha * n * (0.5 + rng.random())))
            i = np.sort(rng.choice(n, size=k, replace=False)).astype(np.int32)
            p.append((i, rng.standard_normal(k).astype(np.float32)))
        pays.append(p)
        w = [1 / (npay + 1)] * npay
        tot = 0
        for v in w:
            tot += v
        weights.append(w)
        w_selfs.append(1 - tot)
    return xs, pays, weights, w_selfs


@pytest.mark.parametrize("m,n,alpha", [(30, 100_003, 0.01), (5, 1_000_000, 0.08),
                                       (23, 65_536, 0.3), (2, 11_000_000, 0.01)])
@pytest.mark.parametrize("also_local", [False, True])
def test_fold_batch_matches_oracle(dev, m, n, alpha, also_local):
    from decentralizepy_amd import _lib
    from decentralizepy_amd._lib import DPZ_FOLD_ALSO_LOCAL, DPZ_FOLD_SELF
    xs, pays, weights, w_selfs = _case(dev, m, n, alpha, seed=m + n)
    locs = [x.to(dev) for x in xs]
    outs = [torch.full((n,), float("nan"), device=dev) for _ in range(m)]
    dp = [[(torch.from_numpy(i).to(dev), torch.from_numpy(v).to(dev)) for i, v in p] for p in pays]
    flags = DPZ_FOLD_SELF | (DPZ_FOLD_ALSO_LOCAL if also_local else 0)
    _batch(_lib.lib(), locs, outs, dp, weights, w_selfs, flags, dev)
    for j in range(m):
        ref = ofold.fold(xs[j].numpy(), pays[j], weights[j], w_selfs[j])
        np.testing.assert_array_equal(outs[j].cpu().numpy().view(np.uint32), ref.view(np.uint32),
                                      err_msg=f"node {j}")
        want_local = ref if also_local else xs[j].numpy()
        np.testing.assert_array_equal(locs[j].cpu().numpy().view(np.uint32),
                                      want_local.view(np.uint32))


def test_fold_batch_equals_per_node_launches(dev, diag_lib, monkeypatch):
    """The diagnostic build's DPZ_FOLD_BATCH=0 forces one launch per node: same bits."""
    from decentralizepy_amd._lib import DPZ_FOLD_SELF
    m, n = 25, 300_007
    xs, pays, weights, w_selfs = _case(dev, m, n, 0.02, seed=7)
    dp = [[(torch.from_numpy(i).to(dev), torch.from_numpy(v).to(dev)) for i, v in p] for p in pays]
    res = []
    for env in ("1", "0"):
        monkeypatch.setenv("DPZ_FOLD_BATCH", env)
        locs = [x.to(dev) for x in xs]
        outs = [torch.empty(n, device=dev) for _ in range(m)]
        _batch(diag_lib, locs, outs, dp, weights, w_selfs, DPZ_FOLD_SELF, dev)
        res.append(torch.stack(outs).cpu().numpy())
    np.testing.assert_array_equal(res[0].view(np.uint32), res[1].view(np.uint32))
