"""GPU parity tests: HIP kernels (through the C ABI) vs the CPU oracle on identical inputs.

Bar: bit-exact for index sets, gathered values, counters, accumulators, the fp32 fold and the
wavelet coefficients (the oracle restates the reference's fp32 operation order exactly).
"""
import numpy as np
import pytest
import torch

from oracle import fold as ofold
from oracle import topk as otopk
from oracle import wavelet as owav

pytestmark = pytest.mark.gpu


def _codec():
    from decentralizepy_amd import codec
    return codec


def _inputs(n, seed, scale=0.01):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, generator=g, dtype=torch.float32)
    x0 = x - scale * torch.randn(n, generator=g, dtype=torch.float32)
    return x.numpy(), x0.numpy()


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def _run_encode(dev, x, x0, acc, mode, k, counter=True, exact=False, vals_src=None):
    codec = _codec()
    tx = torch.from_numpy(x).to(dev)
    tx0 = torch.from_numpy(x0).to(dev) if x0 is not None else None
    tacc = torch.from_numpy(acc.copy()).to(dev) if acc is not None else None
    tcnt = torch.zeros(x.shape[0], dtype=torch.int32, device=dev) if counter else None
    tvs = torch.from_numpy(vals_src).to(dev) if vals_src is not None else None
    ws = codec.Workspace(dev)
    idx, val = codec.topk_encode(tx, k, x0=tx0, acc=tacc, acc_mode=mode, vals_src=tvs,
                                 counter=tcnt, workspace=ws, exact=exact)
    torch.cuda.synchronize()
    return (idx.cpu().numpy(), val.cpu().numpy(),
            tacc.cpu().numpy() if tacc is not None else None,
            tcnt.cpu().numpy() if tcnt is not None else None)


def _check_encode(dev, x, x0, acc, mode, k, exact=False, vals_src=None):
    o_acc = acc.copy() if acc is not None else None
    o_cnt = np.zeros(x.shape[0], dtype=np.int32)
    oi, ov = otopk.encode(x, x0, o_acc, mode, k, vals_src=vals_src, counter=o_cnt)
    gi, gv, gacc, gcnt = _run_encode(dev, x, x0, acc, mode, k, exact=exact, vals_src=vals_src)
    assert gi.dtype == np.int32 and gi.shape == (k,)
    np.testing.assert_array_equal(gi, oi)
    np.testing.assert_array_equal(_bits(gv), _bits(ov))
    np.testing.assert_array_equal(gcnt, o_cnt)
    if acc is not None:
        np.testing.assert_array_equal(_bits(gacc), _bits(o_acc))


@pytest.mark.parametrize("n", [1000, 100_003, 1_000_000, 4_194_307])
@pytest.mark.parametrize("alpha", [0.01, 0.001, 0.1, 0.5])
@pytest.mark.parametrize("exact", [False, True])
def test_topk_matches_oracle(dev, n, alpha, exact):
    x, x0 = _inputs(n, seed=n % 97)
    k = round(alpha * n)
    _check_encode(dev, x, x0, None, otopk.ACC_NONE, k, exact=exact)


@pytest.mark.parametrize("mode", [otopk.ACC_ACCUMULATE, otopk.ACC_ADD])
@pytest.mark.parametrize("n", [5000, 1_048_576 + 3])
def test_topk_accumulation_modes(dev, mode, n):
    x, x0 = _inputs(n, seed=3)
    acc = (0.01 * np.random.default_rng(1).standard_normal(n)).astype(np.float32)
    _check_encode(dev, x, x0, acc, mode, round(0.01 * n))


def test_topk_full_size_c2(dev):
    """configs[1]: N = 11,000,000, k = 1 % — index set bit-exact vs the oracle."""
    n = 11_000_000
    x, x0 = _inputs(n, seed=0)
    _check_encode(dev, x, x0, None, otopk.ACC_NONE, round(0.01 * n))


def test_topk_64mib(dev):
    n = 16_777_216
    x, x0 = _inputs(n, seed=1)
    _check_encode(dev, x, x0, None, otopk.ACC_NONE, round(0.01 * n))


@pytest.mark.parametrize("k", [0, 1, 2, 999, 1000])
def test_topk_edge_k(dev, k):
    n = 1000
    x, x0 = _inputs(n, seed=5)
    _check_encode(dev, x, x0, None, otopk.ACC_NONE, k)


def test_topk_k0_still_accumulates(dev):
    n = 4099
    x, x0 = _inputs(n, seed=6)
    acc = np.zeros(n, dtype=np.float32)
    _check_encode(dev, x, x0, acc, otopk.ACC_ACCUMULATE, 0)


@pytest.mark.parametrize("n", [3001, 600_000])
def test_topk_heavy_ties_lowest_index_wins(dev, n):
    # most of the model unchanged: |change| == 0 for ~99.5 % -> k-th key is 0 with massive ties
    x, x0 = _inputs(n, seed=7)
    rng = np.random.default_rng(7)
    keep = rng.random(n) < 0.995
    x0 = np.where(keep, x, x0).astype(np.float32)
    _check_encode(dev, x, x0, None, otopk.ACC_NONE, round(0.01 * n))
    # quantised changes: many exact duplicates at every magnitude
    x = np.round(x * 64) / 64
    x0 = np.round(x0 * 64) / 64
    _check_encode(dev, x.astype(np.float32), x0.astype(np.float32), None, otopk.ACC_NONE,
                  round(0.02 * n))


def test_topk_nan_inf(dev):
    n = 300_000
    x, x0 = _inputs(n, seed=8)
    x[[5, 100, 2000]] = np.nan
    x[[7, 50_000]] = np.inf
    x[[9]] = -np.inf
    _check_encode(dev, x, x0, None, otopk.ACC_NONE, round(0.01 * n))
    _check_encode(dev, x, x0, None, otopk.ACC_NONE, 4)


def test_topk_unaligned_views(dev):
    n = 300_001
    x, x0 = _inputs(n + 1, seed=9)
    # views starting one element in: not 16-byte aligned -> scalar-load kernels
    _check_encode(dev, x[1:].copy(), x0[1:].copy(), None, otopk.ACC_NONE, 3000)
    codec = _codec()
    tx = torch.from_numpy(x).to(dev)[1:]
    tx0 = torch.from_numpy(x0).to(dev)[1:]
    idx, val = codec.topk_encode(tx, 3000, x0=tx0)
    oi, ov = otopk.encode(x[1:], x0[1:], None, 0, 3000)
    np.testing.assert_array_equal(idx.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(val.cpu().numpy()), _bits(ov))


def test_topk_sampled_miss_falls_back(dev):
    """Adversarial layout: the large changes sit between the sample chunks, so the sampled window
    misses the k-th key; the device flags it and the exact path must still give the oracle's set."""
    from tests.layouts import miss_layout
    codec = _codec()
    n = 1 << 20
    k = round(0.01 * n)
    x, x0 = miss_layout(n, k)
    tx = torch.from_numpy(x).to(dev)
    tx0 = torch.from_numpy(x0).to(dev)
    ws = codec.Workspace(dev)
    idx, val = codec.topk_encode(tx, k, x0=tx0, workspace=ws, asynchronous=True)
    used = codec.topk_complete(tx, k, idx, val, ws, x0=tx0)
    assert used, "the adversarial layout should have forced the exact fallback"
    oi, ov = otopk.encode(x, x0, None, 0, k)
    np.testing.assert_array_equal(idx.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(val.cpu().numpy()), _bits(ov))


def test_topk_dense_segment(dev):
    """One segment holds far more candidates than its list capacity -> re-read path."""
    n = 1 << 21
    x, x0 = _inputs(n, seed=12)
    # segment 1 ([4096, 8192) at this size) holds no sample chunk; 2000 large changes there
    # overflow its candidate list (cap 1024) without moving the sampled window
    sl = slice(4200, 6200)
    x[sl] = x0[sl] + 0.2 * np.sign(np.random.default_rng(2).standard_normal(2000)).astype(np.float32)
    codec = _codec()
    tx, tx0 = torch.from_numpy(x).to(dev), torch.from_numpy(x0).to(dev)
    ws = codec.Workspace(dev)
    k = round(0.01 * n)
    idx, val = codec.topk_encode(tx, k, x0=tx0, workspace=ws, asynchronous=True)
    used = codec.topk_complete(tx, k, idx, val, ws, x0=tx0)
    assert not used, "dense segment should be handled inside the sampled path"
    _check_encode(dev, x, x0, None, otopk.ACC_NONE, k)


def test_topk_wavelet_domain_values(dev):
    """Selection on a change vector with values gathered from another vector (JWINS layout)."""
    n = 1_000_009
    c, w = _inputs(n, seed=13)
    _check_encode(dev, c, None, None, otopk.ACC_NONE, round(0.1 * n), vals_src=w)
    _check_encode(dev, c, None, None, otopk.ACC_NONE, round(0.01 * n), vals_src=w)


# ---------------------------------------------------------------------------------------------
# decode + fold

def _payload(n, k, seed, local):
    rng = np.random.default_rng(seed)
    idx = np.sort(rng.choice(n, size=k, replace=False)).astype(np.int32)
    vals = (local[idx] + 0.05 * rng.standard_normal(k)).astype(np.float32)
    return idx, vals


@pytest.mark.parametrize("n", [1000, 1_000_003, 11_000_000])
@pytest.mark.parametrize("npay", [1, 3, 16, 20])
def test_fold_matches_oracle(dev, n, npay):
    codec = _codec()
    rng = np.random.default_rng(n + npay)
    local = rng.standard_normal(n).astype(np.float32)
    pays, tpays, degrees = [], [], []
    for i in range(npay):
        if i == 1:  # one dense (full-model) payload in the mix
            vals = rng.standard_normal(n).astype(np.float32)
            pays.append((None, vals))
            tpays.append((None, torch.from_numpy(vals).to(dev)))
        else:
            idx, vals = _payload(n, max(1, n // 100), seed=i, local=local)
            pays.append((idx, vals))
            tpays.append((torch.from_numpy(idx).to(dev), torch.from_numpy(vals).to(dev)))
        degrees.append(int(rng.integers(1, 20)))
    weights = [ofold.mh_weight(npay, d) for d in degrees]
    w_self = 1 - sum(weights)
    ref = ofold.fold(local, pays, weights, w_self)
    tl = torch.from_numpy(local).to(dev)
    out = codec.decode_average(tl, tpays, weights, w_self).cpu().numpy()
    np.testing.assert_array_equal(_bits(out), _bits(ref))
    # server variant: no self term
    ref2 = ofold.fold(local, pays, [1 / npay] * npay, None)
    out2 = codec.decode_average(tl, tpays, [1 / npay] * npay, None).cpu().numpy()
    np.testing.assert_array_equal(_bits(out2), _bits(ref2))


@pytest.mark.parametrize("n,alpha,npay", [(1_000_003, 0.01, 16), (1_000_003, 0.05, 16),
                                          (4_000_037, 0.01, 20), (300_001, 0.2, 3),
                                          (300_001, 0.04, 5), (100_003, 0.99, 2),
                                          (200_003, 0.4, 3), (1_000_003, 0.1, 16),
                                          (1_000_003, 0.15, 16), (1_000_003, 0.2, 16),
                                          (2_000_003, 0.1, 20)])
def test_fold_all_sparse_overlapping(dev, n, alpha, npay):
    """All-sparse payload groups: tiles with at most 2,816 entries take the one-phase hit-chain
    fold, denser tiles (JWINS alpha 0.1-0.2 x 16 payloads) the per-payload phases, inside the
    same launch; payloads share many indices so elements carry 2, 3 and more hits."""
    codec = _codec()
    rng = np.random.default_rng(int(n * alpha) + npay)
    local = rng.standard_normal(n).astype(np.float32)
    k = max(1, round(alpha * n))
    base = rng.choice(n, size=k, replace=False)
    pays, tpays = [], []
    for i in range(npay):
        own = rng.choice(n, size=k, replace=False)
        take = rng.random(k) < (0.5 if i % 2 else 0.2)  # shared with payload 0's set
        idx = np.unique(np.where(take, base, own)).astype(np.int32)
        vals = rng.standard_normal(idx.size).astype(np.float32)
        pays.append((idx, vals))
        tpays.append((torch.from_numpy(idx).to(dev), torch.from_numpy(vals).to(dev)))
    weights = [ofold.mh_weight(npay, int(d)) for d in rng.integers(1, 20, size=npay)]
    w_self = 1 - sum(weights)
    tl = torch.from_numpy(local).to(dev)
    ref = ofold.fold(local, pays, weights, w_self)
    out = codec.decode_average(tl, tpays, weights, w_self).cpu().numpy()
    np.testing.assert_array_equal(_bits(out), _bits(ref))
    ref2 = ofold.fold(local, pays, [1 / npay] * npay, None)
    out2 = codec.decode_average(tl, tpays, [1 / npay] * npay, None).cpu().numpy()
    np.testing.assert_array_equal(_bits(out2), _bits(ref2))


@pytest.mark.parametrize("group", ["0", "1"])
@pytest.mark.parametrize("n,alpha,npay", [(1_000_003, 0.01, 16), (1_000_003, 0.1, 16),
                                          (200_003, 0.4, 3), (100_003, 0.99, 2),
                                          (300_001, 0.12, 20)])
def test_fold_paths_forced(dev, diag_lib, monkeypatch, group, n, alpha, npay):
    """The slotted fold (DPZ_FOLD_GROUP=1: every all-sparse group, incl. sparse alpha, several
    rounds per tile at alpha 0.99 x 2) and the hit-chain / phase paths (DPZ_FOLD_GROUP=0, also at
    dense alpha) are each bit-exact vs the oracle, with and without the self term, and with a
    zero base and accumulation."""
    monkeypatch.setenv("DPZ_FOLD_GROUP", group)
    codec = _codec()
    rng = np.random.default_rng(int(n * alpha) + npay + 17)
    local = rng.standard_normal(n).astype(np.float32)
    k = max(1, round(alpha * n))
    pays, tpays = [], []
    for i in range(npay):
        idx = np.sort(rng.choice(n, size=k, replace=False)).astype(np.int32)
        vals = rng.standard_normal(k).astype(np.float32)
        pays.append((idx, vals))
        tpays.append((torch.from_numpy(idx).to(dev), torch.from_numpy(vals).to(dev)))
    weights = [ofold.mh_weight(npay, int(d)) for d in rng.integers(1, 20, size=npay)]
    w_self = 1 - sum(weights)
    tl = torch.from_numpy(local).to(dev)
    ref = ofold.fold(local, pays, weights, w_self)
    out = codec.decode_average(tl, tpays, weights, w_self).cpu().numpy()
    np.testing.assert_array_equal(_bits(out), _bits(ref))
    ref2 = ofold.fold(local, pays, [1 / npay] * npay, None)
    out2 = codec.decode_average(tl, tpays, [1 / npay] * npay, None).cpu().numpy()
    np.testing.assert_array_equal(_bits(out2), _bits(ref2))
    zeros = np.zeros(n, np.float32)
    start = rng.standard_normal(n).astype(np.float32)
    ref3 = start.copy()
    for (idx, vals), wi in zip(pays, weights):
        ref3 = ref3 + ofold.replace(zeros, idx, vals) * np.float32(wi)
    tout = torch.from_numpy(start).to(dev)
    codec.decode_average(torch.zeros(n, device=dev), tpays, weights, None, zero_base=True,
                         accumulate=True, out=tout)
    np.testing.assert_array_equal(_bits(tout.cpu().numpy()), _bits(ref3))


@pytest.mark.parametrize("kind", ["1", "2", "4", "8"])
@pytest.mark.parametrize("n,alpha,npay,ndense", [(1_000_003, 0.01, 16, 0), (1_000_003, 0.1, 16, 0),
                                                 (2_000_001, 0.25, 16, 0), (300_001, 0.3, 3, 1),
                                                 (300_001, 0.1, 3, 3), (100_003, 0.99, 2, 0),
                                                 (50_000, 0.05, 7, 4), (4097, 0.2, 5, 2),
                                                 (300_001, 0.6, 4, 0), (1_000_003, 0.45, 16, 1),
                                                 (300_001, 0.1, 13, 0), (300_001, 0.4, 14, 0),
                                                 (1_000_003, 0.15, 16, 0), (300_001, 0.07, 15, 0)])
def test_fold_kinds_forced(dev, diag_lib, monkeypatch, kind, n, alpha, npay, ndense):
    """Every fold kernel forced in turn (DPZ_FOLD_KIND 1: classic hit-chain / phase, 2: 4-slot
    group, 4: the walk fold) on sparse groups and on groups with dense (full-share) payloads,
    bit-exact vs the oracle with and without the self term and with a zero base; a kind that
    cannot take a group (dense payloads on the 4-slot and walk paths) runs the classic kernel.
    alpha 0.45 / 0.6 overflow the walk fold's 64-entry windows (its synchronous dense-tile
    path); 7 and 16 payloads walk in groups of four, 13..16 with every group's windows issued
    three groups ahead (DPZ_FOLD_DIST=1 below: one group ahead)."""
    monkeypatch.setenv("DPZ_FOLD_KIND", kind)
    codec = _codec()
    rng = np.random.default_rng(int(n * alpha) + npay + 31 * ndense)
    local = rng.standard_normal(n).astype(np.float32)
    k = max(1, round(alpha * n))
    pays, tpays = [], []
    dense_at = set(rng.choice(npay, size=ndense, replace=False).tolist())
    for i in range(npay):
        if i in dense_at:
            vals = rng.standard_normal(n).astype(np.float32)
            pays.append((None, vals))
            tpays.append((None, torch.from_numpy(vals).to(dev)))
            continue
        idx = np.sort(rng.choice(n, size=k, replace=False)).astype(np.int32)
        vals = rng.standard_normal(k).astype(np.float32)
        pays.append((idx, vals))
        tpays.append((torch.from_numpy(idx).to(dev), torch.from_numpy(vals).to(dev)))
    weights = [ofold.mh_weight(npay, int(d)) for d in rng.integers(1, 20, size=npay)]
    w_self = 1 - sum(weights)
    tl = torch.from_numpy(local).to(dev)
    ref = ofold.fold(local, pays, weights, w_self)
    out = codec.decode_average(tl, tpays, weights, w_self).cpu().numpy()
    np.testing.assert_array_equal(_bits(out), _bits(ref))
    ref2 = ofold.fold(local, pays, [1 / npay] * npay, None)
    out2 = codec.decode_average(tl, tpays, [1 / npay] * npay, None).cpu().numpy()
    np.testing.assert_array_equal(_bits(out2), _bits(ref2))
    if ndense == 0:
        zeros = np.zeros(n, np.float32)
        ref3 = np.zeros(n, np.float32)
        for j, ((idx, vals), wi) in enumerate(zip(pays, weights)):
            term = ofold.replace(zeros, idx, vals) * np.float32(wi)
            ref3 = (np.float32(0) + term) if j == 0 else ref3 + term
        out3 = codec.decode_average(torch.zeros(n, device=dev), tpays, weights, None,
                                    zero_base=True).cpu().numpy()
        np.testing.assert_array_equal(_bits(out3), _bits(ref3))
    # in place over local (DPZ_FOLD_ALSO_LOCAL)
    tl2 = torch.from_numpy(local).to(dev)
    out4 = codec.decode_average(tl2, tpays, weights, w_self, also_local=True)
    np.testing.assert_array_equal(_bits(out4.cpu().numpy()), _bits(ref))
    np.testing.assert_array_equal(_bits(tl2.cpu().numpy()), _bits(ref))


@pytest.mark.parametrize("kind", ["4"])
@pytest.mark.parametrize("dist", ["3", "1"])
@pytest.mark.parametrize("alpha", [0.1, 0.3])
def test_walk_fold_unaligned_views(dev, diag_lib, monkeypatch, kind, dist, alpha):
    """The walk fold's scalar-load build (local / out 4 bytes off a 16-byte boundary), 16
    payloads' windows issued three groups ahead (DPZ_FOLD_DIST 3, the default) and one."""
    monkeypatch.setenv("DPZ_FOLD_KIND", kind)
    monkeypatch.setenv("DPZ_FOLD_DIST", dist)
    codec = _codec()
    n, npay = 300_001, 16
    rng = np.random.default_rng(int(alpha * 100) + 9)
    local = rng.standard_normal(n + 1).astype(np.float32)
    k = round(alpha * n)
    pays, tpays = [], []
    for _ in range(npay):
        idx = np.sort(rng.choice(n, size=k, replace=False)).astype(np.int32)
        vals = rng.standard_normal(k).astype(np.float32)
        pays.append((idx, vals))
        tpays.append((torch.from_numpy(idx).to(dev), torch.from_numpy(vals).to(dev)))
    w = [1 / (npay + 1)] * npay
    tl = torch.from_numpy(local).to(dev)[1:]
    out = torch.empty(n + 1, device=dev)[1:]
    codec.decode_average(tl, tpays, w, 1 - sum(w), out=out)
    ref = ofold.fold(local[1:], pays, w, 1 - sum(w))
    np.testing.assert_array_equal(_bits(out.cpu().numpy()), _bits(ref))


@pytest.mark.parametrize("win,epl,alpha", [("128", "16", 0.2), ("128", "8", 0.3), ("128", "16", 0.12),
                                           ("64", "16", 0.1), ("128", "2", 0.05)])
def test_walk_fold_windows_overflow(dev, diag_lib, monkeypatch, win, epl, alpha):
    """The walk fold of 16 payloads with 64- / 128-entry windows forced onto tiles whose entries
    overflow them (the synchronous extra windows after a full 128-entry window) and onto sparse
    tiles, bit-exact vs the oracle."""
    monkeypatch.setenv("DPZ_FOLD_KIND", "4")
    monkeypatch.setenv("DPZ_FOLD_WIN", win)
    monkeypatch.setenv("DPZ_FOLD_WALK_EPL", epl)
    codec = _codec()
    n, npay = 300_001, 16
    rng = np.random.default_rng(int(alpha * 1000) + int(epl))
    local = rng.standard_normal(n).astype(np.float32)
    k = round(alpha * n)
    pays, tpays = [], []
    for i in range(npay):
        # half the payloads clustered in the first third (denser tiles), half uniform
        hi = n // 3 if i % 2 else n
        idx = np.sort(rng.choice(hi, size=min(k, hi), replace=False)).astype(np.int32)
        vals = rng.standard_normal(len(idx)).astype(np.float32)
        pays.append((idx, vals))
        tpays.append((torch.from_numpy(idx).to(dev), torch.from_numpy(vals).to(dev)))
    w = [1 / (npay + 1)] * npay
    tl = torch.from_numpy(local).to(dev)
    out = codec.decode_average(tl, tpays, w, 1 - sum(w)).cpu().numpy()
    ref = ofold.fold(local, pays, w, 1 - sum(w))
    np.testing.assert_array_equal(_bits(out), _bits(ref))


@pytest.mark.parametrize("group", ["0", "1"])
@pytest.mark.parametrize("alpha", [0.01, 0.1])
def test_fold_unaligned_views(dev, diag_lib, monkeypatch, group, alpha):
    """local / out 4 bytes off a 16-byte boundary: the scalar-load (VEC = false) builds of the
    hit-chain, phase and slotted fold kernels, bit-exact."""
    monkeypatch.setenv("DPZ_FOLD_GROUP", group)
    codec = _codec()
    n, npay = 300_001, 16
    rng = np.random.default_rng(int(alpha * 100) + 5)
    local = rng.standard_normal(n + 1).astype(np.float32)
    k = round(alpha * n)
    pays, tpays = [], []
    for i in range(npay):
        idx = np.sort(rng.choice(n, size=k, replace=False)).astype(np.int32)
        vals = rng.standard_normal(k).astype(np.float32)
        pays.append((idx, vals))
        tpays.append((torch.from_numpy(idx).to(dev), torch.from_numpy(vals).to(dev)))
    weights = [1.0 / (npay + 1)] * npay
    tl = torch.from_numpy(local).to(dev)[1:]
    out = torch.empty(n + 1, device=dev)[1:]
    assert tl.data_ptr() % 16 and out.data_ptr() % 16
    codec.decode_average(tl, tpays, weights, 1.0 / (npay + 1), out=out)
    ref = ofold.fold(local[1:], pays, weights, 1.0 / (npay + 1))
    np.testing.assert_array_equal(_bits(out.cpu().numpy()), _bits(ref))


@pytest.mark.parametrize("alpha", [0.01, 0.1])
def test_fold_zero_base_and_accumulate_dense(dev, alpha):
    """DPZ_FOLD_ZERO_BASE (STC's server total: sparse payloads are zero off their entries, the
    total starts from +0.0) and DPZ_FOLD_ACCUMULATE (Choco: continue a running total) on the
    hit-chain (alpha 0.01) and phase (alpha 0.1 x 16) paths, bit-exact."""
    codec = _codec()
    n, npay = 1_000_003, 16
    rng = np.random.default_rng(int(alpha * 1000))
    k = round(alpha * n)
    pays, tpays = [], []
    for i in range(npay):
        idx = np.sort(rng.choice(n, size=k, replace=False)).astype(np.int32)
        vals = rng.standard_normal(k).astype(np.float32)
        pays.append((idx, vals))
        tpays.append((torch.from_numpy(idx).to(dev), torch.from_numpy(vals).to(dev)))
    w = [1.0 / (npay + 1)] * npay
    zeros = np.zeros(n, np.float32)
    ref = zeros.copy()
    for (idx, vals), wi in zip(pays, w):
        ref = ref + ofold.replace(zeros, idx, vals) * np.float32(wi)
    tl = torch.zeros(n, device=dev)
    out = codec.decode_average(tl, tpays, w, None, zero_base=True).cpu().numpy()
    np.testing.assert_array_equal(_bits(out), _bits(ref))
    start = rng.standard_normal(n).astype(np.float32)
    ref2 = start.copy()
    for (idx, vals), wi in zip(pays, w):
        ref2 = ref2 + ofold.replace(zeros, idx, vals) * np.float32(wi)
    tout = torch.from_numpy(start).to(dev)
    codec.decode_average(tl, tpays, w, None, zero_base=True, accumulate=True, out=tout)
    np.testing.assert_array_equal(_bits(tout.cpu().numpy()), _bits(ref2))


@pytest.mark.parametrize("npay", [0, 3, 20])
def test_fold_also_local_in_place(dev, npay):
    """DPZ_FOLD_ALSO_LOCAL: out and local both end as the fold (local read before overwritten,
    also across chained payload groups)."""
    codec = _codec()
    n = 1_000_003
    rng = np.random.default_rng(npay + 7)
    local = rng.standard_normal(n).astype(np.float32)
    pays, tpays = [], []
    for i in range(npay):
        idx, vals = _payload(n, n // 100, seed=100 + i, local=local)
        pays.append((idx, vals))
        tpays.append((torch.from_numpy(idx).to(dev), torch.from_numpy(vals).to(dev)))
    weights = [1 / (npay + 1)] * npay
    w_self = 1 - sum(weights)
    ref = ofold.fold(local, pays, weights, w_self)
    tl = torch.from_numpy(local).to(dev)
    out = codec.decode_average(tl, tpays, weights, w_self, also_local=True)
    np.testing.assert_array_equal(_bits(out.cpu().numpy()), _bits(ref))
    np.testing.assert_array_equal(_bits(tl.cpu().numpy()), _bits(ref))


@pytest.mark.parametrize("n,k", [(1000, 10), (1000, 0), (1000, 1000), (11_000_000, 110_000)])
def test_replace_matches_oracle(dev, n, k):
    codec = _codec()
    rng = np.random.default_rng(k)
    local = rng.standard_normal(n).astype(np.float32)
    idx, vals = _payload(n, k, seed=1, local=local)
    ref = ofold.replace(local, idx, vals)
    out = codec.replace(torch.from_numpy(local).to(dev), torch.from_numpy(idx).to(dev),
                        torch.from_numpy(vals).to(dev)).cpu().numpy()
    np.testing.assert_array_equal(_bits(out), _bits(ref))


def test_encode_decode_roundtrip_property(dev):
    """Full-size property: decode(encode(x)) equals x on the selected set and local elsewhere."""
    codec = _codec()
    n = 16_777_216
    x, x0 = _inputs(n, seed=21)
    tx, tx0 = torch.from_numpy(x).to(dev), torch.from_numpy(x0).to(dev)
    idx, val = codec.topk_encode(tx, round(0.01 * n), x0=tx0)
    out = codec.replace(tx0, idx, val)
    sel = torch.zeros(n, dtype=torch.bool, device=dev)
    sel[idx.long()] = True
    assert torch.equal(out[sel], tx[sel])
    assert torch.equal(out[~sel], tx0[~sel])
    assert bool((idx[1:] > idx[:-1]).all())


# ---------------------------------------------------------------------------------------------
# wavelet

@pytest.mark.parametrize("n", [64, 65, 66, 67, 101, 1001, 4096, 100_003, 1_000_000, 11_000_001,
                               25_000_000])
def test_wavedec_waverec_bit_exact(dev, n):
    codec = _codec()
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n).astype(np.float32)
    x0 = (x - 0.01 * rng.standard_normal(n)).astype(np.float32)
    tx, tx0 = torch.from_numpy(x).to(dev), torch.from_numpy(x0).to(dev)
    wx, wd = codec.wavedec(tx, 4, x0=tx0)
    np.testing.assert_array_equal(_bits(wx.cpu().numpy()), _bits(owav.wavedec_array(x)))
    np.testing.assert_array_equal(_bits(wd.cpu().numpy()), _bits(owav.wavedec_array(x - x0)))
    # accumulate: acc += W(x - x0)
    acc = (0.01 * rng.standard_normal(wx.numel())).astype(np.float32)
    tacc = torch.from_numpy(acc).to(dev)
    codec.wavedec(tx, 4, x0=tx0, want_x=False, coeffs_diff=tacc, accumulate=True)
    np.testing.assert_array_equal(_bits(tacc.cpu().numpy()),
                                  _bits(acc + owav.wavedec_array(x - x0)))
    rec = codec.waverec(wx, n, 4).cpu().numpy()
    np.testing.assert_array_equal(_bits(rec), _bits(owav.waverec_array(owav.wavedec_array(x), n)))


@pytest.mark.parametrize("level", [1, 2, 3, 5, 6, 8])
@pytest.mark.parametrize("n", [301, 4096, 100_003, 1_000_001])
def test_waverec_levels_bit_exact(dev, n, level):
    """The staged IDWT is instantiated per level (1..8); the forward transform supports <= 4."""
    codec = _codec()
    rng = np.random.default_rng(n + level)
    x = rng.standard_normal(n).astype(np.float32)
    coeffs = owav.wavedec_array(x, level)
    if level <= 4:
        wx, _ = codec.wavedec(torch.from_numpy(x).to(dev), level)
        np.testing.assert_array_equal(_bits(wx.cpu().numpy()), _bits(coeffs))
    rec = codec.waverec(torch.from_numpy(coeffs).to(dev), n, level).cpu().numpy()
    np.testing.assert_array_equal(_bits(rec), _bits(owav.waverec_array(coeffs, n, level)))


@pytest.mark.parametrize("level", [1, 2, 3, 4, 6, 8])
@pytest.mark.parametrize("n", [1, 2, 3, 17, 255, 256, 257, 1001, 65_537, 1_000_003, 25_000_000])
def test_haar_bit_exact(dev, n, level):
    """haar DWT pair / accumulate / IDWT (the reference Wavelet's default wavelet) against the
    pywt-pinned oracle, every level 1-8 (chunk edges at 256, odd lengths at every level)."""
    if n > 1_000_003 and level not in (4, 8):
        pytest.skip("full size at two levels")
    codec = _codec()
    rng = np.random.default_rng(n * 10 + level)
    x = rng.standard_normal(n).astype(np.float32)
    x0 = (x - 0.01 * rng.standard_normal(n)).astype(np.float32)
    tx, tx0 = torch.from_numpy(x).to(dev), torch.from_numpy(x0).to(dev)
    wx, wd = codec.wavedec(tx, level, x0=tx0, wavelet="haar")
    cx = owav.wavedec_array(x, level, "haar")
    np.testing.assert_array_equal(_bits(wx.cpu().numpy()), _bits(cx))
    np.testing.assert_array_equal(_bits(wd.cpu().numpy()),
                                  _bits(owav.wavedec_array(x - x0, level, "haar")))
    acc = (0.01 * rng.standard_normal(wx.numel())).astype(np.float32)
    tacc = torch.from_numpy(acc).to(dev)
    codec.wavedec(tx, level, x0=tx0, want_x=False, coeffs_diff=tacc, accumulate=True,
                  wavelet="haar")
    np.testing.assert_array_equal(_bits(tacc.cpu().numpy()),
                                  _bits(acc + owav.wavedec_array(x - x0, level, "haar")))
    wxo, _ = codec.wavedec(tx, level, wavelet="haar")
    np.testing.assert_array_equal(_bits(wxo.cpu().numpy()), _bits(cx))
    rec = codec.waverec(wx, n, level, wavelet="haar").cpu().numpy()
    np.testing.assert_array_equal(_bits(rec), _bits(owav.waverec_array(cx, n, level, "haar")))


def test_fp16_pack_roundtrip(dev):
    codec = _codec()
    for n in [1, 7, 8, 9, 1_000_003]:
        x = (np.random.default_rng(n).standard_normal(n) * 10).astype(np.float32)
        h = codec.pack_fp16(torch.from_numpy(x).to(dev))
        ref = torch.from_numpy(x).half()
        assert torch.equal(h.cpu().view(torch.int16), ref.view(torch.int16))
        back = codec.unpack_fp16(h).cpu()
        assert torch.equal(back, ref.float())


def test_topk_workspace_reuse_across_calls_and_misses(dev):
    """The sampled path's self-cleaning workspace (sample histogram, boundary sub-list counters)
    must be clean after normal calls and after a miss that fell back to the exact path."""
    codec = _codec()
    ws = codec.Workspace(dev)
    n = 1 << 20
    k = round(0.01 * n)
    for seed in (21, 22):
        x, x0 = _inputs(n, seed=seed)
        tx, tx0 = torch.from_numpy(x).to(dev), torch.from_numpy(x0).to(dev)
        for _ in range(2):
            idx, val = codec.topk_encode(tx, k, x0=tx0, workspace=ws)
            oi, ov = otopk.encode(x, x0, None, 0, k)
            np.testing.assert_array_equal(idx.cpu().numpy(), oi)
        # quantised input: thousands of equal keys in the threshold bin overflow the boundary
        # sub-lists -> miss -> exact fallback; the next call must start clean
        xq = (np.round(x * 8) / 8).astype(np.float32)
        tq = torch.from_numpy(xq).to(dev)
        idx, val = codec.topk_encode(tq, k, x0=tx0, workspace=ws)
        oi, ov = otopk.encode(xq, x0, None, 0, k)
        np.testing.assert_array_equal(idx.cpu().numpy(), oi)
        np.testing.assert_array_equal(_bits(val.cpu().numpy()), _bits(ov))


@pytest.mark.parametrize("n,alpha", [(1_000_003, 0.01), (300_000, 0.2)])
def test_split_stream_tail_enqueue(dev, n, alpha):
    """DPZ_TOPK_STREAM then DPZ_TOPK_TAIL (another stream's decode in between) == one-shot encode;
    alpha = 0.2 takes the exact path, where STREAM does everything and TAIL nothing."""
    codec = _codec()
    x, x0 = _inputs(n, 21)
    k = round(alpha * n)
    o_cnt = np.zeros(n, dtype=np.int32)
    oi, ov = otopk.encode(x, x0, None, 0, k, counter=o_cnt)
    tx, tx0 = torch.from_numpy(x).to(dev), torch.from_numpy(x0).to(dev)
    cnt = torch.zeros(n, dtype=torch.int32, device=dev)
    idx = torch.empty(k, dtype=torch.int32, device=dev)
    val = torch.empty(k, dtype=torch.float32, device=dev)
    ws = codec.Workspace(dev)
    side = torch.cuda.Stream(dev)
    codec.topk_encode(tx, k, x0=tx0, counter=cnt, idx_out=idx, val_out=val, workspace=ws,
                      phase="stream")
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):  # unrelated decode on the other stream meanwhile
        other = codec.replace(tx0, torch.tensor([5], dtype=torch.int32, device=dev),
                              torch.tensor([1.5], dtype=torch.float32, device=dev))
    codec.topk_encode(tx, k, x0=tx0, counter=cnt, idx_out=idx, val_out=val, workspace=ws,
                      phase="tail")
    codec.topk_complete(tx, k, idx, val, ws, x0=tx0, counter=cnt)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(idx.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(val.cpu().numpy()), _bits(ov))
    np.testing.assert_array_equal(cnt.cpu().numpy(), o_cnt)
    want = x0.copy()
    want[5] = 1.5
    np.testing.assert_array_equal(_bits(other.cpu().numpy()), _bits(want))


@pytest.mark.parametrize("n,alpha,rn,rk,shares", [
    (11_000_000, 0.01, 11_000_000, 110_000, None),          # C2: the bench's pipelined step
    (16_777_216, 0.01, 1_000_003, 10_000, None),            # different sizes of the two jobs
    (1_000_003, 0.01, 16_777_216, 167_772, "1,0,0"),      # everything in one host launch
    (1_000_003, 0.01, 4_000_000, 40_000, "0,0,1"),
    (1_000_003, 0.01, 4_000_000, 40_000, "0,1,0"),
    (300_000, 0.2, 500_000, 5_000, None),                   # exact path: decode runs on its own
    (1_000_003, 0.01, 1000, 0, None),                        # empty payload: plain copy
])
def test_encode_with_coscheduled_replace(dev, n, alpha, rn, rk, shares, monkeypatch, diag_lib):
    """dpz_topk_encode_replace == dpz_topk_encode + an independent replace decode, bit-exact,
    for any split of the decode's chunks over the encoder's launches (DPZ_COSCHED)."""
    codec = _codec()
    if shares is not None:
        monkeypatch.setenv("DPZ_COSCHED", shares)
    x, x0 = _inputs(n, 5)
    k = round(alpha * n)
    o_cnt = np.zeros(n, dtype=np.int32)
    oi, ov = otopk.encode(x, x0, None, 0, k, counter=o_cnt)
    rng = np.random.default_rng(rk + 3)
    local = rng.standard_normal(rn).astype(np.float32)
    ridx, rvals = _payload(rn, rk, seed=2, local=local)
    ref = ofold.replace(local, ridx, rvals)
    tx, tx0 = torch.from_numpy(x).to(dev), torch.from_numpy(x0).to(dev)
    cnt = torch.zeros(n, dtype=torch.int32, device=dev)
    tl = torch.from_numpy(local).to(dev)
    out = torch.full_like(tl, float("nan"))
    ws = codec.Workspace(dev)
    idx, val = codec.topk_encode(tx, k, x0=tx0, counter=cnt, workspace=ws,
                                 co_replace=(tl, torch.from_numpy(ridx).to(dev),
                                             torch.from_numpy(rvals).to(dev), out))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(idx.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(val.cpu().numpy()), _bits(ov))
    np.testing.assert_array_equal(cnt.cpu().numpy(), o_cnt)
    np.testing.assert_array_equal(_bits(out.cpu().numpy()), _bits(ref))


def test_coscheduled_replace_rejects_aliasing(dev):
    codec = _codec()
    n = 1_000_003
    x, x0 = _inputs(n, 5)
    tx, tx0 = torch.from_numpy(x).to(dev), torch.from_numpy(x0).to(dev)
    p_idx = torch.tensor([3], dtype=torch.int32, device=dev)
    p_val = torch.tensor([1.0], dtype=torch.float32, device=dev)
    with pytest.raises(RuntimeError):  # decode output overlapping the encoder's input
        codec.topk_encode(tx, 10_000, x0=tx0, co_replace=(tx0.clone(), p_idx, p_val, tx))


@pytest.mark.parametrize("where", ["select", "compact", "split", "compact-first"])
@pytest.mark.parametrize("n,alpha,rk,dup,layout", [
    (11_000_000, 0.01, 110_000, False, None),      # C2: the bench's one-node step
    (16_777_216, 0.01, 167_772, False, None),      # 64 MiB
    (1_000_001, 0.01, 7_000, True, None),          # ragged n; adjacent duplicate indices
    (1_000_003, 0.01, 0, False, None),             # empty payload: the copy only
    (1 << 20, 0.01, 9_000, False, "miss"),         # sampled window misses: exact re-run
    (11_000_000, 0.01, 5, True, None),             # far fewer entries than wave segments
    (11_000_000, 0.01, 110_000, True, "cluster"),  # entries packed at both ends: long gaps
])
def test_encode_with_fused_replace(dev, n, alpha, rk, dup, layout, where, monkeypatch, diag_lib):
    """Decoding over the tensor being encoded (co_replace local is x): the encoder's filter
    writes out = x as it streams x and the select launch (or, DPZ_SCATTER_AT=compact, the
    compact launch) scatters the entries (dpz_topk_encode_replace); equals encode +
    T = x.copy(); T[idx] = vals, bit-exact."""
    monkeypatch.setenv("DPZ_SCATTER_AT", where.split("-")[0])
    # compact-first: the decode's blocks dispatched ahead of compact's own (DPZ_SCATTER_FIRST)
    monkeypatch.setenv("DPZ_SCATTER_FIRST", "1" if where.endswith("first") else "0")
    codec = _codec()
    k = round(alpha * n)
    if layout == "miss":
        from tests.layouts import miss_layout
        x, _ = miss_layout(n, k)
        x0 = None
    else:
        x, x0 = _inputs(n, 9)
    o_cnt = np.zeros(n, dtype=np.int32)
    oi, ov = otopk.encode(x, x0, None, 0, k, counter=o_cnt)
    ridx, rvals = _payload(n, rk, seed=4, local=x)
    if layout == "cluster":  # most entries in the first 1 %, the rest in the last 0.1 %
        rng = np.random.default_rng(5)
        a = rng.choice(n // 100, size=rk - rk // 10, replace=False)
        b = n - 1 - rng.choice(n // 1000, size=rk // 10, replace=False)
        ridx = np.sort(np.concatenate([a, b])).astype(np.int32)
    if dup and rk > 2:  # entries j and j + 1 share an index: the later value wins
        ridx[rk // 2 + 1] = ridx[rk // 2]
        ridx[-1] = ridx[-2]
    ref = ofold.replace(x, ridx, rvals)
    tx = torch.from_numpy(x).to(dev)
    tx0 = torch.from_numpy(x0).to(dev) if x0 is not None else None
    cnt = torch.zeros(n, dtype=torch.int32, device=dev)
    out = torch.full_like(tx, float("nan"))
    ws = codec.Workspace(dev)
    idx, val = codec.topk_encode(tx, k, x0=tx0, counter=cnt, workspace=ws,
                                 co_replace=(tx, torch.from_numpy(ridx).to(dev),
                                             torch.from_numpy(rvals).to(dev), out))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(idx.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(val.cpu().numpy()), _bits(ov))
    np.testing.assert_array_equal(cnt.cpu().numpy(), o_cnt)
    np.testing.assert_array_equal(_bits(out.cpu().numpy()), _bits(ref))


def _sampled_status(ws):
    return int(ws.buf[8:12].view(torch.int32).item())


def test_topk_c5_alpha_0001_stays_on_sampled_path(dev):
    """C5 (N = 2^26, alpha = 0.001): bit-exact vs the oracle AND no exact-path fallback (the
    window's top rank is clamped to the largest sample; an open window overflowed the boundary
    list here)."""
    codec = _codec()
    n = 67_108_864
    k = round(0.001 * n)
    x, x0 = _inputs(n, seed=4)
    o_cnt = np.zeros(n, dtype=np.int32)
    oi, ov = otopk.encode(x, x0, None, otopk.ACC_NONE, k, counter=o_cnt)
    tx, tx0 = torch.from_numpy(x).to(dev), torch.from_numpy(x0).to(dev)
    cnt = torch.zeros(n, dtype=torch.int32, device=dev)
    ws = codec.Workspace(dev)
    idx, val = codec.topk_encode(tx, k, x0=tx0, counter=cnt, workspace=ws, asynchronous=True)
    torch.cuda.synchronize()
    assert _sampled_status(ws) == 0, "C5 shape fell back to the exact path"
    np.testing.assert_array_equal(idx.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(val.cpu().numpy()), _bits(ov))
    np.testing.assert_array_equal(cnt.cpu().numpy(), o_cnt)


def test_topk_c3_wavelet_rounds_stay_on_sampled_path(dev):
    """C3 shape (M = 25,000,009 wavelet coefficients, alpha = 0.01, ADD accumulation with the
    rewind of selected coefficients, 4 rounds): no exact-path fallback (256 fine bins
    overflowed the boundary list here) and the last round bit-exact vs the oracle."""
    codec = _codec()
    n = 25_000_000
    m = codec.wavedec_len(n, 4)
    k = round(0.01 * m)
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(n, device=dev, generator=g)
    x0 = x - 0.01 * torch.randn(n, device=dev, generator=g)
    acc = 0.01 * torch.randn(m, device=dev, generator=g)
    wx, wc = codec.wavedec(x, 4, x0=x0)
    ws = codec.Workspace(dev)
    for r in range(4):
        acc_before = acc.cpu().numpy().copy()
        idx, val = codec.topk_encode(wc, k, acc=acc, acc_mode=codec.DPZ_ACC_ADD, vals_src=wx,
                                     workspace=ws, asynchronous=True)
        torch.cuda.synchronize()
        assert _sampled_status(ws) == 0, f"round {r} fell back to the exact path"
    o_acc = acc_before.copy()
    oi, ov = otopk.encode(wc.cpu().numpy(), None, o_acc, otopk.ACC_ADD, k,
                          vals_src=wx.cpu().numpy())
    np.testing.assert_array_equal(idx.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(val.cpu().numpy()), _bits(ov))
    np.testing.assert_array_equal(_bits(acc.cpu().numpy()), _bits(o_acc))


@pytest.mark.parametrize("n,alpha", [(11_000_000, 0.01), (16_777_216, 0.01), (3_000_017, 0.1)])
def test_shared_and_lone_filter_grids_agree(dev, n, alpha):
    """DPZ_TOPK_SHARED (the smaller filter grid for several codecs per GPU) and the lone-codec
    grid select the same payload and make the same counter update, bit for bit."""
    from decentralizepy_amd import codec
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(n, device=dev, generator=g)
    x0 = x - 0.01 * torch.randn(n, device=dev, generator=g)
    k = round(alpha * n)
    res = []
    for shared in (False, True):
        cnt = torch.zeros(n, dtype=torch.int32, device=dev)
        ws = codec.Workspace(dev)
        idx, val = codec.topk_encode(x, k, x0=x0, counter=cnt, workspace=ws, shared=shared)
        assert codec.topk_status(ws) == 0  # the sampled path, no fallback
        res.append((idx.cpu(), val.cpu(), cnt.cpu()))
    for a, b in zip(*res):
        assert torch.equal(a, b)


@pytest.mark.parametrize("plain", ["0", "1"])
@pytest.mark.parametrize("n,alpha,mode", [(3_000_017, 0.01, otopk.ACC_NONE),
                                          (3_000_017, 0.1, otopk.ACC_ADD),
                                          (1_000_003, 0.3, otopk.ACC_ACCUMULATE)])
def test_counter_update_forms_agree(dev, diag_lib, monkeypatch, plain, n, alpha, mode):
    """The compact's counter update as memory-side atomics (DPZ_COUNTER_PLAIN=0) and as gathered
    read + plain store (=1, the dense-alpha default) both give counter[idx] += 1 on a counter
    that already holds counts, with the accumulator rewound, bit-exact vs the oracle."""
    monkeypatch.setenv("DPZ_COUNTER_PLAIN", plain)
    from decentralizepy_amd import codec
    x, x0 = _inputs(n, seed=n % 89 + int(alpha * 100))
    rng = np.random.default_rng(3)
    cnt0 = rng.integers(0, 50, size=n).astype(np.int32)
    acc = (0.01 * rng.standard_normal(n)).astype(np.float32) if mode != otopk.ACC_NONE else None
    k = round(alpha * n)
    o_cnt, o_acc = cnt0.copy(), (acc.copy() if acc is not None else None)
    oi, ov = otopk.encode(x, x0, o_acc, mode, k, counter=o_cnt)
    tcnt = torch.from_numpy(cnt0.copy()).to(dev)
    tacc = torch.from_numpy(acc.copy()).to(dev) if acc is not None else None
    ws = codec.Workspace(dev)
    idx, val = codec.topk_encode(torch.from_numpy(x).to(dev), k, x0=torch.from_numpy(x0).to(dev),
                                 acc=tacc, acc_mode=mode, counter=tcnt, workspace=ws)
    assert codec.topk_status(ws) == 0
    np.testing.assert_array_equal(idx.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(val.cpu().numpy()), _bits(ov))
    np.testing.assert_array_equal(tcnt.cpu().numpy(), o_cnt)
    if acc is not None:
        np.testing.assert_array_equal(_bits(tacc.cpu().numpy()), _bits(o_acc))


@pytest.mark.parametrize("alpha", [0.1, 0.01])
def test_fold_c3_full_size_16_payloads(dev, alpha):
    """The C3 shape the bench times: 16 sparse payloads folded over the sym2
    level-4 coefficient vector of a 25 M model, M = 25,000,009 (odd: the walk fold's ragged
    vector path), at the tutorial's alpha 0.1 (walk fold) and 0.01 (hit-chain fold), bit-exact
    against the oracle's Metro-Hastings fold (reference sharing/JWINS/Wavelet.py:269-309)."""
    codec = _codec()
    m, npay = 25_000_009, 16
    k = round(alpha * m)
    g = torch.Generator(device=dev).manual_seed(31)
    local_t = torch.randn(m, device=dev, generator=g)
    tpays, pays = [], []
    for i in range(npay):
        idx = torch.sort(torch.randperm(m, device=dev, generator=g)[:k])[0].to(torch.int32)
        vals = torch.randn(k, device=dev, generator=g)
        tpays.append((idx, vals))
        pays.append((idx.cpu().numpy(), vals.cpu().numpy()))
    w = [1 / (npay + 1)] * npay
    w_self = 1 - sum(w)
    out = codec.decode_average(local_t, tpays, w, w_self).cpu().numpy()
    ref = ofold.fold(local_t.cpu().numpy(), pays, w, w_self)
    np.testing.assert_array_equal(_bits(out), _bits(ref))
