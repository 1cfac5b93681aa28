"""GPU: the merge fold (csrc/dpz_fold.hip fold_merge_kernel: a group of 5..16 sparse payloads
merged per tile through an LDS hit mask; the JWINS receive, reference sharing/JWINS/Wavelet.py:
269-309, and the Metro-Hastings fold of Sharing.py:156-190) is bit-exact with the oracle's fp32
fold: equal and unequal weights, the server form (no self term), a zero base, the result also
over the local model, ragged sizes, every tile width, and tiles whose entries overflow the value
slots (payloads clustered on one range: the per-payload fallback inside the same launch)."""
import numpy as np
import pytest
import torch

from oracle import fold as ofold

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def _payloads(n, alpha, npay, rng, cluster=None):
    k = max(1, round(alpha * n))
    pays = []
    for i in range(npay):
        if cluster is not None:  # every payload inside one short range: tiles over the slots
            lo, hi = cluster
            idx = np.sort(rng.choice(np.arange(lo, hi), size=min(k, hi - lo), replace=False))
        else:
            idx = np.sort(rng.choice(n, size=k, replace=False))
        pays.append((idx.astype(np.int32), rng.standard_normal(idx.size).astype(np.float32)))
    return pays


def _run(dev, local, pays, weights, w_self, **kw):
    from decentralizepy_amd import codec
    tl = torch.from_numpy(local).to(dev)
    tp = [(torch.from_numpy(i).to(dev), torch.from_numpy(v).to(dev)) for i, v in pays]
    return codec.decode_average(tl, tp, weights, w_self, **kw), tl


@pytest.mark.parametrize("ept", ["4", "8", "16"])
@pytest.mark.parametrize("n,alpha,npay", [(1_000_003, 0.01, 16), (25_009, 0.02, 5),
                                          (2_000_000, 0.005, 12), (300_001, 0.03, 16),
                                          (1_000_003, 0.01, 7)])
def test_merge_fold_matches_oracle(dev, diag_lib, monkeypatch, ept, n, alpha, npay):
    monkeypatch.setenv("DPZ_FOLD_KIND", "8")
    monkeypatch.setenv("DPZ_MERGE_EPT", ept)
    rng = np.random.default_rng(int(alpha * 1000) + npay + n % 97)
    local = rng.standard_normal(n).astype(np.float32)
    pays = _payloads(n, alpha, npay, rng)
    # unequal weights (a node of irregular degree), then the regular graph's equal weights
    weights = [ofold.mh_weight(npay, int(d)) for d in rng.integers(1, 30, size=npay)]
    for w in (weights, [1 / (npay + 1)] * npay):
        w_self = 1 - sum(w)
        out, _ = _run(dev, local, pays, w, w_self)
        np.testing.assert_array_equal(_bits(out.cpu().numpy()),
                                      _bits(ofold.fold(local, pays, w, w_self)))
        out2, _ = _run(dev, local, pays, w, None)  # server form
        np.testing.assert_array_equal(_bits(out2.cpu().numpy()),
                                      _bits(ofold.fold(local, pays, w, None)))


def test_merge_fold_zero_base_and_also_local(dev, diag_lib, monkeypatch):
    monkeypatch.setenv("DPZ_FOLD_KIND", "8")
    n, npay = 700_001, 9
    rng = np.random.default_rng(8)
    local = rng.standard_normal(n).astype(np.float32)
    pays = _payloads(n, 0.02, npay, rng)
    w = [1 / (npay + 1)] * npay
    # zero base (STC's T = zeros; T[idx] = params), fresh total
    zeros = np.zeros(n, np.float32)
    ref = None
    for (i, v), wi in zip(pays, w):
        term = ofold.replace(zeros, i, v) * np.float32(wi)
        ref = (np.float32(0.0) + term) if ref is None else ref + term
    out, _ = _run(dev, np.zeros(n, np.float32), pays, w, None, zero_base=True)
    np.testing.assert_array_equal(_bits(out.cpu().numpy()), _bits(ref))
    # the averaged model also written over the local one
    out, tl = _run(dev, local, pays, w, 1 - sum(w), also_local=True)
    ref = ofold.fold(local, pays, w, 1 - sum(w))
    np.testing.assert_array_equal(_bits(out.cpu().numpy()), _bits(ref))
    np.testing.assert_array_equal(_bits(tl.cpu().numpy()), _bits(ref))


@pytest.mark.parametrize("ept", ["4", "8"])
def test_merge_fold_slot_overflow_falls_back_per_payload(dev, diag_lib, monkeypatch, ept):
    """16 payloads of 3,000 entries each inside one 3,000-element range: every element there is
    hit 16 times, far over the tile's value slots (2 per element) — those tiles fold payload by
    payload; the rest of the tensor takes the merge."""
    monkeypatch.setenv("DPZ_FOLD_KIND", "8")
    monkeypatch.setenv("DPZ_MERGE_EPT", ept)
    n, npay = 400_003, 16
    rng = np.random.default_rng(9)
    local = rng.standard_normal(n).astype(np.float32)
    pays = _payloads(n, 0.0075, npay, rng, cluster=(100_000, 103_000))
    extra = _payloads(n, 0.002, npay, rng)
    pays = [(np.unique(np.concatenate([a[0], b[0]])).astype(np.int32), None)
            for a, b in zip(pays, extra)]
    pays = [(i, rng.standard_normal(i.size).astype(np.float32)) for i, _ in pays]
    w = [ofold.mh_weight(npay, int(d)) for d in rng.integers(1, 30, size=npay)]
    out, _ = _run(dev, local, pays, w, 1 - sum(w))
    np.testing.assert_array_equal(_bits(out.cpu().numpy()),
                                  _bits(ofold.fold(local, pays, w, 1 - sum(w))))
