"""GPU parity of the encode's coalesced side effects (dpz_topk_encode_sliced): the selection is
dpz_topk_encode's, the bit-sliced counter equals the oracle's int32 counter after
``counter[idx] += 1``, the selection mask holds exactly the selected indices, the accumulator is
untouched until the deferred rewind, and the accumulating post-step with the mask
(dpz_dwt_sym2_rewind / dpz_dwt_haar_rewind) equals the reference's rewind-then-add
(sharing/JWINS/Wavelet.py:194-197, models/Model.py:53-64, sharing/PartialModel.py:346-349)."""
import numpy as np
import pytest
import torch

from oracle import topk as otopk
from oracle import wavelet as owav

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.asarray(a, dtype=np.float32).view(np.uint32)


def _mask_of(idx, n):
    words = np.zeros((n + 31) // 32, dtype=np.uint32)
    np.bitwise_or.at(words, idx >> 5, (np.uint32(1) << (idx & 31).astype(np.uint32)))
    return words


def _counter0(rng, n):
    """Initial counters with long carry chains: random small counts, some 2^p - 1 values."""
    c = rng.integers(0, 1 << 12, n).astype(np.int32)
    sel = rng.choice(n, size=max(1, n // 50), replace=False)
    c[sel] = (np.int32(1) << rng.integers(1, 31, sel.size).astype(np.int32)) - 1
    return c


def _run(dev, x, x0, acc, mode, k, vals=None, status=False, exact=False, seed=0, poison=False):
    from decentralizepy_amd import codec
    n = x.size
    rng = np.random.default_rng(seed)
    c0 = _counter0(rng, n)
    tx = torch.from_numpy(x).to(dev)
    tx0 = torch.from_numpy(x0).to(dev) if x0 is not None else None
    tacc = torch.from_numpy(acc).to(dev) if acc is not None else None
    tv = torch.from_numpy(vals).to(dev) if vals is not None else None
    planes = codec.counter_slice(torch.from_numpy(c0).to(dev))
    np.testing.assert_array_equal(codec.counter_unslice(planes, n).cpu().numpy(), c0)
    nw = codec.mask_words(n)
    mask = torch.full((nw,), -0x54545455, dtype=torch.int32, device=dev)  # garbage: overwritten
    ws = codec.Workspace(dev)
    st = torch.full((1,), 7, dtype=torch.int32, device=dev) if status else None
    # poison: idx_out starts with indices far outside [0, n) (what a reused buffer may hold when a
    # sampled miss leaves it unwritten)
    io = torch.full((k,), 0x7FFFFFF0, dtype=torch.int32, device=dev) if poison else None
    idx, val = codec.topk_encode_sliced(tx, k, mask, planes, x0=tx0, acc=tacc, acc_mode=mode,
                                        vals_src=tv, idx_out=io, workspace=ws, status_out=st,
                                        exact=exact)
    if status:
        torch.cuda.synchronize()
        if int(st.item()) != 0:  # a sampled miss wrote nothing: the caller re-runs exactly
            idx, val = codec.topk_encode_sliced(tx, k, mask, planes, x0=tx0, acc=tacc,
                                                acc_mode=mode, vals_src=tv, workspace=ws,
                                                exact=True)
    o_acc = acc.copy() if acc is not None else None
    o_cnt = c0.copy()
    oi, ov = otopk.encode(x, x0, o_acc, mode, k, vals_src=vals, counter=o_cnt)
    np.testing.assert_array_equal(idx.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(val.cpu().numpy()), _bits(ov))
    np.testing.assert_array_equal(codec.counter_unslice(planes, n).cpu().numpy(), o_cnt)
    np.testing.assert_array_equal(mask.cpu().numpy().view(np.uint32), _mask_of(oi, n))
    if tacc is not None:
        # the encode only read acc; the deferred rewind gives the reference's accumulator
        np.testing.assert_array_equal(_bits(tacc.cpu().numpy()), _bits(acc))
        codec.rewind_apply(tacc, mask)
        np.testing.assert_array_equal(_bits(tacc.cpu().numpy()), _bits(o_acc))
    return ws


def _inputs(n, seed):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal(n).astype(np.float32)
    x0 = (x - 0.01 * rng.standard_normal(n)).astype(np.float32)
    acc = (0.01 * rng.standard_normal(n)).astype(np.float32)
    return x, x0, acc


@pytest.mark.parametrize("n,alpha,mode,status", [
    (300_007, 0.1, otopk.ACC_ADD, False),
    (300_007, 0.01, otopk.ACC_ADD, True),
    (1_000_003, 0.3, otopk.ACC_NONE, False),
    (2_000_000, 0.4, otopk.ACC_ADD, True),
    (4_000_037, 0.001, otopk.ACC_NONE, True),
    (100_000, 0.1, otopk.ACC_ADD, False),  # n < 2^18: the exact path, masks from idx_out
    (25_000_009, 0.1, otopk.ACC_ADD, True),  # the C3 shape (JWINS 25 M, tutorial alpha)
])
def test_sliced_encode_matches_oracle(dev, n, alpha, mode, status):
    x, x0, acc = _inputs(n, seed=n % 97)
    k = round(alpha * n)
    if mode == otopk.ACC_ADD:  # the JWINS layout: keys from W(x - x0) + acc, values from W(x)
        _run(dev, x - x0, None, acc, mode, k, vals=x, status=status)
    else:
        _run(dev, x, x0, None, mode, k, status=status)


def test_sliced_exact_flag_and_k0(dev):
    n = 500_003
    x, x0, acc = _inputs(n, seed=4)
    _run(dev, x - x0, None, acc, otopk.ACC_ADD, round(0.05 * n), vals=x, exact=True)
    _run(dev, x - x0, None, acc, otopk.ACC_ADD, 0, vals=x)


def test_sliced_ties_and_dense_segment(dev):
    """Quantised changes (heavy ties at the k-th key: lowest indices win) and one segment whose
    candidates overflow its list (the dense re-read path writes the mask bits too)."""
    n = 1 << 21
    rng = np.random.default_rng(12)
    x = rng.standard_normal(n).astype(np.float32)
    x0 = (x - np.round(100 * 0.01 * rng.standard_normal(n)) / 100).astype(np.float32)
    _run(dev, x, x0, None, otopk.ACC_NONE, round(0.02 * n))
    x, x0, acc = _inputs(n, seed=12)
    sl = slice(4200, 6200)
    x[sl] = x0[sl] + 0.2 * np.sign(rng.standard_normal(2000)).astype(np.float32)
    _run(dev, x, x0, None, otopk.ACC_NONE, round(0.01 * n))


def test_sliced_sampled_miss(dev):
    """The adversarial layout that makes the sampled window miss: blocking call (re-run inside)
    and asynchronous call (status word, caller re-runs exactly) both end at the oracle."""
    from tests.layouts import miss_layout
    n = 1 << 20
    k = round(0.01 * n)
    x, x0 = miss_layout(n, k)
    _run(dev, x, x0, None, otopk.ACC_NONE, k)
    _run(dev, x, x0, None, otopk.ACC_NONE, k, status=True)


@pytest.mark.parametrize("wavelet,n,level", [("sym2", 1_000_003, 4), ("sym2", 25_000_000, 4),
                                             ("sym2", 5_003, 3), ("haar", 1_000_003, 4),
                                             ("haar", 70_001, 7)])
def test_dwt_rewind_matches_rewind_then_accumulate(dev, wavelet, n, level):
    from decentralizepy_amd import codec
    rng = np.random.default_rng(n + level)
    x = rng.standard_normal(n).astype(np.float32)
    x0 = (x - 0.01 * rng.standard_normal(n)).astype(np.float32)
    m = codec.wavedec_len(n, level, wavelet)
    acc = (0.01 * rng.standard_normal(m)).astype(np.float32)
    sel = np.sort(rng.choice(m, size=m // 10, replace=False)).astype(np.int32)
    acc[sel[:7]] = -0.0  # a rewound -0.0 comes back as +0.0 + c
    tx, tx0 = torch.from_numpy(x).to(dev), torch.from_numpy(x0).to(dev)
    mask = torch.from_numpy(_mask_of(sel, m).view(np.int32)).to(dev)
    a1 = torch.from_numpy(acc).to(dev)
    codec.wavedec(tx, level, x0=tx0, want_x=False, coeffs_diff=a1, accumulate=True,
                  wavelet=wavelet, rewind_mask=mask)
    a2 = torch.from_numpy(acc).to(dev)
    codec.scatter_fill(a2, torch.from_numpy(sel).to(dev), 0.0)
    codec.wavedec(tx, level, x0=tx0, want_x=False, coeffs_diff=a2, accumulate=True,
                  wavelet=wavelet)
    got = a1.cpu().numpy()
    np.testing.assert_array_equal(_bits(got), _bits(a2.cpu().numpy()))
    if n <= 1_000_003:
        want = acc.copy()
        want[sel] = 0.0
        want = (want + owav.wavedec_array((x - x0).astype(np.float32), level, wavelet)
                ).astype(np.float32)
        np.testing.assert_array_equal(_bits(got), _bits(want))


def test_sliced_rejects_bad_arguments(dev):
    from decentralizepy_amd import codec
    n = 300_000
    x = torch.randn(n, device=dev)
    acc = torch.randn(n, device=dev)
    mask = torch.empty(codec.mask_words(n), dtype=torch.int32, device=dev)
    with pytest.raises(Exception):  # ACCUMULATE writes acc: not a sliced mode
        codec.topk_encode_sliced(x, 3000, mask, acc=acc, acc_mode=codec.DPZ_ACC_ACCUMULATE)
    with pytest.raises(Exception):  # mask too small
        codec.topk_encode_sliced(x, 3000, mask[:-1])
    with pytest.raises(Exception):  # rewind mask on a non-accumulating pass
        codec.wavedec(x, 4, x0=acc, rewind_mask=mask)


@pytest.mark.parametrize("status", [False, True])
def test_sliced_long_segments_build_the_mask_after_compact(dev, diag_lib, monkeypatch, status):
    """Segments longer than the LDS rows hold (SL_RMAX; n > 67 M at the full grid, forced here
    with the diagnostic build's DPZ_WLONE): compact writes idx / val only and the mask and the
    planes are built from idx_out after it; after a sampled miss the planes stay untouched until
    the exact re-run (blocking and asynchronous)."""
    monkeypatch.setenv("DPZ_WLONE", "64")
    n = 1_000_003
    x, x0, acc = _inputs(n, seed=21)
    _run(dev, x - x0, None, acc, otopk.ACC_ADD, round(0.1 * n), vals=x, status=status)
    from tests.layouts import miss_layout
    n = 1 << 20
    k = round(0.01 * n)
    x, x0 = miss_layout(n, k)
    _run(dev, x, x0, None, otopk.ACC_NONE, k, status=status)
    # the mask build after compact must not follow the stale indices of a missed sampled run
    _run(dev, x, x0, None, otopk.ACC_NONE, k, status=status, poison=True)
