"""GPU: the prior-round key window (DPZ_TOPK_HINT: the filter's window from the previous encode's
exact threshold on the workspace, no sample launch) and the keep-x cache policy
(DPZ_TOPK_KEEP_X) leave every result of the reference's top-k encode unchanged
(sharing/PartialModel.py:164-255): index sets, values and the shared-parameter counter are
bit-exact against the oracle over a node's consecutive rounds, and a window that no longer
brackets the k-th key (a jump in the change distribution, a prior of another size) is a miss
that the blocking call / dpz_topk_complete recovers on the sampled path."""
import numpy as np
import pytest
import torch

from oracle import topk as otopk

pytestmark = pytest.mark.gpu

# TopkCtrl word offsets (csrc/dpz_topk.h)
_STATUS, _STICKY, _HINT_T, _HINT_SIG, _HINTED = 2, 11, 13, 14, 15


def _ctrl(ws):
    torch.cuda.synchronize()
    return ws.buf[:256].view(torch.int32).cpu().numpy().view(np.uint32)


def _inputs(n, seed, scale):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, generator=g)
    x0 = x - scale * torch.randn(n, generator=g)
    return x.numpy(), x0.numpy()


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def _round(dev, ws, x, x0, k, tcnt, o_cnt, **kw):
    from decentralizepy_amd import codec
    idx, val = codec.topk_encode(torch.from_numpy(x).to(dev), k, x0=torch.from_numpy(x0).to(dev),
                                 counter=tcnt, workspace=ws, **kw)
    oi, ov = otopk.encode(x, x0, None, otopk.ACC_NONE, k, counter=o_cnt)
    np.testing.assert_array_equal(idx.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(val.cpu().numpy()), _bits(ov))
    np.testing.assert_array_equal(tcnt.cpu().numpy(), o_cnt)


@pytest.mark.parametrize("n,alpha", [(1_000_003, 0.01), (16_777_216, 0.01), (2_000_000, 0.05)])
def test_hinted_rounds_match_oracle(dev, n, alpha):
    """A node's rounds with a slowly drifting change scale: from round 1 on the window is the
    prior one (no sample launch: ctrl.hinted), every round bit-exact; keep_x alternates."""
    from decentralizepy_amd import codec
    k = round(alpha * n)
    ws = codec.Workspace(dev)
    tcnt = torch.zeros(n, dtype=torch.int32, device=dev)
    o_cnt = np.zeros(n, dtype=np.int32)
    for r in range(4):
        x, x0 = _inputs(n, 100 + r, 0.01 * (1.0 + 0.04 * r))
        _round(dev, ws, x, x0, k, tcnt, o_cnt, hint=True, keep_x=bool(r % 2))
        c = _ctrl(ws)
        assert c[_STATUS] == 0 and c[_HINTED] == (1 if r else 0)
        assert c[_HINT_SIG] != 0
    assert codec.topk_sticky_status(ws) == 0


def test_hint_miss_blocking_recovers_on_sampled_path(dev):
    """The change scale doubles between rounds: the prior window misses, the blocking call
    re-runs the sampled path (its sample launch resets ctrl.hinted) and the result is exact;
    the miss shows in the sticky status word."""
    from decentralizepy_amd import codec
    n, k = 1_000_003, 10_000
    ws = codec.Workspace(dev)
    tcnt = torch.zeros(n, dtype=torch.int32, device=dev)
    o_cnt = np.zeros(n, dtype=np.int32)
    for r, scale in enumerate((0.01, 0.02, 0.02)):
        x, x0 = _inputs(n, 200 + r, scale)
        _round(dev, ws, x, x0, k, tcnt, o_cnt, hint=True)
        c = _ctrl(ws)
        assert c[_STATUS] == 0
        if r == 1:
            assert c[_HINTED] == 0  # re-run with the sample launch
            assert codec.topk_sticky_status(ws, clear=True) != 0
        if r == 2:
            assert c[_HINTED] == 1  # the re-run's threshold is the new prior
            assert codec.topk_sticky_status(ws) == 0


def test_hint_miss_asynchronous_then_complete(dev):
    """An asynchronous hinted call that misses wrote nothing and reports it; dpz_topk_complete
    re-runs it (sampled path) to the exact result."""
    from decentralizepy_amd import codec
    n, k = 1_000_003, 10_000
    ws = codec.Workspace(dev)
    x, x0 = _inputs(n, 300, 0.01)
    tcnt = torch.zeros(n, dtype=torch.int32, device=dev)
    o_cnt = np.zeros(n, dtype=np.int32)
    _round(dev, ws, x, x0, k, tcnt, o_cnt, hint=True)
    x, x0 = _inputs(n, 301, 0.005)  # the k-th key halves: below the window
    tx, tx0 = torch.from_numpy(x).to(dev), torch.from_numpy(x0).to(dev)
    idx = torch.full((k,), -7, dtype=torch.int32, device=dev)
    val = torch.empty(k, device=dev)
    codec.topk_encode(tx, k, x0=tx0, counter=tcnt, idx_out=idx, val_out=val, workspace=ws,
                      asynchronous=True, hint=True)
    assert _ctrl(ws)[_STATUS] != 0
    assert (idx.cpu().numpy() == -7).all()  # a miss writes nothing
    np.testing.assert_array_equal(tcnt.cpu().numpy(), o_cnt)  # and counts nothing
    assert codec.topk_complete(tx, k, idx, val, ws, x0=tx0, counter=tcnt)
    oi, ov = otopk.encode(x, x0, None, otopk.ACC_NONE, k, counter=o_cnt)
    np.testing.assert_array_equal(idx.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(val.cpu().numpy()), _bits(ov))
    np.testing.assert_array_equal(tcnt.cpu().numpy(), o_cnt)


def test_hint_from_another_signature_is_a_miss(dev):
    """A prior of another k on the same workspace (the flag forced past the Python check): the
    device signature does not match, the call misses at once and is re-run, exact."""
    from decentralizepy_amd import codec
    n = 1_000_003
    ws = codec.Workspace(dev)
    big = int(codec._lib.lib().dpz_topk_workspace_bytes(n, 20_000))
    ws.buf = torch.zeros(big, dtype=torch.uint8, device=dev)  # room for both k
    tcnt = torch.zeros(n, dtype=torch.int32, device=dev)
    o_cnt = np.zeros(n, dtype=np.int32)
    x, x0 = _inputs(n, 400, 0.01)
    _round(dev, ws, x, x0, 20_000, tcnt, o_cnt, hint=True)
    ws.hint_key = (n, 10_000, False, 0, True)  # pretend the prior was a k = 10,000 call
    _round(dev, ws, x, x0, 10_000, tcnt, o_cnt, hint=True)
    assert codec.topk_sticky_status(ws, clear=True) != 0  # it missed, then recovered


def test_hint_with_fold_base_and_fp16(dev):
    """The prior window under the fold-base encode (PartialModel's one-neighbour path) and the
    fp16 value format: results equal the non-hinted encode's."""
    from decentralizepy_amd import codec
    n, k = 2_000_003, 20_000
    x, x0 = _inputs(n, 500, 0.01)
    tx, tx0 = torch.from_numpy(x).to(dev), torch.from_numpy(x0).to(dev)
    outs = []
    for hint in (False, True):
        ws = codec.Workspace(dev)
        for _ in range(2):  # the second call takes the prior window when hint is set
            base = torch.empty(n, device=dev)
            i1, v1 = codec.topk_encode(tx, k, x0=tx0, workspace=ws, hint=hint, keep_x=True,
                                       fold_base=(base, [0.25, 0.25], 0.5))
            i2, v2 = codec.topk_encode(tx, k, x0=tx0, workspace=ws, hint=hint, val_fp16=True)
        assert _ctrl(ws)[_HINTED] == (1 if hint else 0)
        outs.append([t.cpu().numpy().copy() for t in (i1, v1, base, i2, v2)])
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a.view(np.uint8), b.view(np.uint8))


@pytest.mark.parametrize("alpha,blocking", [(0.01, True), (0.1, False)])
def test_hinted_sliced_rounds_match_oracle(dev, alpha, blocking):
    """The JWINS encode in coalesced form (dpz_topk_encode_sliced: keys |W(x - x0) + acc|, values
    W(x), the counter as bit planes, the selection mask) over a node's rounds with the prior
    window: rounds 1-2 hinted (no sample launch), round 3 doubles the change scale (the window
    misses: a blocking call runs the sampled path again, an asynchronous one reports the miss,
    wrote nothing, and is re-run exactly), round 4 hinted again — every round's index set,
    values, counter and mask bit-exact against the oracle."""
    from decentralizepy_amd import codec
    n = 2_000_003
    k = round(alpha * n)
    ws = codec.Workspace(dev)
    planes = codec.counter_slice(torch.zeros(n, dtype=torch.int32, device=dev))
    nw = codec.mask_words(n)
    mask = torch.zeros(nw, dtype=torch.int32, device=dev)
    o_cnt = np.zeros(n, dtype=np.int32)
    rng = np.random.default_rng(11)
    for r, scale in enumerate((0.01, 0.0104, 0.0108, 0.0216, 0.022)):
        wx = rng.standard_normal(n).astype(np.float32)
        wc = (scale * rng.standard_normal(n)).astype(np.float32)
        acc = (0.5 * scale * rng.standard_normal(n)).astype(np.float32)
        t = [torch.from_numpy(a).to(dev) for a in (wx, wc, acc)]
        st = None if blocking else torch.full((1,), 7, dtype=torch.int32, device=dev)
        io = torch.full((k,), 0x7FFFFFF0, dtype=torch.int32, device=dev)
        idx, val = codec.topk_encode_sliced(t[1], k, mask, planes, acc=t[2],
                                            acc_mode=codec.DPZ_ACC_ADD, vals_src=t[0],
                                            idx_out=io, workspace=ws, status_out=st, hint=True)
        c = _ctrl(ws)
        # (an exact re-run leaves no prior: the asynchronous caller's next round samples again)
        if r in (1, 2) or (r == 4 and blocking):
            assert c[_HINTED] == 1 and c[_STATUS] == 0
        if r == 3:
            if blocking:
                assert c[_HINTED] == 0 and codec.topk_sticky_status(ws, clear=True) != 0
            else:
                assert int(st.item()) != 0 and c[_HINTED] == 1
                assert (io.cpu().numpy() == 0x7FFFFFF0).all()  # a miss writes nothing
                codec.topk_sticky_status(ws, clear=True)
                idx, val = codec.topk_encode_sliced(t[1], k, mask, planes, acc=t[2],
                                                    acc_mode=codec.DPZ_ACC_ADD, vals_src=t[0],
                                                    idx_out=io, workspace=ws, exact=True)
        oi, ov = otopk.encode(wc, None, acc.copy(), otopk.ACC_ADD, k, vals_src=wx, counter=o_cnt)
        np.testing.assert_array_equal(idx.cpu().numpy(), oi)
        np.testing.assert_array_equal(_bits(val.cpu().numpy()), _bits(ov))
        np.testing.assert_array_equal(codec.counter_unslice(planes, n).cpu().numpy(), o_cnt)
        words = np.zeros(nw, dtype=np.uint32)
        np.bitwise_or.at(words, oi >> 5, (np.uint32(1) << (oi & 31).astype(np.uint32)))
        np.testing.assert_array_equal(mask.cpu().numpy().view(np.uint32), words)


@pytest.mark.parametrize("what", ["fold_base", "co_replace"])
def test_unusable_prior_still_writes_the_copy(dev, what):
    """A hinted call whose prior window is unusable (here: a prior of another k, the flag forced
    past the Python check) misses at once and is re-run by the blocking call — which encodes
    only.  The copy the missed filter owed is written all the same: the fold's no-hit base
    (dpz_topk_encode_foldbase, PartialModel's one-neighbour fold) and the fused replace decode's
    out = x (dpz_topk_encode_replace, whose payload entries the compact launch still scatters):
    reference Sharing.py:156-190 / PartialModel.py:257-303 over the node's own model."""
    from decentralizepy_amd import codec
    n, k = 1_000_003, 10_000
    ws = codec.Workspace(dev)
    big = int(codec._lib.lib().dpz_topk_workspace_bytes(n, 20_000))
    ws.buf = torch.zeros(big, dtype=torch.uint8, device=dev)
    x, x0 = _inputs(n, 600, 0.01)
    tx, tx0 = torch.from_numpy(x).to(dev), torch.from_numpy(x0).to(dev)
    codec.topk_encode(tx, 20_000, x0=tx0, workspace=ws, hint=True)  # the prior: another k
    codec.topk_sticky_status(ws, clear=True)
    ws.hint_key = (n, k, False, 0, True)  # the flag is passed; the device signature differs
    if what == "fold_base":
        out = torch.full((n,), float("nan"), device=dev)
        i, v = codec.topk_encode(tx, k, x0=tx0, workspace=ws, hint=True, keep_x=True,
                                 fold_base=(out, [0.25, 0.25], 0.5))
        q = np.float32(0.25)
        ref = ((x * q) + (x * q)) + (x * np.float32(0.5))  # fp32, one rounding per op
    else:
        rng = np.random.default_rng(601)
        ri = np.sort(rng.choice(n, size=5_000, replace=False)).astype(np.int32)
        rv = rng.standard_normal(5_000).astype(np.float32)
        out = torch.full((n,), float("nan"), device=dev)
        i, v = codec.topk_encode(tx, k, x0=tx0, workspace=ws, hint=True,
                                 co_replace=(tx, torch.from_numpy(ri).to(dev),
                                             torch.from_numpy(rv).to(dev), out))
        ref = x.copy()
        ref[ri] = rv
    assert codec.topk_sticky_status(ws, clear=True) != 0  # the hinted call did miss
    np.testing.assert_array_equal(_bits(out.cpu().numpy()), _bits(ref))
    oi, ov = otopk.encode(x, x0, None, otopk.ACC_NONE, k)
    np.testing.assert_array_equal(i.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(v.cpu().numpy()), _bits(ov))
