"""GPU: the device steps of the sharded top-k (decentralizepy_amd/shard.py) — per-shard candidate
selection, the merge over the concatenated candidates and the per-shard counter update — emulate
a world-size-G run in one process (the all-gather replaced by a concatenation) and must equal the
one-tensor encode bit-exactly, at the C5 shape (N = 2^26, alpha = 0.001, 8 shards) and with
ties straddling shard boundaries."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,alpha,world,ties", [(67_108_864, 0.001, 8, False),
                                                (3_000_000, 0.01, 3, True),
                                                (1_000_000, 0.1, 2, False)])
def test_sharded_steps_equal_whole_tensor_encode(dev, n, alpha, world, ties):
    """the per-rank steps, emulated in one process"""
    from decentralizepy_amd import codec
    from decentralizepy_amd.shard import HipShardOps
    g = torch.Generator(device=dev).manual_seed(11)
    x = torch.randn(n, device=dev, generator=g)
    x0 = x - 0.01 * torch.randn(n, device=dev, generator=g)
    if ties:
        x0 = x - torch.round((x - x0) * 300) / 300
    k = round(alpha * n)
    cnt_ref = torch.zeros(n, dtype=torch.int32, device=dev)
    ref_idx, ref_val = codec.topk_encode(x, k, x0=x0, counter=cnt_ref)
    ops = HipShardOps(dev)
    bounds = np.linspace(0, n, world + 1).astype(int)
    cands = []
    for lo, hi in zip(bounds[:-1], bounds[1:]):
        c = ops.local_candidates(x[lo:hi], x0[lo:hi], k, int(lo))
        if int(ops.local_status().item()) != 0:  # sampled-path miss (heavy ties): exact re-run
            assert ties
            c = ops.local_candidates(x[lo:hi], x0[lo:hi], k, int(lo), exact=True)
        cands.append(c)
    gidx = torch.cat([c[0] for c in cands])
    gchg = torch.cat([c[1] for c in cands])
    gval = torch.cat([c[2] for c in cands])
    widx, wval = ops.merge(gidx, gchg, gval, k)
    if int(ops.merge_status().item()) != 0:
        assert ties
        widx, wval = ops.merge(gidx, gchg, gval, k, exact=True)
    cnt = torch.zeros(n, dtype=torch.int32, device=dev)
    for lo, hi in zip(bounds[:-1], bounds[1:]):
        ops.count(cnt[lo:hi], widx, int(lo))
    torch.cuda.synchronize()
    assert torch.equal(widx, ref_idx)
    assert torch.equal(wval.view(torch.int32), ref_val.view(torch.int32))
    assert torch.equal(cnt, cnt_ref)


def test_sharded_topk_encode_one_rank_api(dev):
    """the public entry on one rank (no process group): the whole tensor's payload + counter"""
    from decentralizepy_amd import codec
    from decentralizepy_amd.shard import sharded_topk_encode
    n, k = 2_000_003, 20_000
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(n, device=dev, generator=g)
    x0 = x - 0.01 * torch.randn(n, device=dev, generator=g)
    cnt_ref = torch.zeros(n, dtype=torch.int32, device=dev)
    ref_idx, ref_val = codec.topk_encode(x, k, x0=x0, counter=cnt_ref)
    cnt = torch.zeros(n, dtype=torch.int32, device=dev)
    idx, val = sharded_topk_encode(x, x0, k, 0, counter=cnt)
    assert torch.equal(idx, ref_idx) and torch.equal(val, ref_val) and torch.equal(cnt, cnt_ref)


@pytest.mark.parametrize("n,world", [(1_000_003, 2), (1_000_003, 3), (25_000_000, 8),
                                     (100_000, 5), (16_484, 4), (28_572, 8)])
def test_sharded_wavelet_equals_whole_tensor(dev, n, world):
    """SURVEY §8e wavelet row: per-rank forward tiles from halo'd slice buffers (the halo being
    the previous slice's tail) and per-rank inverse tiles, emulated in one process, equal the
    one-GPU transforms bit-exactly (plain and accumulate)."""
    from decentralizepy_amd import codec
    from decentralizepy_amd.shard import (dwt_rank_part, halo_len, idwt_rank_part,
                                          tile_widths, wavelet_slice)
    level = 4
    g = torch.Generator(device=dev).manual_seed(n + world)
    x = torch.randn(n, device=dev, generator=g)
    x0 = x - 0.01 * torch.randn(n, device=dev, generator=g)
    ref_x, ref_d = codec.wavedec(x, level, x0=x0)
    m = ref_x.numel()
    acc0 = 0.01 * torch.randn(m, device=dev, generator=g)
    ref_acc = acc0.clone()
    codec.wavedec(x, level, x0=x0, want_x=False, coeffs_diff=ref_acc, accumulate=True)
    cx = torch.full((m,), float("nan"), device=dev)
    cd = torch.full((m,), float("nan"), device=dev)
    acc = acc0.clone()
    H = halo_len(level)
    rec = torch.full((n,), float("nan"), device=dev)
    for r in range(world):
        sl = wavelet_slice(n, level, world, r, *tile_widths())
        first = max(0, sl["lo"] - H) if r > 0 else 0
        # the rank's buffer: a COPY of its halo + slice (nothing else of x is reachable)
        xb = x[first:sl["hi"]].clone()
        x0b = x0[first:sl["hi"]].clone()
        if sl["t_lo"] < sl["t_hi"]:
            assert sl["lo"] < sl["hi"], "an empty slice must own no forward tile"
            dwt_rank_part(xb, x0b, first, n, level, sl["t_lo"], sl["t_hi"], cx, cd)
            dwt_rank_part(xb, x0b, first, n, level, sl["t_lo"], sl["t_hi"], None, acc,
                          accumulate=True)
        out = torch.empty(sl["hi"] - sl["lo"], device=dev)
        if out.numel():
            idwt_rank_part(ref_x, n, level, sl["u_lo"], sl["u_hi"], out, sl["lo"])
            rec[sl["lo"]:sl["hi"]] = out
    torch.cuda.synchronize()
    assert torch.equal(cx.view(torch.int32), ref_x.view(torch.int32))
    assert torch.equal(cd.view(torch.int32), ref_d.view(torch.int32))
    assert torch.equal(acc.view(torch.int32), ref_acc.view(torch.int32))
    ref_rec = codec.waverec(ref_x, n, level)
    assert torch.equal(rec.view(torch.int32), ref_rec.view(torch.int32))


def test_sharded_wavelet_one_rank_api(dev):
    from decentralizepy_amd import codec
    from decentralizepy_amd.shard import sharded_wavedec, sharded_waverec
    n = 3_000_017
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(n, device=dev, generator=g)
    x0 = x - 0.01 * torch.randn(n, device=dev, generator=g)
    ref_x, ref_d = codec.wavedec(x, 4, x0=x0)
    cx, cd = sharded_wavedec(x, x0, n, 4)
    assert torch.equal(cx, ref_x) and torch.equal(cd, ref_d)
    assert torch.equal(sharded_waverec(cx, n, 4), codec.waverec(ref_x, n, 4))


def test_sharded_wavedec_headroom_slices(dev):
    """Slices from alloc_wavelet_slice get the halo written into their own headroom (no copy of
    the slice); the result equals the one-GPU transform (one rank: no exchange needed)."""
    from decentralizepy_amd import codec
    from decentralizepy_amd.shard import alloc_wavelet_slice, sharded_wavedec
    n = 2_000_003
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(n, device=dev, generator=g)
    x0 = x - 0.01 * torch.randn(n, device=dev, generator=g)
    xs = alloc_wavelet_slice(n, 4, 1, 0, dev)
    x0s = alloc_wavelet_slice(n, 4, 1, 0, dev)
    xs.copy_(x)
    x0s.copy_(x0)
    cx, cd = sharded_wavedec(xs, x0s, n, 4)
    rx, rd = codec.wavedec(x, 4, x0=x0)
    assert torch.equal(cx, rx) and torch.equal(cd, rd)


@pytest.mark.parametrize("n,world,alpha", [(1_000_003, 3, 0.01), (4_000_000, 8, 0.001),
                                           (100_001, 5, 0.3)])
def test_sharded_replace_equals_whole_tensor(dev, n, world, alpha):
    """SURVEY §8e "one tensor, decode": every rank replaces the GLOBAL payload into its own slice
    (most entries fall outside it, some slices hold none); the slices assemble the one-GPU
    replace bit-exactly."""
    from decentralizepy_amd import codec
    from decentralizepy_amd.shard import sharded_replace
    g = torch.Generator(device=dev).manual_seed(n + world)
    x = torch.randn(n, device=dev, generator=g)
    x0 = x - 0.01 * torch.randn(n, device=dev, generator=g)
    k = round(alpha * n)
    idx, val = codec.topk_encode(x, k, x0=x0)
    ref = codec.replace(x0, idx, val)
    bounds = [0, 3, n // 3] + [n // 3 + (j * (n - n // 3)) // (world - 2) for j in range(1, world - 2)] + [n]
    bounds = sorted(set(bounds))
    rec = torch.full((n,), float("nan"), device=dev)
    for lo, hi in zip(bounds[:-1], bounds[1:]):
        loc = x0[lo:hi].clone()  # the rank's own (aligned) slice buffer
        rec[lo:hi] = sharded_replace(loc, lo, idx, val)
    # a slice no payload entry falls into
    empty_lo = int(idx[0].item()) - 2 if int(idx[0].item()) >= 2 else None
    torch.cuda.synchronize()
    assert torch.equal(rec.view(torch.int32), ref.view(torch.int32))
    if empty_lo is not None:
        loc = x0[:empty_lo].clone()
        assert torch.equal(sharded_replace(loc, 0, idx, val), loc)


@pytest.mark.parametrize("n,alpha,world", [(67_108_864, 0.001, 8), (3_000_001, 0.01, 3)])
def test_sharded_fp16_values_written_by_the_encode(dev, n, alpha, world):
    """BASELINE config 5 as named: the sharded one-tensor encode whose values are packed to fp16
    by the local encodes themselves (DPZ_TOPK_VAL_FP16, no pack_fp16 launch) and carried as fp16
    through the merge: equal to the oracle's top-k with the reference rule and torch.half values
    (round to nearest even)."""
    from decentralizepy_amd import codec
    from decentralizepy_amd.shard import HipShardOps
    from oracle import topk as otopk
    g = torch.Generator(device=dev).manual_seed(23)
    x = torch.randn(n, device=dev, generator=g)
    x0 = x - 0.01 * torch.randn(n, device=dev, generator=g)
    k = round(alpha * n)
    o_cnt = np.zeros(n, dtype=np.int32)
    oi, ov = otopk.encode(x.cpu().numpy(), x0.cpu().numpy(), None, 0, k, counter=o_cnt)
    want_h = ov.astype(np.float16)  # RNE, as torch.Tensor.half()
    # the one-tensor encode with fp16 values
    cnt1 = torch.zeros(n, dtype=torch.int32, device=dev)
    i1, v1 = codec.topk_encode(x, k, x0=x0, counter=cnt1, val_fp16=True)
    assert v1.dtype == torch.float16
    np.testing.assert_array_equal(i1.cpu().numpy(), oi)
    np.testing.assert_array_equal(v1.cpu().numpy().view(np.uint16), want_h.view(np.uint16))
    np.testing.assert_array_equal(cnt1.cpu().numpy(), o_cnt)
    # the sharded steps, emulated in one process
    ops = HipShardOps(dev)
    bounds = np.linspace(0, n, world + 1).astype(int)
    cands = [ops.local_candidates(x[lo:hi], x0[lo:hi], k, int(lo), val_fp16=True)
             for lo, hi in zip(bounds[:-1], bounds[1:])]
    widx, wval = ops.merge(torch.cat([c[0] for c in cands]), torch.cat([c[1] for c in cands]),
                           torch.cat([c[2] for c in cands]), k)
    assert int(ops.merge_status().item()) == 0
    np.testing.assert_array_equal(widx.cpu().numpy(), oi)
    np.testing.assert_array_equal(wval.cpu().numpy().view(np.uint16), want_h.view(np.uint16))


@pytest.mark.parametrize("n,k", [(100_000, 1_000), (1_000_000, 600_000)])
def test_fp16_values_on_the_exact_path(dev, n, k):
    """small n / dense alpha take the exact path: the same fp16 values; overflow to inf and NaN
    keep torch.half semantics"""
    from decentralizepy_amd import codec
    from oracle import topk as otopk
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n).astype(np.float32) * 1e3
    x[:5] = [7e4, -7e4, np.inf, np.nan, 65519.0]  # overflow, inf, NaN, rounds up to inf
    x0 = (x - rng.standard_normal(n).astype(np.float32)).astype(np.float32)
    x0[:5] = 0.0
    oi, ov = otopk.encode(x, x0, None, 0, k)
    i, v = codec.topk_encode(torch.from_numpy(x).to(dev), k, x0=torch.from_numpy(x0).to(dev),
                             val_fp16=True)
    np.testing.assert_array_equal(i.cpu().numpy(), oi)
    np.testing.assert_array_equal(v.cpu().numpy().view(np.uint16),
                                  ov.astype(np.float16).view(np.uint16))
    ref_t = torch.from_numpy(ov).half().numpy()
    np.testing.assert_array_equal(v.cpu().numpy().view(np.uint16), ref_t.view(np.uint16))
