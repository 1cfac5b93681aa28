"""CPU (gloo, world_size 2 and 3): the sharded top-k protocol (decentralizepy_amd/shard.py) with
the oracle standing in for the HIP steps gives exactly the one-tensor encode of the reference rule
(k largest |x - x0|, lowest-index ties), payload and counter, on every rank — including ties that
straddle the shard boundary.  The device steps are covered by tests/test_gpu_shard.py."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import topk as otopk


class OracleOps:
    def local_candidates(self, x, x0, k, offset, exact=False, val_fp16=False):
        idx, val = otopk.encode(x.numpy(), x0.numpy(), None, otopk.ACC_NONE, k)
        chg = (x.numpy() - x0.numpy())[idx]
        if val_fp16:  # the encode's own RNE packing (torch.half)
            val = val.astype(np.float16)
        return (torch.from_numpy(idx.astype(np.int32)) + int(offset), torch.from_numpy(chg),
                torch.from_numpy(val))

    def merge(self, gidx, gchg, gval, k, exact=False):
        pos = otopk.topk_select(otopk.keys_u32(gchg.numpy()), k)
        return gidx[torch.from_numpy(pos)], gval[torch.from_numpy(pos)]

    def count(self, counter, idx, offset):
        i = idx.long() - offset
        i = i[(i >= 0) & (i < counter.numel())]
        counter.index_add_(0, i, torch.ones_like(i, dtype=torch.int32))

    def replace_slice(self, local_slice, offset, idx, vals, out):
        from oracle import fold as ofold
        i = idx.numpy().astype(np.int64) - offset
        inside = (i >= 0) & (i < local_slice.numel())
        out.copy_(torch.from_numpy(ofold.replace(local_slice.numpy(), i[inside],
                                                 vals.numpy()[inside])))


def _inputs(n, ties):
    g = torch.Generator().manual_seed(7)
    x = torch.randn(n, generator=g)
    x0 = x - 0.01 * torch.randn(n, generator=g)
    if ties:
        d = torch.round((x - x0) * 300) / 300  # heavy ties at the k-th key
        x0 = x - d
    return x, x0


def _worker(rank, world, port, n, k, ties, out_q, fp16=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from decentralizepy_amd.shard import sharded_topk_encode
        x, x0 = _inputs(n, ties)
        bounds = np.linspace(0, n, world + 1).astype(int)
        lo, hi = int(bounds[rank]), int(bounds[rank + 1])
        cnt = torch.zeros(hi - lo, dtype=torch.int32)
        from decentralizepy_amd.shard import sharded_replace
        ops = OracleOps()
        idx, val = sharded_topk_encode(x[lo:hi].contiguous(), x0[lo:hi].contiguous(), k, lo,
                                       counter=cnt, ops=ops, val_fp16=fp16)
        if fp16:
            out_q.put((rank, idx.numpy(), val.numpy(), lo, cnt.numpy(), None))
            return
        # decode of the global payload into this rank's slice: most entries lie outside it
        dec = sharded_replace(x0[lo:hi].contiguous(), lo, idx, val, ops=ops)
        out_q.put((rank, idx.numpy(), val.numpy(), lo, cnt.numpy(), dec.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,ties", [(2, False), (2, True), (3, True)])
def test_sharded_topk_equals_whole_tensor_encode(world, ties):
    n, k = 30_000, 1_500
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29650 + world * 2 + int(ties)
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, k, ties, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    x, x0 = _inputs(n, ties)
    o_cnt = np.zeros(n, dtype=np.int32)
    oi, ov = otopk.encode(x.numpy(), x0.numpy(), None, otopk.ACC_NONE, k, counter=o_cnt)
    full_cnt = np.zeros(n, dtype=np.int32)
    full_dec = np.full(n, np.nan, dtype=np.float32)
    for rank, idx, val, lo, cnt, dec in res:
        np.testing.assert_array_equal(idx, oi)
        np.testing.assert_array_equal(val.view(np.uint32), ov.view(np.uint32))
        full_cnt[lo:lo + cnt.shape[0]] = cnt
        full_dec[lo:lo + dec.shape[0]] = dec
    np.testing.assert_array_equal(full_cnt, o_cnt)
    # the slices' decodes assemble the whole-tensor decode (SURVEY §8e "one tensor, decode")
    from oracle import fold as ofold
    ref = ofold.replace(x0.numpy(), oi, ov)
    np.testing.assert_array_equal(full_dec.view(np.uint32), ref.view(np.uint32))


# ---------------------------------------------------------------------------------------------
# sharded wavelet: halo exchange + owned-range all-gather over gloo, the per-rank
# forward tiles emulated with the oracle on a NaN-padded copy of the rank's halo'd buffer (any
# input a rank's owned coefficients need but it does not hold turns them into NaN)

def _fake_dwt_rank_part(xb, x0b, first, n, level, t_lo, t_hi, cx, cd, accumulate=False):
    from oracle import wavelet as owav
    from decentralizepy_amd.shard import owned_coeff_ranges
    full = np.full(n, np.nan, dtype=np.float32)
    full0 = np.full(n, np.nan, dtype=np.float32)
    full[first:first + xb.numel()] = xb.numpy()
    full0[first:first + x0b.numel()] = x0b.numpy()
    wx = owav.wavedec_array(full, level)
    wd = owav.wavedec_array(full - full0, level)
    for s, e in owned_coeff_ranges(n, level, t_lo, t_hi, _DW):
        if cx is not None:
            cx[s:e] = torch.from_numpy(wx[s:e])
        if cd is not None:
            cd[s:e] = (cd[s:e] + torch.from_numpy(wd[s:e])) if accumulate else torch.from_numpy(wd[s:e])


# the built kernels' tile widths (the library loads without a GPU; its host entry points run)
_DW, _IW = 128, 4096


def _wavelet_worker(rank, world, port, n, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from decentralizepy_amd import shard
        shard.dwt_rank_part = _fake_dwt_rank_part
        shard._DEVICE_ONLY = False
        assert shard.tile_widths() == (_DW, _IW)
        g = torch.Generator().manual_seed(n)
        x = torch.randn(n, generator=g)
        x0 = x - 0.01 * torch.randn(n, generator=g)
        sl = shard.wavelet_slice(n, 4, world, rank, _DW, _IW)
        cx, cd = shard.sharded_wavedec(x[sl["lo"]:sl["hi"]].contiguous(),
                                       x0[sl["lo"]:sl["hi"]].contiguous(), n, 4)
        out_q.put((rank, cx.numpy(), cd.numpy()))
    except Exception as e:  # surface the failure instead of a queue timeout
        out_q.put((rank, repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 100_003), (3, 100_003), (4, 16_484)])
def test_sharded_wavedec_exchange(world, n):
    """(4, 16484): ranks 2 and 3 hold empty slices (5 inverse tiles over 4 ranks at 2 each), so
    the tail forward tiles belong to rank 2's predecessor, the slice holding element n - 1."""
    from oracle import wavelet as owav
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29710 + world
    procs = [ctx.Process(target=_wavelet_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    g = torch.Generator().manual_seed(n)
    x = torch.randn(n, generator=g)
    x0 = x - 0.01 * torch.randn(n, generator=g)
    ref_x = owav.wavedec_array(x.numpy(), 4)
    ref_d = owav.wavedec_array(x.numpy() - x0.numpy(), 4)
    for rank, cx, cd in res:
        assert cd is not None, f"rank {rank} failed: {cx}"
        np.testing.assert_array_equal(cx.view(np.uint32), ref_x.view(np.uint32))
        np.testing.assert_array_equal(cd.view(np.uint32), ref_d.view(np.uint32))


@pytest.mark.parametrize("n,world", [(16_484, 4), (28_572, 8), (100_003, 3), (4096 * 7, 8),
                                     (1_000_003, 8), (33, 2)])
def test_wavelet_slices_partition_tiles_and_coefficients(n, world):
    """Every forward tile, inverse tile and coefficient is owned by exactly one rank, and a rank's
    forward tiles read only inputs inside its slice plus the left halo (the ADVICE r1 case:
    empty last slices must not be handed the tail tiles)."""
    from decentralizepy_amd.shard import (_level_lengths, halo_len, owned_coeff_ranges,
                                          wavelet_slice)
    from oracle import wavelet as owav
    level = 4
    lens = _level_lengths(n, level)
    n_fwd = -(-lens[level] // _DW)
    m = len(owav.wavedec_array(np.zeros(n, dtype=np.float32), level))
    fwd = np.zeros(n_fwd, dtype=int)
    inv = np.zeros(-(-n // _IW), dtype=int)
    cov = np.zeros(m, dtype=int)
    H = halo_len(level)
    span = (1 << level) * _DW
    for r in range(world):
        sl = wavelet_slice(n, level, world, r, _DW, _IW)
        fwd[sl["t_lo"]:sl["t_hi"]] += 1
        inv[sl["u_lo"]:sl["u_hi"]] += 1
        for s, e in owned_coeff_ranges(n, level, sl["t_lo"], sl["t_hi"], _DW):
            cov[s:e] += 1
        if sl["t_lo"] < sl["t_hi"]:
            # inputs the tiles read: [span * t_lo - 2 (2^L - 1), min(n, span * t_hi))
            assert max(0, span * sl["t_lo"] - 2 * ((1 << level) - 1)) >= max(0, sl["lo"] - H)
            assert sl["hi"] == n or span * sl["t_hi"] <= sl["hi"]
            assert sl["lo"] < sl["hi"]
    assert (fwd == 1).all() and (inv == 1).all() and (cov == 1).all()


@pytest.mark.parametrize("world,k", [(2, 1_500), (3, 1_500), (2, 1_501)])
def test_sharded_topk_fp16_values(world, k):
    """BASELINE config 5: fp16 values (RNE) packed by the local encodes travel through the one
    all-gather (10 bytes per candidate) and the merge: the whole-tensor payload with torch.half
    values on every rank.  Odd k: the value section is padded to 4 bytes in the packed row."""
    n = 30_000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29690 + world + (k % 2) * 5
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, k, True, q, True))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    x, x0 = _inputs(n, True)
    oi, ov = otopk.encode(x.numpy(), x0.numpy(), None, otopk.ACC_NONE, k)
    for rank, idx, val, lo, cnt, _ in res:
        assert val.dtype == np.float16
        np.testing.assert_array_equal(idx, oi)
        np.testing.assert_array_equal(val.view(np.uint16),
                                      torch.from_numpy(ov).half().numpy().view(np.uint16))
