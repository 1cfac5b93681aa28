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
    def local_candidates(self, x, x0, k, offset, exact=False):
        idx, val = otopk.encode(x.numpy(), x0.numpy(), None, otopk.ACC_NONE, k)
        chg = (x.numpy() - x0.numpy())[idx]
        return (torch.from_numpy(idx.astype(np.int32)) + int(offset), torch.from_numpy(chg),
                torch.from_numpy(val))

    def merge(self, gidx, gchg, gval, k, exact=False):
        pos = otopk.topk_select(otopk.keys_u32(gchg.numpy()), k)
        return gidx[torch.from_numpy(pos)], gval[torch.from_numpy(pos)]

    def count(self, counter, idx, offset):
        i = idx.long() - offset
        i = i[(i >= 0) & (i < counter.numel())]
        counter.index_add_(0, i, torch.ones_like(i, dtype=torch.int32))


def _inputs(n, ties):
    g = torch.Generator().manual_seed(7)
    x = torch.randn(n, generator=g)
    x0 = x - 0.01 * torch.randn(n, generator=g)
    if ties:
        d = torch.round((x - x0) * 300) / 300  # heavy ties at the k-th key
        x0 = x - d
    return x, x0


def _worker(rank, world, port, n, k, ties, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from decentralizepy_amd.shard import sharded_topk_encode
        x, x0 = _inputs(n, ties)
        bounds = np.linspace(0, n, world + 1).astype(int)
        lo, hi = int(bounds[rank]), int(bounds[rank + 1])
        cnt = torch.zeros(hi - lo, dtype=torch.int32)
        idx, val = sharded_topk_encode(x[lo:hi].contiguous(), x0[lo:hi].contiguous(), k, lo,
                                       counter=cnt, ops=OracleOps())
        out_q.put((rank, idx.numpy(), val.numpy(), lo, cnt.numpy()))
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
    for rank, idx, val, lo, cnt in res:
        np.testing.assert_array_equal(idx, oi)
        np.testing.assert_array_equal(val.view(np.uint32), ov.view(np.uint32))
        full_cnt[lo:lo + cnt.shape[0]] = cnt
    np.testing.assert_array_equal(full_cnt, o_cnt)
