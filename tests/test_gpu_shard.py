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
