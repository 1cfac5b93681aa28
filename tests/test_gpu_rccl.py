"""GPU: the multi-GPU data paths through RCCL itself, as a one-rank loopback (the box has one
GPU; RCCL refuses two ranks on one device, and the 2-rank semantics are covered with gloo on the
CPU).  A process group of world size 1 on the "nccl" backend (= RCCL on ROCm) is handed to each
engine explicitly, which makes it issue its real collectives — the C4 payload
all_gather_into_tensor, the over-HBM packed reduce_scatter_tensor, the JWINS variable-size
all-gather, the sharded top-k's candidate all-gather and the sharded DWT's halo / owned-range
all-gathers — on device buffers; every result must equal the same engine run without a group
bit-for-bit."""
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rccl_group(dev):
    import torch.distributed as dist
    if dist.is_initialized():
        pytest.skip("a process group already exists in this process")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=dev)
    assert dist.get_backend() == "nccl"
    try:
        yield dist.group.WORLD
    finally:
        dist.destroy_process_group()


def _bits(t):
    return t.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("exchange", ["allgather", "reduce_scatter"])
def test_gossip_round_through_rccl(dev, rccl_group, exchange):
    from decentralizepy_amd.gossip import GossipRound, read_edges
    from tests.test_cpu_gossip import EDGES96, _models
    adj = read_edges(EDGES96)
    n = 40_000
    x = _models(len(adj), n).to(dev)
    kw = dict(exchange=exchange, hbm_budget=(1 if exchange == "reduce_scatter" else None))
    ref = GossipRound(adj, x.clone(), 0.02, **kw)
    eng = GossipRound(adj, x.clone(), 0.02, rank=0, world=1, group=rccl_group, **kw)
    assert eng.coll and not ref.coll and eng.exchange_mode == exchange
    for r in range(2):
        g = torch.Generator().manual_seed(100 + r)
        noise = (0.01 * torch.randn(len(adj), n, generator=g)).to(dev)
        ref.x += noise
        eng.x += noise
        ref.step()
        eng.step()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(_bits(eng.x), _bits(ref.x))
        np.testing.assert_array_equal(eng.counter.cpu().numpy(), ref.counter.cpu().numpy())


def test_jwins_round_through_rccl(dev, rccl_group):
    from decentralizepy_amd.gossip import read_edges
    from decentralizepy_amd.gossip_jwins import JwinsRound
    from tests.test_cpu_gossip_jwins import EDGES16, TUTORIAL_ALPHAS, _noise
    adj = read_edges(EDGES16)
    n = 300_001
    x = torch.randn(16, n, generator=torch.Generator().manual_seed(11)).to(dev)
    ref = JwinsRound(adj, x.clone(), TUTORIAL_ALPHAS)
    eng = JwinsRound(adj, x.clone(), TUTORIAL_ALPHAS, rank=0, world=1, group=rccl_group)
    assert eng.coll and not ref.coll
    kinds = set()
    for r in range(2):
        for j in range(16):
            nz = torch.from_numpy(_noise(r, j, n)).to(dev)
            ref.x[j] += nz
            eng.x[j] += nz
        ref.step()
        eng.step()
        kinds |= {a >= 0.5 for a in eng.alphas}
        torch.cuda.synchronize()
        for name in ("x", "x0", "acc"):
            np.testing.assert_array_equal(_bits(getattr(eng, name)), _bits(getattr(ref, name)),
                                          err_msg=name)
        np.testing.assert_array_equal(eng.counter.cpu().numpy(), ref.counter.cpu().numpy())
    assert kinds == {True, False}  # partial and full shares both crossed the all-gather


@pytest.mark.parametrize("val_fp16,k", [(False, 20_000), (True, 20_000), (True, 20_001)])
def test_sharded_topk_through_rccl(dev, rccl_group, val_fp16, k):
    """k = 20,001 with fp16 values: an odd number of 2-byte values, so the packed row's status
    word would sit 2 bytes off a 4-byte boundary without the value section's padding (the
    one-rank gather hands back a view, no copy)."""
    from decentralizepy_amd.shard import sharded_topk_encode
    n = 2_000_003
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(n, device=dev, generator=g)
    x0 = x - 0.01 * torch.randn(n, device=dev, generator=g)
    c1 = torch.zeros(n, dtype=torch.int32, device=dev)
    c2 = torch.zeros(n, dtype=torch.int32, device=dev)
    i1, v1 = sharded_topk_encode(x, x0, k, 0, counter=c1, val_fp16=val_fp16)
    i2, v2 = sharded_topk_encode(x, x0, k, 0, counter=c2, group=rccl_group, val_fp16=val_fp16)
    torch.cuda.synchronize()
    assert torch.equal(i1, i2) and torch.equal(c1, c2)
    assert torch.equal(v1.view(torch.int16 if val_fp16 else torch.int32),
                       v2.view(torch.int16 if val_fp16 else torch.int32))


def test_sharded_wavedec_through_rccl(dev, rccl_group):
    from decentralizepy_amd import codec
    from decentralizepy_amd.shard import sharded_wavedec, sharded_waverec
    n, level = 1_000_003, 4
    g = torch.Generator(device=dev).manual_seed(9)
    x = torch.randn(n, device=dev, generator=g)
    x0 = x - 0.01 * torch.randn(n, device=dev, generator=g)
    wx, wd = codec.wavedec(x, level, x0=x0)
    cx, cd = sharded_wavedec(x, x0, n, level, group=rccl_group)
    torch.cuda.synchronize()
    assert torch.equal(cx.view(torch.int32), wx.view(torch.int32))
    assert torch.equal(cd.view(torch.int32), wd.view(torch.int32))
    out = sharded_waverec(cx, n, level, group=rccl_group)
    assert torch.equal(out.view(torch.int32), codec.waverec(wx, n, level).view(torch.int32))
