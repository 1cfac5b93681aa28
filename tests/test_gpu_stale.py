"""GPU: nothing that runs after a missed sampled encode follows the stale contents of its output
buffers.  A layout whose large changes hide between the sample chunks
(tests/layouts.py) makes the sampled path miss; idx_out starts poisoned with indices far outside
[0, n), as a reused buffer may hold them.  The fold-base encode (PartialModel's one-neighbour
path, reference sharing/PartialModel.py:188-255 + Sharing.py:156-190) and the sharded encode with
fp16 values (BASELINE config 5, shard.py) must still give the oracle's result."""
import numpy as np
import pytest
import torch

from oracle import fold as ofold
from oracle import topk as otopk
from tests.layouts import miss_layout

pytestmark = pytest.mark.gpu

POISON = 0x7FFFFFF0


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


@pytest.mark.parametrize("asynchronous", [False, True])
def test_foldbase_encode_after_forced_miss(dev, asynchronous):
    from decentralizepy_amd import codec
    n = 1 << 20
    k = round(0.01 * n)
    x, x0 = miss_layout(n, k)
    tx, tx0 = torch.from_numpy(x).to(dev), torch.from_numpy(x0).to(dev)
    tcnt = torch.zeros(n, dtype=torch.int32, device=dev)
    idx = torch.full((k,), POISON, dtype=torch.int32, device=dev)
    val = torch.empty(k, device=dev)
    base = torch.full((n,), float("nan"), device=dev)
    ws = codec.Workspace(dev)
    w, w_self = [0.25], 0.75
    codec.topk_encode(tx, k, x0=tx0, counter=tcnt, idx_out=idx, val_out=val, workspace=ws,
                      fold_base=(base, w, w_self), asynchronous=asynchronous)
    if asynchronous:
        torch.cuda.synchronize()
        assert codec.topk_sticky_status(ws) != 0  # the layout made the sampled path miss
        assert (idx.cpu().numpy() == POISON).all()  # and nothing was written
        codec.topk_complete(tx, k, idx, val, ws, x0=tx0, counter=tcnt)
    o_cnt = np.zeros(n, dtype=np.int32)
    oi, ov = otopk.encode(x, x0, None, otopk.ACC_NONE, k, counter=o_cnt)
    np.testing.assert_array_equal(idx.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(val.cpu().numpy()), _bits(ov))
    np.testing.assert_array_equal(tcnt.cpu().numpy(), o_cnt)
    # the round's fold over the base: a neighbour's payload (here the node's own selection)
    out = codec.decode_average(tx, [(idx, val)], w, w_self, out=base, workspace=ws,
                               base_ready=True)
    ref = ofold.fold(x, [(oi, ov)], w, w_self)
    np.testing.assert_array_equal(_bits(out.cpu().numpy()), _bits(ref))


def test_sharded_fp16_encode_after_forced_miss(dev):
    from decentralizepy_amd import codec
    from decentralizepy_amd.shard import HipShardOps, sharded_topk_encode

    class PoisonedOps(HipShardOps):
        """The local encode writes into an idx buffer that starts poisoned."""

        def local_candidates(self, x, x0, k, offset, exact=False, val_fp16=False):
            io = torch.full((k,), POISON, dtype=torch.int32, device=x.device)
            idx, val = codec.topk_encode(x, k, x0=x0, workspace=self.ws, asynchronous=not exact,
                                         exact=exact, val_fp16=val_fp16, idx_out=io)
            chg = codec_gather_change(x, x0, idx)
            return (idx + int(offset)).to(torch.int32), chg, val

    from decentralizepy_amd.shard import _gather_change as codec_gather_change
    n = 1 << 20
    k = round(0.01 * n)
    x, x0 = miss_layout(n, k)
    tx, tx0 = torch.from_numpy(x).to(dev), torch.from_numpy(x0).to(dev)
    tcnt = torch.zeros(n, dtype=torch.int32, device=dev)
    ops = PoisonedOps(dev)
    idx, val = sharded_topk_encode(tx, tx0, k, 0, counter=tcnt, ops=ops, val_fp16=True)
    o_cnt = np.zeros(n, dtype=np.int32)
    oi, ov = otopk.encode(x, x0, None, otopk.ACC_NONE, k, counter=o_cnt)
    np.testing.assert_array_equal(idx.cpu().numpy(), oi)
    np.testing.assert_array_equal(val.cpu().numpy().view(np.uint16),
                                  torch.from_numpy(ov).half().numpy().view(np.uint16))
    np.testing.assert_array_equal(tcnt.cpu().numpy(), o_cnt)
