"""Top-k encode of ONE tensor split over ranks ("one tensor, top-k encode: yes,
one small exchange step"; the C5 shape: a 256 MiB model on 8 MI355X).

Rank r holds the contiguous slice [offset_r, offset_r + n_r) of the flat model (and of init_model,
shared_parameters_counter).  The global top-k under the reference's rule (k largest |x - x0|,
ties to the lowest index; sharing/PartialModel.py:164-186) is found with ONE collective:

  1. every rank selects its local top-k (the full k, not k / world) with the HIP encoder — the
     global top-k is contained in the union: a rank contributes at most k entries, and those are
     its k largest with the lowest local (= lowest global) indices among ties;
  2. one all-gather of the k candidates of every rank (global index, change, value: 12 B each;
     6.4 MB for C5 on 8 ranks) over RCCL;
  3. every rank runs the same top-k over the world * k gathered changes (their concatenation is
     in global index order, so the encoder's lowest-position tie rule is the lowest global index)
     and gathers the winners' indices and values — identical on every rank, no second exchange;
  4. each rank applies counter[idx] += 1 to the winners inside its own slice.

The result is bit-identical to a one-GPU encode of the whole tensor (tests/test_gpu_shard.py,
tests/test_cpu_shard.py).  Only the all-gather crosses xGMI; no reduce-scatter is needed.
"""
import torch

from . import _lib, codec
from .codec import _ptr, _stream


def _gather_change(x, x0, idx):
    out = torch.empty(idx.numel(), dtype=torch.float32, device=x.device)
    rc = _lib.lib().dpz_gather_change(_ptr(x), _ptr(x0), x.numel(), _ptr(idx), idx.numel(),
                                      _ptr(out), _stream(x.device))
    _lib.check(rc, "dpz_gather_change")
    return out


def _gather_u32(src, pos):
    out = torch.empty(pos.numel(), dtype=src.dtype, device=src.device)
    rc = _lib.lib().dpz_gather_u32(_ptr(src), src.numel(), _ptr(pos), pos.numel(), _ptr(out),
                                   _stream(src.device))
    _lib.check(rc, "dpz_gather_u32")
    return out


def _scatter_add(counter, idx, offset):
    rc = _lib.lib().dpz_scatter_add_i32(_ptr(counter), counter.numel(), _ptr(idx), idx.numel(),
                                        int(offset), 1, _stream(counter.device))
    _lib.check(rc, "dpz_scatter_add_i32")


class HipShardOps:
    """Device implementation of the per-rank steps (the HIP codec).  The encodes are enqueued
    optimistically (no host sync); their sampled-path status words travel with the candidates
    and the caller re-runs the round exactly in the rare case one of them missed."""

    def __init__(self, device):
        self.ws = codec.Workspace(device)
        self.ws_merge = codec.Workspace(device)

    def local_candidates(self, x, x0, k, offset, exact=False):
        idx, val = codec.topk_encode(x, k, x0=x0, workspace=self.ws, asynchronous=not exact,
                                     exact=exact)
        chg = _gather_change(x, x0, idx)
        return (idx + int(offset)).to(torch.int32), chg, val

    def local_status(self):
        """This rank's sampled-path status word (device int32[1]; 0 = the result is final)."""
        return self.ws.buf[8:12].view(torch.int32)

    def merge(self, gidx, gchg, gval, k, exact=False):
        # positions of the k winners among the gathered changes, in ascending position order
        pos, _ = codec.topk_encode(gchg, k, workspace=self.ws_merge, asynchronous=not exact,
                                   exact=exact)
        return _gather_u32(gidx, pos), _gather_u32(gval, pos)

    def merge_status(self):
        return self.ws_merge.buf[8:12].view(torch.int32)

    def count(self, counter, idx, offset):
        _scatter_add(counter, idx, offset)


def sharded_topk_encode(x, x0, k, offset, counter=None, group=None, ops=None):
    """Global top-k of a tensor sharded over the ranks of `group`.

    x, x0: this rank's slice (flat fp32); offset: the slice's first global index; k: the GLOBAL
    k (every slice must hold at least k elements).  Returns ``(idx int32[k] global ascending,
    val fp32[k])`` — the whole payload, identical on every rank.  ``counter`` (this rank's slice
    of shared_parameters_counter) gets += 1 at the winners inside the slice.
    """
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if x.numel() < k:
        raise ValueError("every shard must hold at least k elements")
    ops = ops or HipShardOps(x.device)
    for exact in (False, True):
        idx, chg, val = ops.local_candidates(x, x0, k, offset, exact=exact)
        st = (ops.local_status() if hasattr(ops, "local_status")
              else torch.zeros(1, dtype=torch.int32, device=idx.device))
        if world > 1:
            # one exchange: the three candidate arrays and the status word, packed as 32-bit
            # words in ONE all-gather
            pack = torch.cat([idx.view(torch.float32), chg, val, st.view(torch.float32)])
            gflat = torch.empty(world * (3 * k + 1), dtype=torch.float32, device=idx.device)
            dist.all_gather_into_tensor(gflat, pack, group=group)
            gpack = gflat.view(world, 3 * k + 1)
            gidx = gpack[:, :k].reshape(-1).contiguous().view(torch.int32)
            gchg = gpack[:, k:2 * k].reshape(-1).contiguous()
            gval = gpack[:, 2 * k:3 * k].reshape(-1).contiguous()
            gst = gpack[:, 3 * k].contiguous().view(torch.int32)
        else:
            gidx, gchg, gval, gst = idx, chg, val, st
        widx, wval = ops.merge(gidx, gchg, gval, k, exact=exact)
        mst = (ops.merge_status() if hasattr(ops, "merge_status")
               else torch.zeros(1, dtype=torch.int32, device=idx.device))
        # every rank sees the same gathered statuses and the same merge: the same decision
        if exact or int(gst.abs().sum().item()) + int(mst.abs().sum().item()) == 0:
            break
    if counter is not None:
        ops.count(counter, widx, offset)
    return widx, wval
