"""CPU (gloo, world_size 2): ``bench.py --gpus N``'s multi-rank legs — the C4 gossip round
(bench.gossip_case, both exchange modes) and the one-tensor sharded top-k (bench_workloads.shard_case)
— run through the very functions the nccl ranks run, with the oracle injected in place of the HIP
codec.  Every rank must issue the identical sequence of collectives (a mismatch hangs RCCL), and
the bench line's ``gossip_round`` / ``shard`` objects must carry the same keys at N = 2 as at
N = 1 (the first multi-rank RCCL run is the driver's SCALE run)."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.test_cpu_gossip import _oracle_encode, _oracle_fold, _torch_combine, _torch_partial
from tests.test_cpu_shard import OracleOps

COLLECTIVES = ("all_gather_into_tensor", "reduce_scatter_tensor", "all_reduce", "barrier",
               "all_gather", "broadcast")


class _Recorder:
    """Wraps torch.distributed's collectives: records (name, shape, dtype, op) per call."""

    def __init__(self):
        self.calls = []
        self._orig = {}

    def __enter__(self):
        for name in COLLECTIVES:
            fn = getattr(dist, name)
            self._orig[name] = fn

            def wrapped(*a, _fn=fn, _name=name, **kw):
                t = a[0] if a and isinstance(a[0], torch.Tensor) else None
                op = kw.get("op", a[1] if len(a) > 1 and not isinstance(a[1], torch.Tensor)
                            else None)
                self.calls.append((_name, tuple(t.shape) if t is not None else None,
                                   str(t.dtype) if t is not None else None, str(op)))
                return _fn(*a, **kw)
            setattr(dist, name, wrapped)
        return self

    def __exit__(self, *exc):
        for name, fn in self._orig.items():
            setattr(dist, name, fn)


def _legs(rank, world, d):
    import bench
    import bench_workloads as bw
    dev = torch.device("cpu")
    kw = dict(encode=_oracle_encode, fold=_oracle_fold, partial=_torch_partial,
              combine=_torch_combine)
    out = {}
    n = 3_000
    for mode in ("allgather", "reduce_scatter"):
        ekw = dict(kw, hbm_budget=1 << 40)
        gr = bench.gossip_case(n, 0.01, dev, rank, world, d, rounds=2, warmup=1, exchange=mode,
                               engine_kw=ekw)
        out[mode] = bench.gossip_line(gr, world)
    sh = bw.shard_case(dev, rank, world, d, n=40_000, alpha=0.01, steps=2, warmup=1,
                       ops=OracleOps(), unpack=lambda v: v.float())
    out["shard"] = {k_: (round(v, 4) if isinstance(v, float) else v) for k_, v in sh.items()}
    return out


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        with _Recorder() as rec:
            out = _legs(rank, world, dist)
        q.put((rank, rec.calls, {k: sorted(v) for k, v in out.items()}))
    except Exception as e:  # noqa: BLE001 - reported to the parent instead of a queue timeout
        import traceback
        q.put((rank, None, traceback.format_exc() + repr(e)))
    finally:
        dist.destroy_process_group()


def test_multi_rank_legs_issue_identical_collectives():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, 29740, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
    for rank, calls, keys in res:
        assert calls is not None, keys
    calls0, calls1 = res[0][1], res[1][1]
    assert len(calls0) > 0 and calls0 == calls1  # the same collectives, shapes, dtypes, ops
    names = {c[0] for c in calls0}
    assert {"all_gather_into_tensor", "reduce_scatter_tensor", "all_reduce", "barrier"} <= names
    # the N = 1 line's objects keep their keys at N = 2
    one = {k: sorted(v) for k, v in _legs(0, 1, None).items()}
    assert res[0][2] == one and res[1][2] == one
