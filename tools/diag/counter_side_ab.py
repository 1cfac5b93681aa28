"""A/B: the plugin path's one-node step (encode + fold of 1 / 3 payloads, bench.product_one_node)
with the counter update inside the encode's compact (the reference's order) vs deferred to a
second stream (dpz_scatter_add_i32 after an event, joined at the end of the timed loop so the
region still holds every byte).  C2 and 64 MiB, HBM-rotated states."""
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from decentralizepy_amd import codec  # noqa: E402
from decentralizepy_amd.shard import _scatter_add  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
for n in (11_000_000, 16_777_216):
    k = round(0.01 * n)
    R = max(1, math.ceil(2 * bench.L3_BYTES / (16 * n + 8 * k)) + 1)
    g = torch.Generator(device=dev).manual_seed(5)
    sets = []
    for _ in range(R):
        x = torch.randn(n, device=dev, generator=g)
        sets.append(dict(x=x, x0=x - 0.01 * torch.randn(n, device=dev, generator=g),
                         counter=torch.zeros(n, dtype=torch.int32, device=dev),
                         idx=torch.empty(k, dtype=torch.int32, device=dev),
                         val=torch.empty(k, device=dev), out=torch.empty(n, device=dev)))
    st = torch.cuda.Stream(dev)
    side = torch.cuda.Stream(dev)
    ws = codec.Workspace(dev)
    res = {}
    for npay in (1, 3):
        w = [1.0 / (npay + 1)] * npay
        wt = 0
        for v in w:
            wt += v
        pays = [[(sets[(j - q) % R]["idx"], sets[(j - q) % R]["val"]) for q in range(1, npay + 1)]
                for j in range(R)]
        for mode in ("inline", "side", "inline", "side"):
            def step(j):
                d = sets[j % R]
                if mode == "inline":
                    codec.topk_encode(d["x"], k, x0=d["x0"], counter=d["counter"], idx_out=d["idx"],
                                      val_out=d["val"], workspace=ws, asynchronous=True)
                else:
                    codec.topk_encode(d["x"], k, x0=d["x0"], idx_out=d["idx"], val_out=d["val"],
                                      workspace=ws, asynchronous=True)
                    side.wait_stream(st)
                    with torch.cuda.stream(side):
                        _scatter_add(d["counter"], d["idx"], 0)
                codec.decode_average(d["x"], pays[j % R], w, 1 - wt, out=d["out"], workspace=ws)
            with torch.cuda.stream(st):
                for j in range(R):
                    step(j)
            torch.cuda.synchronize()
            reps = 200
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(st):
                torch.cuda._sleep(int(400e6))
                ev0.record(st)
                for j in range(reps):
                    step(j)
                st.wait_stream(side)
                ev1.record(st)
            ev1.synchronize()
            res.setdefault(f"{npay}_{mode}", []).append(round(ev0.elapsed_time(ev1) / reps * 1e3, 2))
    print(json.dumps({"n": n, "step_us": res, "status": codec.topk_sticky_status(ws, clear=True)}),
          flush=True)
