"""Diagnostic: where the one-node step's time goes (C2 and 64 MiB, HBM-rotated states).

1. Per-kernel averages of the encode with the lone (W_MAX) and the shared (W_SMALL) filter
   grid, with and without the counter update (the scattered counter[idx] += 1 in compact).
2. The one-node serial step (encode of state i + co-scheduled replace decode of state i-1's
   payload, one stream) for several DPZ_COSCHED splits of the decode over sample / select /
   compact, HIP events around the loop, median of 5 regions.
Prints one JSON object per line.
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from decentralizepy_amd import codec  # noqa: E402
from decentralizepy_amd._lib import DPZ_BATCH_DECODE, DPZ_BATCH_ENCODE  # noqa: E402

dev = torch.device("cuda", 0)


def states(n, R):
    k = round(0.01 * n)
    g = torch.Generator(device=dev).manual_seed(3)
    sets = []
    for _ in range(R):
        x = torch.randn(n, device=dev, generator=g)
        sets.append(dict(x=x, x0=x - 0.01 * torch.randn(n, device=dev, generator=g),
                         counter=torch.zeros(n, dtype=torch.int32, device=dev),
                         idx=torch.empty(k, dtype=torch.int32, device=dev),
                         val=torch.empty(k, device=dev), out=torch.empty(n, device=dev)))
    return sets, k


def kernels(n, sets, k, shared, counter):
    ws = codec.Workspace(dev)
    for d in sets:
        codec.topk_encode(d["x"], k, x0=d["x0"], counter=d["counter"] if counter else None,
                          idx_out=d["idx"], val_out=d["val"], workspace=ws, asynchronous=True,
                          shared=shared)
    torch.cuda.synchronize()
    with codec.KernelTimer() as kt:
        torch.cuda._sleep(int(50e6))
        for _ in range(4):
            for d in sets:
                codec.topk_encode(d["x"], k, x0=d["x0"],
                                  counter=d["counter"] if counter else None, idx_out=d["idx"],
                                  val_out=d["val"], workspace=ws, asynchronous=True, shared=shared)
        torch.cuda.synchronize()
    st = codec.topk_sticky_status(ws, clear=True)
    return {nm: round(ms / c * 1e3, 2) for nm, (ms, c) in kt.result.items()}, st


def serial_step(sets, n, k, reps=60):
    st = torch.cuda.Stream(dev)
    one = codec.NodeStepBatch(sets, n, k, [st], [codec.Workspace(dev)],
                              decode_src=lambda j: (j - 1) % len(sets))
    for _ in range(2):
        one.run()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(st):
            torch.cuda._sleep(int(20e6))
            e0.record(st)
        for _ in range(reps // len(sets)):
            one.run(DPZ_BATCH_ENCODE | DPZ_BATCH_DECODE)
        e1.record(st)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / (reps // len(sets) * len(sets)) * 1e3)
    return round(sorted(ts)[2], 2), one.sticky_status(clear=True)


def main():
    shares = sys.argv[1:] or ["0.45,0.55,0", "0,0.4,0.6", "0,0.3,0.7", "0,0.5,0.5", "0.2,0.4,0.4",
                              "0,1,0", "0,0,1"]
    for n in (11_000_000, 16_777_216):
        R = max(2, -(-2 * 256 * 2 ** 20 // (16 * n + 8 * round(0.01 * n))) + 1)
        sets, k = states(n, R)
        for shared in (False, True):
            for counter in (True, False):
                kk, stt = kernels(n, sets, k, shared, counter)
                print(json.dumps({"n": n, "shared": shared, "counter": counter, "status": stt,
                                  "kernels_us_event_pair": kk}), flush=True)
        for sh in shares:
            os.environ["DPZ_COSCHED"] = sh
            t, stt = serial_step(sets, n, k)
            print(json.dumps({"n": n, "cosched": sh, "serial_step_us": t, "status": stt}),
                  flush=True)
        os.environ.pop("DPZ_COSCHED", None)
        del sets
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
