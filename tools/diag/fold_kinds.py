"""A/B of the fold kernels (DPZ_FOLD_KIND 0 = auto, 1 = classic hit-chain / phase, 2 = 4-slot
group, 3 = one-phase slot fold) at the C3 shape: M = 25,000,009 coefficients, 16 sparse payloads
at JWINS alphas, and a JWINS-round node's 3 neighbours with full-share payloads among them.
Per case: fold-kernel average (library event pairs) and the whole call (HIP events around the
loop on the current stream).  One JSON object per line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from decentralizepy_amd import codec  # noqa: E402


def case(dev, m, alpha, npay, ndense, kinds, reps=20):
    k = round(alpha * m)
    g = torch.Generator(device=dev).manual_seed(1)
    pays = []
    for j in range(npay):
        if j < ndense:
            pays.append((None, torch.randn(m, device=dev, generator=g)))
            continue
        idx = torch.sort(torch.randperm(m, device=dev, generator=g)[:k])[0].to(torch.int32)
        pays.append((idx, torch.randn(k, device=dev, generator=g)))
    locs = [torch.randn(m, device=dev, generator=g) for _ in range(3)]
    outs = [torch.empty(m, device=dev) for _ in range(3)]
    w = [1 / (npay + 1)] * npay
    ws = codec.Workspace(dev)
    res = {}
    for kind in kinds:
        os.environ["DPZ_FOLD_KIND"] = kind
        for i in range(3):
            codec.decode_average(locs[i % 3], pays, w, 1 / (npay + 1), out=outs[i % 3],
                                 workspace=ws)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(int(20e6))
        e0.record()
        for i in range(reps):
            codec.decode_average(locs[i % 3], pays, w, 1 / (npay + 1), out=outs[i % 3],
                                 workspace=ws)
        e1.record()
        e1.synchronize()
        call_us = e0.elapsed_time(e1) / reps * 1e3
        with codec.KernelTimer() as kt:
            for i in range(6):
                codec.decode_average(locs[i % 3], pays, w, 1 / (npay + 1), out=outs[i % 3],
                                     workspace=ws)
            torch.cuda.synchronize()
        kern = {nm: round(ms / c * 1e3, 1) for nm, (ms, c) in kt.result.items()}
        alg = 8 * m + sum(8 * p[1].numel() if p[0] is not None else 4 * m for p in pays)
        res[kind] = {"call_us": round(call_us, 1), "kernels_us_event_pair": kern,
                     "frac": round(alg / (call_us * 1e-6) / 8e12, 3)}
    os.environ.pop("DPZ_FOLD_KIND", None)
    return res


def main():
    dev = torch.device("cuda:0")
    m = 25_000_009
    kinds = os.environ.get("FOLD_KINDS", "0 1 2 4").split()
    # FOLD_CASES="m:alpha:npay:ndense ..." replaces the default list
    cases = [tuple(t(v) for t, v in zip((int, float, int, int), c.split(":")))
             for c in os.environ.get("FOLD_CASES", "").split()]
    for mm, alpha, npay, nd in cases or ((m, 0.01, 16, 0), (m, 0.03, 16, 0), (m, 0.05, 16, 0),
                                (m, 0.1, 16, 0), (m, 0.2, 16, 0), (m, 0.3, 16, 0),
                                (m, 0.01, 3, 0), (m, 0.1, 3, 0), (m, 0.3, 3, 0), (m, 0.4, 3, 0),
                                (m, 0.1, 3, 1), (11_000_000, 0.01, 3, 0),
                                (11_000_000, 0.01, 4, 0), (11_000_000, 0.01, 1, 0)):
        r = case(dev, mm, alpha, npay, nd, kinds)
        print(json.dumps({"m": mm, "alpha": alpha, "npay": npay, "dense": nd,
                          "walk_epl": os.environ.get("DPZ_FOLD_WALK_EPL"), "kinds": r}),
              flush=True)


if __name__ == "__main__":
    main()
