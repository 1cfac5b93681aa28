"""Diagnostic: the few-payload walk fold (the plugin path's _averaging, sharing/Sharing.py:156-190)
at 64 MiB, back-to-back launches over HBM-rotated locals timed with HIP events around the loop:
1..4 payloads at alpha 0.01, one nearly empty payload (64 entries: streaming + start-up only), the
replace decode and a torch copy of the same bytes.  Diagnostic-build knobs from the environment
(DPZ_FOLD_WALK_EPL, DPZ_FOLD_BLOCKS, ...) when run with DPZ_CODEC_LIB=...diag.so.  One JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from decentralizepy_amd import codec  # noqa: E402


def timed(fn, reps):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    torch.cuda.synchronize()
    torch.cuda._sleep(int(20e6))
    ev[0].record()
    for i in range(reps):
        fn(i)
    ev[1].record()
    torch.cuda.synchronize()
    return round(ev[0].elapsed_time(ev[1]) * 1e3 / reps, 2)


def main():
    dev = torch.device("cuda:0")
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16_777_216
    k = round(0.01 * n)
    g = torch.Generator(device=dev).manual_seed(1)
    R = 6
    locs = [torch.randn(n, device=dev, generator=g) for _ in range(R)]
    outs = [torch.empty(n, device=dev) for _ in range(R)]
    pays = []
    for _ in range(4):
        idx = torch.sort(torch.randperm(n, device=dev, generator=g)[:k])[0].to(torch.int32)
        pays.append((idx, torch.randn(k, device=dev, generator=g)))
    tiny = (torch.sort(torch.randperm(n, device=dev, generator=g)[:64])[0].to(torch.int32),
            torch.randn(64, device=dev, generator=g))
    ws = codec.Workspace(dev)
    res = {"n": n, "env": {kk: v for kk, v in os.environ.items() if kk.startswith("DPZ_")}}
    reps = 48
    for npay in (1, 2, 3, 4):
        w = [1 / (npay + 1)] * npay
        p = pays[:npay]
        f = (lambda i, p=p, w=w: codec.decode_average(locs[i % R], p, w, 1 / (len(p) + 1),
                                                      out=outs[i % R], workspace=ws))
        f(0)
        res[f"fold{npay}_us"] = timed(f, reps)
    f = (lambda i: codec.decode_average(locs[i % R], [tiny], [0.5], 0.5, out=outs[i % R],
                                        workspace=ws))
    f(0)
    res["fold_tiny_us"] = timed(f, reps)
    f = (lambda i: codec.replace(locs[i % R], pays[0][0], pays[0][1], out=outs[i % R],
                                 workspace=ws))
    f(0)
    res["replace_us"] = timed(f, reps)
    res["torch_copy_us"] = timed(lambda i: outs[i % R].copy_(locs[i % R]), reps)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
