"""Diagnostic: per-kernel times (library event pairs) of the plain encode and of the fold-base
encode + patch decode at C2 and 64 MiB.  One JSON line per case."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from decentralizepy_amd import codec  # noqa: E402

dev = torch.device("cuda", 0)
for n in (11_000_000, 16_777_216):
    k = round(0.01 * n)
    g = torch.Generator(device=dev).manual_seed(5)
    R = 6
    xs = [torch.randn(n, device=dev, generator=g) for _ in range(R)]
    x0s = [x - 0.01 * torch.randn(n, device=dev, generator=g) for x in xs]
    outs = [torch.empty(n, device=dev) for _ in range(R)]
    ws = codec.Workspace(dev)
    pays = [codec.topk_encode(xs[j], k, x0=x0s[j], workspace=ws) for j in range(R)]
    pays = [(i.clone(), v.clone()) for i, v in pays]
    for fused in (False, True):
        for npay in (1, 3):
            w = [1 / (npay + 1)] * npay
            wsf = 1 - sum(w)
            for rep in range(2):
                with codec.KernelTimer() as kt:
                    torch.cuda._sleep(int(100e6))
                    for j in range(R * 4):
                        codec.topk_encode(xs[j % R], k, x0=x0s[j % R], workspace=ws,
                                          asynchronous=True,
                                          fold_base=(outs[j % R], w, wsf) if fused else None)
                        codec.decode_average(xs[j % R], [pays[(j + q) % R] for q in range(1, npay + 1)],
                                             w, wsf, out=outs[j % R], workspace=ws,
                                             base_ready=fused)
                    torch.cuda.synchronize()
            print(json.dumps({"n": n, "fused": fused, "npay": npay, "lib": os.environ.get("DPZ_CODEC_LIB", "product"),
                              "kernels_us": {nm: round(ms / c * 1e3, 2) for nm, (ms, c) in kt.result.items()},
                              "launches": {nm: c for nm, (ms, c) in kt.result.items()}}), flush=True)
    del xs, x0s, outs
    torch.cuda.empty_cache()
