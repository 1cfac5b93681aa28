"""Diagnostic: replace-decode kernel time at C2 / 64 MiB on HBM-rotated inputs (KernelTimer)."""
import sys

import torch

sys.path.insert(0, ".")
from decentralizepy_amd import codec  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1)
for n in (11_000_000, 16_777_216, 25_000_000):
    k = round(0.01 * n)
    R = 6
    locs = [torch.randn(n, device=dev, generator=g) for _ in range(R)]
    outs = [torch.empty(n, device=dev) for _ in range(R)]
    pays = [(torch.sort(torch.randperm(n, device=dev, generator=g)[:k])[0].to(torch.int32),
             torch.randn(k, device=dev, generator=g)) for _ in range(R)]
    ws = codec.Workspace(dev)
    for i in range(R):
        codec.replace(locs[i], *pays[i], out=outs[i], workspace=ws)
    with codec.KernelTimer() as kt:
        torch.cuda._sleep(int(50e6))
        for i in range(60):
            codec.replace(locs[i % R], *pays[i % R], out=outs[i % R], workspace=ws)
        torch.cuda.synchronize()
    us = kt.result["fold"][0] / kt.result["fold"][1] * 1e3
    # back to back, one event pair around the loop (no per-launch events)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(int(50e6))
    e0.record()
    for i in range(60):
        codec.replace(locs[i % R], *pays[i % R], out=outs[i % R], workspace=ws)
    e1.record()
    e1.synchronize()
    us2 = e0.elapsed_time(e1) / 60 * 1e3
    print(f"n={n} replace {us:.2f} us (per-launch events)  {us2:.2f} us (loop)  "
          f"{(8 * n + 8 * k) / us2 / 1e3:.0f} GB/s", flush=True)
    del locs, outs, pays
# reference: a plain device copy of the same bytes (torch), HBM-rotated
for n in (11_000_000, 16_777_216):
    R = 6
    src = [torch.randn(n, device=dev, generator=g) for _ in range(R)]
    dst = [torch.empty(n, device=dev) for _ in range(R)]
    for i in range(R):
        dst[i].copy_(src[i])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(60):
        dst[i % R].copy_(src[i % R])
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) / 60 * 1e3
    print(f"n={n} torch copy {us:.2f} us  {8 * n / us / 1e3:.0f} GB/s", flush=True)
    del src, dst
