"""Diagnostic: fold kernel time vs number of payloads at N = 25M (and the replace kernel)."""
import sys

import torch

sys.path.insert(0, ".")
from decentralizepy_amd import codec  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 25_000_000
k = n // 100
locs = [torch.randn(n, device=dev, generator=g) for _ in range(3)]
outs = [torch.empty(n, device=dev) for _ in range(3)]
pays = [(torch.sort(torch.randperm(n, device=dev, generator=g)[:k])[0].to(torch.int32),
         torch.randn(k, device=dev, generator=g)) for _ in range(16)]
ws = codec.Workspace(dev)
for npay in (1, 2, 4, 8, 16):
    w = [1 / (npay + 1)] * npay
    for i in range(3):
        codec.decode_average(locs[i], pays[:npay], w, 1 / (npay + 1), out=outs[i], workspace=ws)
    with codec.KernelTimer() as kt:
        torch.cuda._sleep(int(50e6))
        for i in range(30):
            codec.decode_average(locs[i % 3], pays[:npay], w, 1 / (npay + 1), out=outs[i % 3],
                                 workspace=ws)
        torch.cuda.synchronize()
    r = {nm: round(ms / c * 1e3, 1) for nm, (ms, c) in kt.result.items()}
    print("np", npay, r, "GB/s fold", round((8 * n + 8 * k * npay) / (r["fold"] * 1e-6) / 1e9))
with codec.KernelTimer() as kt:
    torch.cuda._sleep(int(50e6))
    for i in range(30):
        codec.replace(locs[i % 3], pays[0][0], pays[0][1], out=outs[i % 3], workspace=ws)
    torch.cuda.synchronize()
print("replace", {nm: round(ms / c * 1e3, 1) for nm, (ms, c) in kt.result.items()})
