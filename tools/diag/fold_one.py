"""Diagnostic: one fold shape (alpha, payloads) timed on M = 25,000,009 (for rocprofv3 passes)."""
import sys

import torch

sys.path.insert(0, ".")
from decentralizepy_amd import codec  # noqa: E402

alpha = float(sys.argv[1]) if len(sys.argv) > 1 else 0.01
npay = int(sys.argv[2]) if len(sys.argv) > 2 else 16
dev = torch.device("cuda:0")
m = 25_000_009
k = round(alpha * m)
g = torch.Generator(device=dev).manual_seed(1)
pays = []
for _ in range(npay):
    idx = torch.sort(torch.randperm(m, device=dev, generator=g)[:k])[0].to(torch.int32)
    pays.append((idx, torch.randn(k, device=dev, generator=g)))
locs = [torch.randn(m, device=dev, generator=g) for _ in range(3)]
outs = [torch.empty(m, device=dev) for _ in range(3)]
w = [1 / (npay + 1)] * npay
ws = codec.Workspace(dev)
for i in range(10):
    codec.decode_average(locs[i % 3], pays, w, 1 / (npay + 1), out=outs[i % 3], workspace=ws)
torch.cuda.synchronize()
print("done")
