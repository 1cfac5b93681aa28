"""Diagnostic: per-kernel device time of the sampled top-k encode on HBM-rotated inputs.
Pick the library build with DPZ_CODEC_LIB."""
import sys

import torch

sys.path.insert(0, ".")
from decentralizepy_amd import codec  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 11_000_000
R = 6
k = round(0.01 * n)
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(3)
sets = []
for _ in range(R):
    x = torch.randn(n, device=dev, generator=g)
    sets.append((x, x - 0.01 * torch.randn(n, device=dev, generator=g)))
ws = codec.Workspace(dev)
idx = torch.empty(k, dtype=torch.int32, device=dev)
val = torch.empty(k, dtype=torch.float32, device=dev)
for i in range(2 * R):
    x, x0 = sets[i % R]
    codec.topk_encode(x, k, x0=x0, idx_out=idx, val_out=val, workspace=ws, asynchronous=True)
torch.cuda.synchronize()
with codec.KernelTimer() as kt:
    torch.cuda._sleep(int(100e6))
    for i in range(60):
        x, x0 = sets[i % R]
        codec.topk_encode(x, k, x0=x0, idx_out=idx, val_out=val, workspace=ws, asynchronous=True)
    torch.cuda.synchronize()
print({kk: round(v[0] / v[1] * 1e3, 2) for kk, v in kt.result.items()})
