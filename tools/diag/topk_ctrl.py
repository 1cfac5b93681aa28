"""Diagnostic: run one sampled encode and print the control block (window, b*, need, T, icut)
plus the size of the threshold bin computed on the host."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from decentralizepy_amd import codec  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 11_000_000
k = round(0.01 * n)
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1234)
x = torch.randn(n, device=dev, generator=g)
x0 = x - 0.01 * torch.randn(n, device=dev, generator=g)
ws = codec.Workspace(dev)
idx, val = codec.topk_encode(x, k, x0=x0, workspace=ws)
torch.cuda.synchronize()
c = ws.buf[:64].cpu().numpy().view(np.uint32)
names = ["prefix", "krem", "status", "nbound", "lo", "hi", "shift", "bstar", "need", "T", "icut"]
ctrl = dict(zip(names, c[:11].tolist()))
print(ctrl)
key = (x - x0).abs().cpu().numpy().view(np.uint32)
lo, hi, sh, bs = ctrl["lo"], ctrl["hi"], ctrl["shift"], ctrl["bstar"]
inwin = key >= lo
b = np.where(key >= hi, 256, (key - lo) >> sh)
print("candidates >= lo:", int(inwin.sum()), " >= hi:", int((key >= hi).sum()),
      " bin b* size:", int((inwin & (b == bs)).sum()), " above b*:", int((inwin & (b > bs)).sum()))
with codec.KernelTimer() as kt:
    torch.cuda._sleep(int(100e6))
    for _ in range(20):
        codec.topk_encode(x, k, x0=x0, workspace=ws, asynchronous=True)
    torch.cuda.synchronize()
print({kk: round(v[0] / v[1] * 1e3, 2) for kk, v in kt.result.items()})
