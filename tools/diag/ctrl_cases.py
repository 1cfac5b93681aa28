"""Diagnostic: control block (window, b*, need, T, icut, status) of one sampled encode for the
C3 (wavelet domain, accumulation) and C5 (alpha = 0.001) shapes."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from decentralizepy_amd import codec  # noqa: E402

names = ["prefix", "krem", "status", "nbound", "lo", "hi", "shift", "bstar", "need", "T", "icut"]
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(3)


def show(tag, ws):
    torch.cuda.synchronize()
    c = ws.buf[:64].cpu().numpy().view(np.uint32)
    print(tag, dict(zip(names, c[:11].tolist())), flush=True)


# C5
n = 67_108_864
x = torch.randn(n, device=dev, generator=g)
x0 = x - 0.01 * torch.randn(n, device=dev, generator=g)
ws = codec.Workspace(dev)
codec.topk_encode(x, round(0.001 * n), x0=x0, workspace=ws, asynchronous=True)
show("C5", ws)
del x, x0
# C3
n = 25_000_000
m = codec.wavedec_len(n, 4)
x = torch.randn(n, device=dev, generator=g)
x0 = x - 0.01 * torch.randn(n, device=dev, generator=g)
acc = 0.01 * torch.randn(m, device=dev, generator=g)
wx, wc = codec.wavedec(x, 4, x0=x0)
ws = codec.Workspace(dev)
codec.topk_encode(wc, round(0.01 * m), acc=acc.clone(), acc_mode=codec.DPZ_ACC_ACCUMULATE,
                  vals_src=wx, workspace=ws, asynchronous=True)
show("C3 acc", ws)
ws = codec.Workspace(dev)
codec.topk_encode(wc, round(0.01 * m), vals_src=wx, workspace=ws, asynchronous=True)
show("C3 noacc", ws)
key = (wc + acc).abs()
print("C3 key quantiles", torch.quantile(key[:1_000_000], torch.tensor([0.5, 0.99, 0.999], device=dev)).tolist())
