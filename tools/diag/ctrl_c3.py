"""Diagnostic: control block over repeated C3 (wavelet, ADD accumulation) encodes of one state."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from decentralizepy_amd import codec  # noqa: E402

names = ["prefix", "krem", "status", "nbound", "lo", "hi", "shift", "bstar", "need", "T", "icut"]
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(3)
n = 25_000_000
m = codec.wavedec_len(n, 4)
k = round(0.01 * m)
x = torch.randn(n, device=dev, generator=g)
x0 = x - 0.01 * torch.randn(n, device=dev, generator=g)
acc = 0.01 * torch.randn(m, device=dev, generator=g)
cnt = torch.zeros(m, dtype=torch.int32, device=dev)
wx, wc = codec.wavedec(x, 4, x0=x0)
ws = codec.Workspace(dev)
for it in range(25):
    idx, val = codec.topk_encode(wc, k, acc=acc, acc_mode=codec.DPZ_ACC_ADD, vals_src=wx,
                                 counter=cnt, workspace=ws, asynchronous=True)
    torch.cuda.synchronize()
    c = ws.buf[:64].cpu().numpy().view(np.uint32)
    d = dict(zip(names, c[:11].tolist()))
    key = (wc + acc).abs()
    print(it, d["status"], d["lo"], d["hi"], d["shift"], d["bstar"], d["need"],
          "zeros(acc)", int((acc == 0).sum()), flush=True)
