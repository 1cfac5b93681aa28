"""Diagnostic: the generic-filter wavelet kernels' times at N = 25 M, level 4 (db4, sym8, coif3,
dmey at level 2) beside the fused sym2 kernel: the W(x), W(x - x0) pair and the IDWT.  One JSON
line."""
import json
import sys

import torch

sys.path.insert(0, ".")
from decentralizepy_amd import codec  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1)
n = 25_000_000
x = [torch.randn(n, device=dev, generator=g) for _ in range(2)]
x0 = [torch.randn(n, device=dev, generator=g) for _ in range(2)]
res = {}
for name, level in (("sym2", 4), ("db4", 4), ("sym8", 4), ("coif3", 4), ("dmey", 2)):
    m = codec.wavedec_len(n, level, name)
    wx = [torch.empty(m, device=dev) for _ in range(2)]
    wc = [torch.empty(m, device=dev) for _ in range(2)]
    out = torch.empty(n, device=dev)
    for j in range(2):
        codec.wavedec(x[j], level, x0=x0[j], coeffs_x=wx[j], coeffs_diff=wc[j], wavelet=name)
        codec.waverec(wx[j], n, level, out=out, wavelet=name)
    torch.cuda.synchronize()
    with codec.KernelTimer() as kt:
        for i in range(10):
            codec.wavedec(x[i % 2], level, x0=x0[i % 2], coeffs_x=wx[i % 2], coeffs_diff=wc[i % 2],
                          wavelet=name)
            codec.waverec(wx[i % 2], n, level, out=out, wavelet=name)
        torch.cuda.synchronize()
    r = {k: round(ms / c * 1e3, 1) for k, (ms, c) in kt.result.items()}
    res[f"{name}/L{level}"] = {"pair_us": r.get("dwt"), "idwt_us": r.get("idwt"),
                               "filter_len": codec.filter_len(name)}
print(json.dumps(res))
