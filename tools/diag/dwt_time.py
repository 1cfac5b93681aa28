"""Diagnostic: DWT pair / IDWT kernel times at N = 25M (HBM-rotated inputs)."""
import sys

import torch

sys.path.insert(0, ".")
from decentralizepy_amd import codec  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1)
n = 25_000_000
m = codec.wavedec_len(n, 4)
R = 3
xs = [torch.randn(n, device=dev, generator=g) for _ in range(R)]
x0s = [torch.randn(n, device=dev, generator=g) for _ in range(R)]
wx = [torch.empty(m, device=dev) for _ in range(R)]
wc = [torch.empty(m, device=dev) for _ in range(R)]
out = [torch.empty(n, device=dev) for _ in range(R)]
for i in range(R):
    codec.wavedec(xs[i], 4, x0=x0s[i], coeffs_x=wx[i], coeffs_diff=wc[i])
with codec.KernelTimer() as kt:
    torch.cuda._sleep(int(50e6))
    for i in range(30):
        j = i % R
        codec.wavedec(xs[j], 4, x0=x0s[j], coeffs_x=wx[j], coeffs_diff=wc[j])
        codec.waverec(wx[j], n, 4, out=out[j])
    torch.cuda.synchronize()
r = {nm: round(ms / c * 1e3, 1) for nm, (ms, c) in kt.result.items()}
print(r, "dwt GB/s", round((8 * n + 8 * m) / r["dwt"] / 1e3), "idwt GB/s", round((4 * m + 4 * n) / r["idwt"] / 1e3))
