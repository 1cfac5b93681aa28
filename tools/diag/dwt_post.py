"""Diagnostic: the accumulating post-step DWT (acc += W(x_new - prev), optionally with the sliced
encode's rewind mask) against the plain single-output W(x - x0) and the pair W(x), W(x - x0),
N = 25 M, HBM-rotated inputs; kernel averages from library event pairs."""
import json
import sys

import torch

sys.path.insert(0, ".")
from decentralizepy_amd import codec  # noqa: E402

WV = sys.argv[1] if len(sys.argv) > 1 else "sym2"
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1)
n = 25_000_000
m = codec.wavedec_len(n, 4, WV)
R = 3
xs = [torch.randn(n, device=dev, generator=g) for _ in range(R)]
x0s = [torch.randn(n, device=dev, generator=g) for _ in range(R)]
acc = [torch.randn(m, device=dev, generator=g) for _ in range(R)]
wx = [torch.empty(m, device=dev) for _ in range(R)]
wc = [torch.empty(m, device=dev) for _ in range(R)]
mask = torch.zeros(codec.mask_words(m), dtype=torch.int32, device=dev)
res = {}
for name, fn in (
        ("pair", lambda j: codec.wavedec(xs[j], 4, x0=x0s[j], coeffs_x=wx[j], coeffs_diff=wc[j], wavelet=WV)),
        ("diff_only", lambda j: codec.wavedec(xs[j], 4, x0=x0s[j], want_x=False,
                                              coeffs_diff=wc[j], wavelet=WV)),
        ("accumulate", lambda j: codec.wavedec(xs[j], 4, x0=x0s[j], want_x=False,
                                               coeffs_diff=acc[j], accumulate=True, wavelet=WV)),
        ("accumulate_rewind", lambda j: codec.wavedec(xs[j], 4, x0=x0s[j], want_x=False,
                                                      coeffs_diff=acc[j], accumulate=True,
                                                      rewind_mask=mask, wavelet=WV))):
    for j in range(R):
        fn(j)
    torch.cuda.synchronize()
    with codec.KernelTimer() as kt:
        torch.cuda._sleep(int(20e6))
        for i in range(30):
            fn(i % R)
        torch.cuda.synchronize()
    res[name] = {nm: round(ms / c * 1e3, 1) for nm, (ms, c) in kt.result.items()}
res["wavelet"] = WV
print(json.dumps(res))
