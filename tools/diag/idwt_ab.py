"""Diagnostic A/B of IDWT builds: for the library named by DPZ_CODEC_LIB (tools/diag/variants),
the waverec output hash at several sizes (must equal the product build's) and the kernel time
at N = 25 M (HBM-rotated coefficients).  One JSON line."""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, ".")
from decentralizepy_amd import codec  # noqa: E402

WV = sys.argv[1] if len(sys.argv) > 1 else "sym2"
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(3)
hashes = {}
for n in (1_000_003, 70_001, 4_096 * 3 + 7, 25_000_000):
    for lev in (4, 2):
        m = codec.wavedec_len(n, lev, WV)
        c = torch.randn(m, device=dev, generator=g)
        o = codec.waverec(c, n, lev, wavelet=WV)
        hashes[f"{n}/{lev}"] = hashlib.sha256(o.cpu().numpy().tobytes()).hexdigest()[:16]
n = 25_000_000
m = codec.wavedec_len(n, 4, WV)
R = 4
cs = [torch.randn(m, device=dev, generator=g) for _ in range(R)]
outs = [torch.empty(n, device=dev) for _ in range(R)]
for i in range(R):
    codec.waverec(cs[i], n, 4, out=outs[i], wavelet=WV)
with codec.KernelTimer() as kt:
    torch.cuda._sleep(int(50e6))
    for i in range(40):
        codec.waverec(cs[i % R], n, 4, out=outs[i % R], wavelet=WV)
    torch.cuda.synchronize()
ms, cnt = kt.result["haar" if WV == "haar" else "idwt"]
us = ms / cnt * 1e3
print(json.dumps({"lib": os.path.basename(os.environ.get("DPZ_CODEC_LIB", "product")),
                  "wavelet": WV, "idwt_us": round(us, 1), "GBps": round((4 * m + 4 * n) / us / 1e3),
                  "hashes": hashes}), flush=True)
