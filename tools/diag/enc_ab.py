"""The PartialModel encode alone (dpz_topk_encode: x, x0, counter, values from x) at C2 and
64 MiB, one stream, HBM-rotated states, with the library DPZ_CODEC_LIB selects — run once per
library on the same box (e.g. tools/diag/variants/lib_r03.so) for a same-box per-kernel A/B."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from decentralizepy_amd import codec  # noqa: E402

dev = torch.device("cuda:0")
for n in (11_000_000, 16_777_216):
    k = round(0.01 * n)
    g = torch.Generator(device=dev).manual_seed(1)
    sets = []
    for _ in range(6):
        x = torch.randn(n, device=dev, generator=g)
        sets.append(dict(x=x, x0=x - 0.01 * torch.randn(n, device=dev, generator=g),
                         cnt=torch.zeros(n, dtype=torch.int32, device=dev),
                         idx=torch.empty(k, dtype=torch.int32, device=dev),
                         val=torch.empty(k, device=dev)))
    ws = codec.Workspace(dev)

    def enc(d):
        codec.topk_encode(d["x"], k, x0=d["x0"], counter=d["cnt"], idx_out=d["idx"],
                          val_out=d["val"], workspace=ws, asynchronous=True)
    for d in sets:
        enc(d)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(10):
        for d in sets:
            enc(d)
    ev[1].record()
    torch.cuda.synchronize()
    with codec.KernelTimer() as kt:
        torch.cuda._sleep(int(20e6))
        for _ in range(5):
            for d in sets:
                enc(d)
        torch.cuda.synchronize()
    print(json.dumps({"lib": os.path.basename(os.environ.get("DPZ_CODEC_LIB", "product")), "n": n,
                      "encode_us": round(ev[0].elapsed_time(ev[1]) * 1e3 / 60, 2),
                      "kernels_us": {nm: round(ms / c * 1e3, 2) for nm, (ms, c) in kt.result.items()},
                      "status": codec.topk_sticky_status(ws, clear=True)}), flush=True)
