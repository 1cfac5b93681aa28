"""Diagnostic: bench.py's product_one_node (the plugin path: codec.topk_encode then
codec.decode_average over x, one stream) at C2 and 64 MiB, for A/B of diagnostic-build switches
(run with DPZ_CODEC_LIB=decentralizepy_amd/libdpzcodec_diag.so DPZ_<SWITCH>=...).  One JSON line
per size."""
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from decentralizepy_amd import codec  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
for n in (11_000_000, 16_777_216):
    k = round(0.01 * n)
    R = max(1, math.ceil(2 * bench.L3_BYTES / (16 * n + 8 * k)) + 1)
    g = torch.Generator(device=dev).manual_seed(5)
    sets = []
    for _ in range(R):
        x = torch.randn(n, device=dev, generator=g)
        sets.append(dict(x=x, x0=x - 0.01 * torch.randn(n, device=dev, generator=g),
                         counter=torch.zeros(n, dtype=torch.int32, device=dev),
                         idx=torch.empty(k, dtype=torch.int32, device=dev),
                         val=torch.empty(k, device=dev), out=torch.empty(n, device=dev)))
    st = torch.cuda.Stream(dev)
    flags = dict(hint=os.environ.get("AB_HINT", "1") != "0",
                 keep_x=os.environ.get("AB_KEEP_X", "1") != "0")
    res = [bench.product_one_node(sets, n, k, st, codec.Workspace(dev), 120, **flags)
           for _ in range(3)]
    best = {}
    for key in ("1_payload", "3_payload", "1_payload_foldbase", "3_payload_foldbase"):
        rs = sorted(res, key=lambda r: r[key]["step_us"])
        best[key] = rs[1][key]  # the median of three
    env = {kk: v for kk, v in os.environ.items() if kk.startswith(("DPZ_", "AB_"))}
    print(json.dumps({"n": n, "env": env, **best, "fell_back": any(r["fell_back"] for r in res)}),
          flush=True)
    del sets
    torch.cuda.empty_cache()
