"""The sliced encode (dpz_topk_encode_sliced) at the C3 shape with and without the bit-sliced
counter update (planes=None: compact writes idx / val and the selection mask only) — what a
counter update deferred to the post-step pass would take out of compact.  Kernel averages
(library event pairs), HBM-rotated inputs.  One JSON line per alpha."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from decentralizepy_amd import codec  # noqa: E402

dev = torch.device("cuda", 0)
m = 25_000_009
R = 3
g = torch.Generator(device=dev).manual_seed(3)
wc = [0.01 * torch.randn(m, device=dev, generator=g) for _ in range(R)]
acc = [0.01 * torch.randn(m, device=dev, generator=g) for _ in range(R)]
wx = [torch.randn(m, device=dev, generator=g) for _ in range(R)]
nw = codec.mask_words(m)
for alpha in (0.01, 0.1):
    k = round(alpha * m)
    idx = torch.empty(k, dtype=torch.int32, device=dev)
    val = torch.empty(k, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    res = {"alpha": alpha}
    for planes_on in (True, False, True, False):
        planes = torch.zeros(32 * nw, dtype=torch.int32, device=dev) if planes_on else None
        mask = torch.zeros(nw, dtype=torch.int32, device=dev)
        ws = codec.Workspace(dev)

        def enc(j):
            codec.topk_encode_sliced(wc[j], k, mask, planes, acc=acc[j], acc_mode=codec.DPZ_ACC_ADD,
                                     vals_src=wx[j], idx_out=idx, val_out=val, workspace=ws,
                                     status_out=st)
        for j in range(R):
            enc(j)
        torch.cuda.synchronize()
        with codec.KernelTimer() as kt:
            torch.cuda._sleep(int(20e6))
            for i in range(30):
                enc(i % R)
            torch.cuda.synchronize()
        key = "planes" if planes_on else "no_planes"
        res.setdefault(key, []).append({nm: round(ms / c * 1e3, 2) for nm, (ms, c) in kt.result.items()})
    print(json.dumps(res), flush=True)
