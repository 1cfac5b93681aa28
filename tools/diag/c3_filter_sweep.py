"""C3 encode filter shape sweep (run with DPZ_CODEC_LIB=decentralizepy_amd/libdpzcodec_diag.so):
the ADD-accumulation pipelined filter over M = 25,000,009 coefficients at alpha 0.1 and 0.01 with
DPZ_WLONE (segments) x DPZ_FILTER_DEPTH; sliced encode as the JWINS plugin runs it.  Per-kernel
averages (library event pairs), HBM-rotated states.  One JSON line per setting."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from decentralizepy_amd import codec  # noqa: E402

dev = torch.device("cuda:0")
m = 25_000_009
g = torch.Generator(device=dev).manual_seed(3)
R = 4
nw = codec.mask_words(m)
sets = [dict(wc=0.01 * torch.randn(m, device=dev, generator=g),
             wx=torch.randn(m, device=dev, generator=g),
             acc=0.01 * torch.randn(m, device=dev, generator=g),
             planes=torch.zeros(32 * nw, dtype=torch.int32, device=dev),
             mask=torch.zeros(nw, dtype=torch.int32, device=dev)) for _ in range(R)]
st = torch.zeros(1, dtype=torch.int32, device=dev)
for alpha in (0.1, 0.01):
    k = round(alpha * m)
    for d in sets:
        d["idx"] = torch.empty(k, dtype=torch.int32, device=dev)
        d["val"] = torch.empty(k, device=dev)
    ws = codec.Workspace(dev)
    for wl, depth in ((0, 4), (4096, 4), (4096, 6), (4096, 8), (6144, 4), (3072, 4), (2048, 8)):
        os.environ["DPZ_WLONE"] = str(wl)
        os.environ["DPZ_FILTER_DEPTH"] = str(depth)

        def enc(d):
            codec.topk_encode_sliced(d["wc"], k, d["mask"], d["planes"], acc=d["acc"],
                                     acc_mode=codec.DPZ_ACC_ADD, vals_src=d["wx"],
                                     idx_out=d["idx"], val_out=d["val"], workspace=ws,
                                     status_out=st)
        for d in sets:
            enc(d)
        torch.cuda.synchronize()
        with codec.KernelTimer() as kt:
            torch.cuda._sleep(int(20e6))
            for _ in range(5):
                for d in sets:
                    enc(d)
            torch.cuda.synchronize()
        res = {nm: round(ms / c * 1e3, 2) for nm, (ms, c) in kt.result.items()}
        tot = round(sum(res.values()), 1)
        print(json.dumps({"alpha": alpha, "wlone": wl, "depth": depth, "kernels_us": res,
                          "sum_us": tot, "status": int(st.item())}), flush=True)
