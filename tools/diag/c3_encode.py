"""The C3 encode alone (bench_workloads.c3_case's encode: one DWT launch W(x), W(x - x0), then
top-k of |W(x - x0) + acc| with ADD accumulation, values gathered from W(x), counter and acc
rewind), ALPHA (default 0.1) at N = 25 M parameters, over HBM-rotated states; optionally the
16-payload fold + IDWT too (DECODE=1).  For rocprofv3 traces and PMC passes of those kernels."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from decentralizepy_amd import codec  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    n, level, wavelet = 25_000_000, 4, "sym2"
    alpha = float(os.environ.get("ALPHA", "0.1"))
    iters = int(os.environ.get("ITERS", "40"))
    m = codec.wavedec_len(n, level, wavelet)
    k = round(alpha * m)
    g = torch.Generator(device=dev).manual_seed(3)
    R = 3
    sets = []
    for _ in range(R):
        x = torch.randn(n, device=dev, generator=g)
        sets.append(dict(x=x, x0=x - 0.01 * torch.randn(n, device=dev, generator=g),
                         acc=0.01 * torch.randn(m, device=dev, generator=g),
                         cnt=torch.zeros(m, dtype=torch.int32, device=dev),
                         wx=torch.empty(m, device=dev), wc=torch.empty(m, device=dev),
                         idx=torch.empty(k, dtype=torch.int32, device=dev),
                         val=torch.empty(k, device=dev), tot=torch.empty(m, device=dev),
                         out=torch.empty(n, device=dev)))
    pays = []
    if os.environ.get("DECODE") == "1":
        for _ in range(16):
            idx = torch.sort(torch.randperm(m, device=dev, generator=g)[:k])[0].to(torch.int32)
            pays.append((idx, torch.randn(k, device=dev, generator=g)))
    ws = codec.Workspace(dev)
    for i in range(iters):
        d = sets[i % R]
        codec.wavedec(d["x"], level, x0=d["x0"], coeffs_x=d["wx"], coeffs_diff=d["wc"],
                      wavelet=wavelet)
        codec.topk_encode(d["wc"], k, acc=d["acc"], acc_mode=codec.DPZ_ACC_ADD,
                          vals_src=d["wx"], counter=d["cnt"], idx_out=d["idx"],
                          val_out=d["val"], workspace=ws, asynchronous=True)
        if pays:
            codec.decode_average(d["wx"], pays, [1 / 17] * 16, 1 / 17, out=d["tot"], workspace=ws)
            codec.waverec(d["tot"], n, level, out=d["out"], wavelet=wavelet)
    torch.cuda.synchronize()
    print("status", codec.topk_sticky_status(ws, clear=True), "k", k, "m", m, flush=True)


if __name__ == "__main__":
    main()
