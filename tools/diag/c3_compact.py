"""A/B of the compact's counter update (DPZ_COUNTER_PLAIN 0 = memory-side atomics, 1 = gathered
read + plain store) at the C3 shape (M = 25,000,009 wavelet coefficients, ADD accumulation, the
encode of bench_workloads.c3_case) and at C2 / 64 MiB (PartialModel, no accumulation).
Per-kernel averages (library event pairs), HBM-rotated states.  One JSON object per line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from decentralizepy_amd import codec  # noqa: E402


def run(dev, n, alpha, acc_mode, R=3):
    k = round(alpha * n)
    g = torch.Generator(device=dev).manual_seed(2)
    sets = []
    for _ in range(R):
        x = torch.randn(n, device=dev, generator=g)
        sets.append(dict(x=x, x0=x - 0.01 * torch.randn(n, device=dev, generator=g),
                         acc=0.01 * torch.randn(n, device=dev, generator=g),
                         cnt=torch.zeros(n, dtype=torch.int32, device=dev),
                         idx=torch.empty(k, dtype=torch.int32, device=dev),
                         val=torch.empty(k, device=dev)))
    ws = codec.Workspace(dev)
    out = {}
    for plain in ("0", "1"):
        os.environ["DPZ_COUNTER_PLAIN"] = plain

        def enc(d):
            codec.topk_encode(d["x"], k, x0=d["x0"],
                              acc=d["acc"] if acc_mode else None, acc_mode=acc_mode,
                              counter=d["cnt"], idx_out=d["idx"], val_out=d["val"], workspace=ws,
                              asynchronous=True)
        for d in sets:
            enc(d)
        torch.cuda.synchronize()
        with codec.KernelTimer() as kt:
            torch.cuda._sleep(int(20e6))
            for _ in range(4):
                for d in sets:
                    enc(d)
            torch.cuda.synchronize()
        out[plain] = {nm: round(ms / c * 1e3, 2) for nm, (ms, c) in kt.result.items()}
        out[plain]["status"] = codec.topk_sticky_status(ws, clear=True)
    os.environ.pop("DPZ_COUNTER_PLAIN", None)
    return out


def main():
    dev = torch.device("cuda:0")
    for n, alpha, mode in ((25_000_009, 0.01, codec.DPZ_ACC_ADD), (25_000_009, 0.1, codec.DPZ_ACC_ADD),
                           (25_000_009, 0.3, codec.DPZ_ACC_ADD), (11_000_000, 0.01, 0),
                           (16_777_216, 0.01, 0)):
        print(json.dumps({"n": n, "alpha": alpha, "acc_mode": mode,
                          "kernels_us_event_pair": run(dev, n, alpha, mode)}), flush=True)


if __name__ == "__main__":
    main()
