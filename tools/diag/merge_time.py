"""Kernel time of the fold kinds at the C3 shape (16 sparse payloads over M = 25,000,009
coefficients) and the plugin's 3 payloads at 64 MiB: the merge fold (DPZ_FOLD_KIND=8, tile width
DPZ_MERGE_EPT 4 / 8 / 16) beside the walk (4) and the classic hit-chain / phase fold (1).  Run
with DPZ_CODEC_LIB=decentralizepy_amd/libdpzcodec_diag.so.  One JSON line per case."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from decentralizepy_amd import codec  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    cases = [(25_000_009, 0.005, 16), (25_000_009, 0.01, 16), (25_000_009, 0.02, 16),
             (25_000_009, 0.03, 16), (25_000_009, 0.05, 16), (25_000_009, 0.01, 8),
             (25_000_009, 0.01, 5), (11_000_000, 0.01, 16), (16_777_216, 0.01, 3)]
    kinds = [("8", "8"), ("4", "8"), ("1", "8")]
    for m, alpha, npay in cases:
        k = round(alpha * m)
        g = torch.Generator(device=dev).manual_seed(1)
        pays = []
        for _ in range(npay):
            idx = torch.sort(torch.randperm(m, device=dev, generator=g)[:k])[0].to(torch.int32)
            pays.append((idx, torch.randn(k, device=dev, generator=g)))
        locs = [torch.randn(m, device=dev, generator=g) for _ in range(4)]
        outs = [torch.empty(m, device=dev) for _ in range(4)]
        w = [1 / (npay + 1)] * npay
        ws = codec.Workspace(dev)
        res = {}
        for kind, ept in kinds:
            os.environ["DPZ_FOLD_KIND"] = kind
            os.environ["DPZ_MERGE_EPT"] = ept
            for i in range(4):
                codec.decode_average(locs[i], pays, w, 1 / (npay + 1), out=outs[i], workspace=ws)
            torch.cuda.synchronize()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            torch.cuda._sleep(int(20e6))
            ev[0].record()
            for i in range(24):
                codec.decode_average(locs[i % 4], pays, w, 1 / (npay + 1), out=outs[i % 4],
                                     workspace=ws)
            ev[1].record()
            torch.cuda.synchronize()
            us = ev[0].elapsed_time(ev[1]) * 1e3 / 24
            nm = {"8": f"merge{ept}", "4": "walk", "1": "classic"}[kind]
            res[nm] = round(us, 2)
        b = 8 * m + 8 * npay * k
        best = min(res.values())
        print(json.dumps({"m": m, "alpha": alpha, "npay": npay, "us": res,
                          "best_frac": round(b / (best * 1e-6) / 8e12, 4)}), flush=True)
    os.environ.pop("DPZ_FOLD_KIND", None)


if __name__ == "__main__":
    main()
