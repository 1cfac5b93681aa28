"""Merge-fold phase ablations (DPZ_MERGE_ABL, diagnostic build; timing only) at the C3 shape
(16 x alpha 0.01 over M = 25,000,009) and 3 x 0.01 at 64 MiB."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from decentralizepy_amd import codec  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    os.environ["DPZ_FOLD_KIND"] = "8"
    for m, alpha, npay in ((25_000_009, 0.01, 16), (16_777_216, 0.01, 3)):
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
        for ept in ("8",):
            for abl in ("0", "32", "1", "3", "7", "15", "31"):
                os.environ["DPZ_MERGE_ABL"] = abl
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
                res[f"ept{ept}_abl{abl}"] = round(ev[0].elapsed_time(ev[1]) * 1e3 / 24, 2)
        print(json.dumps({"m": m, "alpha": alpha, "npay": npay, "us": res}), flush=True)


if __name__ == "__main__":
    main()
