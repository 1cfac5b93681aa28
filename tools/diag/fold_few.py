"""The plugin-path fold of a node's few neighbours (PartialModel payloads over the node's model,
sharing/Sharing.py:156-190): 1 and 3 sparse payloads at alpha 0.01 over N = 11 M and 16.8 M,
per fold kind (DPZ_FOLD_KIND 0 = auto (walk), 1 = hit-chain / phase; run with DPZ_CODEC_LIB=
decentralizepy_amd/libdpzcodec_diag.so), beside the replace decode and a torch copy of the same
bytes.  HBM-rotated locals; kernel averages from library event pairs.  One JSON line per case."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from decentralizepy_amd import codec  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    for n in (11_000_000, 16_777_216):
        k = round(0.01 * n)
        g = torch.Generator(device=dev).manual_seed(1)
        R = 6
        locs = [torch.randn(n, device=dev, generator=g) for _ in range(R)]
        outs = [torch.empty(n, device=dev) for _ in range(R)]
        pays = []
        for _ in range(4):
            idx = torch.sort(torch.randperm(n, device=dev, generator=g)[:k])[0].to(torch.int32)
            pays.append((idx, torch.randn(k, device=dev, generator=g)))
        ws = codec.Workspace(dev)
        res = {}
        for npay in (1, 3, 4):
            w = [1 / (npay + 1)] * npay
            for kind in ("0", "1"):
                os.environ["DPZ_FOLD_KIND"] = kind
                for i in range(R):
                    codec.decode_average(locs[i], pays[:npay], w, 1 / (npay + 1), out=outs[i],
                                         workspace=ws)
                torch.cuda.synchronize()
                with codec.KernelTimer() as kt:
                    torch.cuda._sleep(int(20e6))
                    for _ in range(4):
                        for i in range(R):
                            codec.decode_average(locs[i], pays[:npay], w, 1 / (npay + 1),
                                                 out=outs[i], workspace=ws)
                    torch.cuda.synchronize()
                res[f"fold{npay}_kind{kind}"] = {nm: round(ms / c * 1e3, 2)
                                                 for nm, (ms, c) in kt.result.items()}
        os.environ.pop("DPZ_FOLD_KIND", None)
        with codec.KernelTimer() as kt:
            torch.cuda._sleep(int(20e6))
            for _ in range(4):
                for i in range(R):
                    codec.replace(locs[i], pays[0][0], pays[0][1], out=outs[i], workspace=ws)
            torch.cuda.synchronize()
        res["replace"] = {nm: round(ms / c * 1e3, 2) for nm, (ms, c) in kt.result.items()}
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(4):
            for i in range(R):
                outs[i].copy_(locs[i])
        ev[1].record()
        torch.cuda.synchronize()
        res["torch_copy_us"] = round(ev[0].elapsed_time(ev[1]) * 1e3 / (4 * R), 2)
        print(json.dumps({"n": n, "alpha": 0.01, "us": res}), flush=True)


if __name__ == "__main__":
    main()
