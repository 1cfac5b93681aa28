"""A/B timing of the batched fold (dpz_decode_average) at the C3 shape: 16 sparse payloads over
M = 25,000,009 coefficients.  Run twice, with and without DPZ_FOLD_PHASES=1."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from decentralizepy_amd import codec  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    m = 25_000_009
    for alpha, npay in ((0.01, 16), (0.02, 16), (0.03, 16), (0.04, 16), (0.1, 16), (0.2, 16), (0.4, 3)):
        k = round(alpha * m)
        g = torch.Generator(device=dev).manual_seed(1)
        pays = []
        for _ in range(npay):
            idx = torch.sort(torch.randperm(m, device=dev, generator=g)[:k])[0].to(torch.int32)
            pays.append((idx, torch.randn(k, device=dev, generator=g)))
        locs = [torch.randn(m, device=dev, generator=g) for _ in range(3)]
        outs = [torch.empty(m, device=dev) for _ in range(3)]
        w = [1 / (npay + 1)] * npay
        ws = codec.Workspace(dev)
        for i in range(5):
            codec.decode_average(locs[i % 3], pays, w, 1 / (npay + 1), out=outs[i % 3], workspace=ws)
        torch.cuda.synchronize()
        with codec.KernelTimer() as kt:
            for i in range(30):
                codec.decode_average(locs[i % 3], pays, w, 1 / (npay + 1), out=outs[i % 3],
                                     workspace=ws)
            torch.cuda.synchronize()
        res = {nm: round(ms / c * 1e3, 2) for nm, (ms, c) in kt.result.items()}
        print(f"group={os.environ.get('DPZ_FOLD_GROUP', 'auto')} alpha={alpha} npay={npay} {res}",
              flush=True)


if __name__ == "__main__":
    main()
