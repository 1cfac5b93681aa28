"""The C3 shape's 16-payload fold alone (M = 25,000,009 coefficients, 16 sparse payloads of
alpha = 0.01, equal weights), `reps` launches on rotated locals, for rocprofv3 passes over the
merge fold.  Usage: python tools/diag/fold16_run.py [alpha] [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from decentralizepy_amd import codec  # noqa: E402


def main():
    alpha = float(sys.argv[1]) if len(sys.argv) > 1 else 0.01
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda:0")
    m, npay = 25_000_009, 16
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
    for i in range(reps):
        codec.decode_average(locs[i % 4], pays, w, 1 / (npay + 1), out=outs[i % 4], workspace=ws)
    torch.cuda.synchronize()
    print("fold16_run done", alpha, reps, flush=True)


if __name__ == "__main__":
    main()
