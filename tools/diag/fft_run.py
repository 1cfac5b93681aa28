"""rfft + irfft of one size, `reps` times back to back (the product library's default passes), for
rocprofv3 passes over the FFT kernels alone.  Usage: python tools/diag/fft_run.py [n] [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from decentralizepy_amd import codec  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 11_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(1)
    xs = [torch.randn(n, device=dev, generator=g) for _ in range(3)]
    out = torch.empty(n, device=dev)
    ws = codec.Workspace(dev)
    for i in range(reps):
        f = codec.rfft(xs[i % 3], workspace=ws)
        codec.irfft(f, n, out=out, workspace=ws)
    torch.cuda.synchronize()
    print("fft_run done", n, reps, flush=True)


if __name__ == "__main__":
    main()
