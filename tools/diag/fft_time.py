"""Device time of dpz_rfft / dpz_irfft (HIP events around 20 back-to-back calls on rotated inputs)
at the FFT workload sizes, for each tile configuration (DPZ_FFT_ELEMS / DPZ_FFT_BMAX) and hipFFT
(DPZ_FFT_LIB=1).  Run with DPZ_CODEC_LIB=decentralizepy_amd/libdpzcodec_diag.so.  One JSON line
per size."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from decentralizepy_amd import codec  # noqa: E402

CONFIGS = [("lib", {"DPZ_FFT_LIB": "1"}), ("default", {}),
           ("pingpong", {"DPZ_FFT_INPLACE": "0"}), ("pair_sep", {"DPZ_FFT_PAIR_FUSED": "0"}),
           ("pack128", {"DPZ_FFT_PACK": "128"}), ("pack64", {"DPZ_FFT_PACK": "64"}),
           ("e4096_b16", {"DPZ_FFT_ELEMS": "4096", "DPZ_FFT_BMAX": "16"}),
           ("e2048_b8", {"DPZ_FFT_ELEMS": "2048", "DPZ_FFT_BMAX": "8"})]
if os.environ.get("FFT_CONFIGS") == "short":
    CONFIGS = CONFIGS[:4]
elif os.environ.get("FFT_CONFIGS") == "pack":
    CONFIGS = [CONFIGS[1], CONFIGS[4], CONFIGS[5], ("default_again", {})]


def main():
    dev = torch.device("cuda:0")
    sizes = [int(a) for a in sys.argv[1:]] or [11_000_000, 25_000_000, 1 << 24]
    reps, R = 20, 3
    for n in sizes:
        g = torch.Generator(device=dev).manual_seed(1)
        xs = [torch.randn(n, device=dev, generator=g) for _ in range(R)]
        outs = [torch.empty(n, device=dev) for _ in range(R)]
        row = {"n": n}
        for name, env in CONFIGS:
            for k_ in ("DPZ_FFT_LIB", "DPZ_FFT_ELEMS", "DPZ_FFT_BMAX", "DPZ_FFT_INPLACE",
                       "DPZ_FFT_PAIR_FUSED", "DPZ_FFT_PACK"):
                os.environ.pop(k_, None)
            os.environ.update(env)
            ws = codec.Workspace(dev)
            specs = [codec.rfft(x, workspace=ws) for x in xs]
            bufs = [s.clone() for s in specs]

            def t_of(fn):
                fn(0)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(reps):
                    fn(i)
                e1.record()
                torch.cuda.synchronize()
                return e0.elapsed_time(e1) / reps * 1e3

            tr = t_of(lambda i: codec.rfft(xs[i % R], out=specs[i % R], workspace=ws))
            tc = t_of(lambda i: bufs[i % R].copy_(specs[i % R]))

            def inv(i):
                bufs[i % R].copy_(specs[i % R])
                codec.irfft(bufs[i % R], n, out=outs[i % R], workspace=ws)
            ti = t_of(inv) - tc
            err = float((outs[0] - xs[0]).abs().max())
            row[name] = {"rfft_us": round(tr, 2), "irfft_us": round(ti, 2), "roundtrip_err": err}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
