"""A/B of the counter update form at the PartialModel shapes (run with DPZ_CODEC_LIB=
decentralizepy_amd/libdpzcodec_diag.so): C2 (N = 11 M) and the 64 MiB tensor at alpha = 0.01,
change against x0, values from x: int32 counter with memory-side atomics (dpz_topk_encode),
the bit-sliced counter + selection mask (dpz_topk_encode_sliced), and no counter at all
(DPZ_COMPACT_ABLATE=2, a lower bound).  Per-kernel averages (library event pairs) over
HBM-rotated states; one JSON object per line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from decentralizepy_amd import codec  # noqa: E402


def run(dev, n, alpha, R=6):
    k = round(alpha * n)
    nw = codec.mask_words(n)
    g = torch.Generator(device=dev).manual_seed(1)
    sets = []
    for _ in range(R):
        x = torch.randn(n, device=dev, generator=g)
        sets.append(dict(x=x, x0=x - 0.01 * torch.randn(n, device=dev, generator=g),
                         cnt=torch.zeros(n, dtype=torch.int32, device=dev),
                         planes=torch.zeros(32 * nw, dtype=torch.int32, device=dev),
                         mask=torch.zeros(nw, dtype=torch.int32, device=dev),
                         idx=torch.empty(k, dtype=torch.int32, device=dev),
                         val=torch.empty(k, device=dev)))
    ws = codec.Workspace(dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    out = {}
    for form in ("atomic", "sliced", "none", "atomic"):
        os.environ["DPZ_COMPACT_ABLATE"] = "2" if form == "none" else "0"

        def enc(d):
            if form == "sliced":
                codec.topk_encode_sliced(d["x"], k, d["mask"], d["planes"], x0=d["x0"],
                                         idx_out=d["idx"], val_out=d["val"], workspace=ws,
                                         status_out=st)
            else:
                codec.topk_encode(d["x"], k, x0=d["x0"], counter=d["cnt"], idx_out=d["idx"],
                                  val_out=d["val"], workspace=ws, asynchronous=True)
        for d in sets:
            enc(d)
        torch.cuda.synchronize()
        with codec.KernelTimer() as kt:
            torch.cuda._sleep(int(20e6))
            for _ in range(5):
                for d in sets:
                    enc(d)
            torch.cuda.synchronize()
        out[form] = {nm: round(ms / c * 1e3, 2) for nm, (ms, c) in kt.result.items()}
    os.environ.pop("DPZ_COMPACT_ABLATE", None)
    out["status"] = codec.topk_sticky_status(ws, clear=True) | int(st.item())
    return out


def main():
    dev = torch.device("cuda:0")
    for n in (11_000_000, 16_777_216):
        print(json.dumps({"n": n, "alpha": 0.01, "kernels_us": run(dev, n, 0.01)}), flush=True)


if __name__ == "__main__":
    main()
