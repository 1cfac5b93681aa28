"""Per-side-effect cost of the C3 compact (run with DPZ_CODEC_LIB=decentralizepy_amd/
libdpzcodec_diag.so): the encode of bench_workloads.c3_case at ALPHA (default 0.1) on the
M = 25,000,009 coefficients of a 25 M model, with DPZ_COMPACT_ABLATE = 0 (full), 1 (no acc
rewind), 2 (no counter), 3 (neither), and with the values taken from the key operand itself
(vals = W(x - x0): the filter carries them, no gather).  Ablated runs differ from the reference
by construction; only their kernel times are of interest.  One JSON object per line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from decentralizepy_amd import codec  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    m = 25_000_009
    alpha = float(os.environ.get("ALPHA", "0.1"))
    k = round(alpha * m)
    g = torch.Generator(device=dev).manual_seed(3)
    R = 4
    sets = [dict(wc=0.01 * torch.randn(m, device=dev, generator=g),
                 wx=torch.randn(m, device=dev, generator=g),
                 acc=0.01 * torch.randn(m, device=dev, generator=g),
                 cnt=torch.zeros(m, dtype=torch.int32, device=dev),
                 idx=torch.empty(k, dtype=torch.int32, device=dev),
                 val=torch.empty(k, device=dev)) for _ in range(R)]
    ws = codec.Workspace(dev)
    for ablate, vals in (("0", "wx"), ("1", "wx"), ("2", "wx"), ("3", "wx"), ("0", "wc"),
                         ("3", "wc"), ("0", "wx")):
        os.environ["DPZ_COMPACT_ABLATE"] = ablate

        def enc(d):
            codec.topk_encode(d["wc"], k, acc=d["acc"], acc_mode=codec.DPZ_ACC_ADD,
                              vals_src=d[vals], counter=d["cnt"], idx_out=d["idx"],
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
        res = {nm: round(ms / c * 1e3, 2) for nm, (ms, c) in kt.result.items()}
        print(json.dumps({"alpha": alpha, "ablate": int(ablate), "vals": vals, "kernels_us": res,
                          "status": codec.topk_sticky_status(ws, clear=True)}), flush=True)
    os.environ.pop("DPZ_COMPACT_ABLATE", None)
    # the coalesced side effects (dpz_topk_encode_sliced): bit-sliced counter + selection mask
    nw = codec.mask_words(m)
    for d in sets:
        d["planes"] = torch.zeros(32 * nw, dtype=torch.int32, device=dev)
        d["mask"] = torch.zeros(nw, dtype=torch.int32, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)

    def enc_sl(d):
        codec.topk_encode_sliced(d["wc"], k, d["mask"], d["planes"], acc=d["acc"],
                                 acc_mode=codec.DPZ_ACC_ADD, vals_src=d["wx"], idx_out=d["idx"],
                                 val_out=d["val"], workspace=ws, status_out=st)
    for _ in range(3):
        for d in sets:
            enc_sl(d)
    torch.cuda.synchronize()
    with codec.KernelTimer() as kt:
        torch.cuda._sleep(int(20e6))
        for _ in range(5):
            for d in sets:
                enc_sl(d)
        torch.cuda.synchronize()
    res = {nm: round(ms / c * 1e3, 2) for nm, (ms, c) in kt.result.items()}
    print(json.dumps({"alpha": alpha, "sliced": True, "vals": "wx", "kernels_us": res,
                      "status": int(st.item())}), flush=True)


if __name__ == "__main__":
    main()
