"""Per-phase wall time of the batched fold at the C3 shape (16 payloads x alpha over 25,000,009
coefficients) from s_memrealtime stamps (100 MHz) in the diagnostic build
decentralizepy_amd/libdpzcodec_stamps.so (make -C decentralizepy_amd/csrc stamps).
Phases per (block, tile iteration): 0 tile start, 1 ranges visible, 2 entries scattered,
3 base fold done, 4 exact hit fold done, 5 stored."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["DPZ_CODEC_LIB"] = os.path.join(ROOT, "decentralizepy_amd", "libdpzcodec_stamps.so")
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from decentralizepy_amd import _lib, codec  # noqa: E402


def main():
    alpha = float(sys.argv[1]) if len(sys.argv) > 1 else 0.01
    npay = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    L = _lib.lib()
    L.dpz_debug_fold_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.dpz_debug_fold_stamps.restype = ctypes.c_int
    dev = torch.device("cuda:0")
    m = 25_000_009
    k = round(alpha * m)
    g = torch.Generator(device=dev).manual_seed(1)
    pays = []
    for _ in range(npay):
        idx = torch.sort(torch.randperm(m, device=dev, generator=g)[:k])[0].to(torch.int32)
        pays.append((idx, torch.randn(k, device=dev, generator=g)))
    locs = [torch.randn(m, device=dev, generator=g) for _ in range(3)]
    out = torch.empty(m, device=dev)
    w = [1 / (npay + 1)] * npay
    ws = codec.Workspace(dev)
    buf = np.zeros((6, 8192), dtype=np.uint64)
    for i in range(6):
        L.dpz_debug_fold_stamps(None, 1)
        torch.cuda.synchronize()
        codec.decode_average(locs[i % 3], pays, w, 1 / (npay + 1), out=out, workspace=ws)
        torch.cuda.synchronize()
    L.dpz_debug_fold_stamps(buf.ctypes.data, 0)
    st = buf.astype(np.int64).reshape(6, 512, 16)
    ok = (st[0] > 0) & (st[1] > 0) & (st[5] > 0)  # the phase path stamps 0, 1, 5 only
    t0 = st[0][ok].min()
    print(f"alpha={alpha} npay={npay}: span {(st[5][ok].max() - t0) / 100:.1f} us, "
          f"{ok.sum()} (block, iteration) samples")
    marks = [0, 1, 2, 3, 4, 5] if (st[2][ok] > 0).all() else [0, 1, 5]
    for a, b in zip(marks[:-1], marks[1:]):
        v = (st[b] - st[a])[ok] / 100.0
        print(f"  phase {a}->{b}: mean {v.mean():6.2f} us  p50 {np.median(v):6.2f}  "
              f"p90 {np.percentile(v, 90):6.2f}")
    it = (st[5] - st[0])[ok] / 100.0
    print(f"  tile iteration: mean {it.mean():.2f} us; iterations per block "
          f"{ok.sum(axis=1).mean():.1f}")
    gap = (st[0][:, 1:] - st[5][:, :-1])[ok[:, 1:] & ok[:, :-1]] / 100.0
    print(f"  between iterations: mean {gap.mean():.2f} us")


if __name__ == "__main__":
    main()
