"""Per-kernel wall-time breakdown of one sampled top-k encode from s_memrealtime stamps.

Uses the diagnostic build decentralizepy_amd/libdpzcodec_stamps.so (make -C decentralizepy_amd/csrc stamps).
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["DPZ_CODEC_LIB"] = os.path.join(ROOT, "decentralizepy_amd", "libdpzcodec_stamps.so")
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from decentralizepy_amd import _lib, codec  # noqa: E402

NAMES = {0: "sample first-in", 1: "sample last-out", 2: "filter first-in", 3: "filter last-out",
         6: "select first-in", 7: "select last-out", 13: "compact first-in"}
PHASES = ["entry", "loads", "counted", "end"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 11_000_000
    L = _lib.lib()
    L.dpz_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.dpz_debug_stamps.restype = ctypes.c_int
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    sets = []  # rotated so that every encode streams from HBM (6 x 8n bytes > the 256 MiB L3)
    for _ in range(6):
        x = torch.randn(n, device=dev, generator=g)
        sets.append((x, x - 0.01 * torch.randn(n, device=dev, generator=g)))
    ws = codec.Workspace(dev)
    k = round(0.01 * n)
    idx = torch.empty(k, dtype=torch.int32, device=dev)
    val = torch.empty(k, dtype=torch.float32, device=dev)
    for it in range(12):
        x, x0 = sets[it % 6]
        torch.cuda.synchronize()
        L.dpz_debug_stamps(None, 1)
        codec.topk_encode(x, k, x0=x0, idx_out=idx, val_out=val, workspace=ws, asynchronous=True)
        torch.cuda.synchronize()
        arr = (ctypes.c_ulonglong * 64)()
        L.dpz_debug_stamps(ctypes.addressof(arr), 0)
        t0 = arr[0]
        line = "  ".join(f"{NAMES[i]}={(arr[i] - t0) / 100:.1f}" for i in sorted(NAMES) if 0 < arr[i] < 2**63)
        print(f"iter {it}: (us from sample start) {line}")
        if it == 11:
            import numpy as np
            L.dpz_debug_block_stamps.argtypes = [ctypes.c_void_p]
            bs = (ctypes.c_ulonglong * (16 * 4096))()
            L.dpz_debug_block_stamps(ctypes.addressof(bs))
            ball = np.frombuffer(bs, dtype=np.uint64).reshape(16, 4096).astype(np.int64)
            sel = ball[8:12]
            ns = int((sel[0] > 0).sum())
            rs = ball[12:15, 0]
            print(f"resolve: start->gathered {(rs[1]-rs[0])/100:.2f} us, ->T {(rs[2]-rs[1])/100:.2f}, ->end {(rs[2]-rs[0])/100:.2f}")
            sel = sel[:, :ns]
            print(f"select blocks: {ns}")
            sp = ["entry", "b*", "appended", "arrived"]
            for p in range(1, 4):
                d = (sel[p] - sel[p - 1]) / 100
                print(f"  {sp[p - 1]:>8} -> {sp[p]:<8} {d.mean():7.2f} {d.max():7.2f}")
            b = ball[:8]
            L.dpz_debug_filter_stamps.argtypes = [ctypes.c_void_p]
            fs = (ctypes.c_ulonglong * (6 * 8192))()
            L.dpz_debug_filter_stamps(ctypes.addressof(fs))
            f = np.frombuffer(fs, dtype=np.uint64).reshape(6, 8192).astype(np.int64)
            nw = int((f[0] > 0).sum())
            f = f[:, :nw]
            t0 = f[0].min()
            fp = ["entry", "pre-barrier", "post-barrier", "loop done", "flushed", "end"]
            print(f"filter waves: {nw}; start spread {(f[0].max()-t0)/100:.2f} us, last end {(f[5].max()-t0)/100:.2f} us")
            for p in range(1, 6):
                d = (f[p] - f[p - 1]) / 100
                print(f"  {fp[p - 1]:>12} -> {fp[p]:<12} mean {d.mean():6.2f}  p50 {np.median(d):6.2f}  max {d.max():6.2f}")
            w0 = f[:, 0::4]
            print(f"  wave0: entry->pre-barrier mean {((w0[1]-w0[0])/100).mean():.2f}; others {((f[1]-f[0])/100).mean():.2f}")
            life = (f[5] - f[0]) / 100
            print(f"  wave lifetime mean {life.mean():.2f} max {life.max():.2f}; end times p10/p50/p90 "
                  f"{np.percentile((f[5]-t0)/100, 10):.2f}/{np.percentile((f[5]-t0)/100, 50):.2f}/{np.percentile((f[5]-t0)/100, 90):.2f}")
            nblk = int((b[0] > 0).sum())
            b = b[:, :nblk]
            ok = b[3] > 0
            print(f"compact blocks: {nblk}; per-block phase latency (us, mean/max over blocks):")
            for p in range(1, 4):
                d = (b[p] - b[p - 1])[ok] / 100
                print(f"  {PHASES[p - 1]:>8} -> {PHASES[p]:<8} {d.mean():7.2f} {d.max():7.2f}")
            e = (b[0][ok] - b[0][ok].min()) / 100
            print(f"  block entry spread: {e.max():.2f} us; block start->end mean {((b[3]-b[0])[ok]/100).mean():.2f}")


if __name__ == "__main__":
    main()
