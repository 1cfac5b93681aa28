"""Phase timeline of one sampled top-k encode (sample -> filter -> select -> compact) from the
s_memrealtime stamps of the diagnostic build (make -C decentralizepy_amd/csrc stamps).  Times in
us from the sample kernel's first block; per stamp row: min / median / max over blocks, so the
gap between one kernel's last block and the next kernel's first block is visible.  Usage:
encode_timeline.py [n] [foldbase].  Diagnostic only."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["DPZ_CODEC_LIB"] = os.path.join(ROOT, "decentralizepy_amd", "libdpzcodec_stamps.so")
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from decentralizepy_amd import _lib, codec  # noqa: E402

ROWS = (("sample", [13, 14]), ("filter", [5, 6, 7]), ("select", [8, 12, 9, 10, 11]), ("compact", [0, 1, 2, 3, 4]))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 11_000_000
    fbase = len(sys.argv) > 2 and sys.argv[2] == "foldbase"
    L = _lib.lib()
    L.dpz_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.dpz_debug_block_stamps.argtypes = [ctypes.c_void_p]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    sets = []
    for _ in range(6):
        x = torch.randn(n, device=dev, generator=g)
        sets.append((x, x - 0.01 * torch.randn(n, device=dev, generator=g)))
    ws = codec.Workspace(dev)
    k = round(0.01 * n)
    idx = torch.empty(k, dtype=torch.int32, device=dev)
    val = torch.empty(k, dtype=torch.float32, device=dev)
    cnt = torch.zeros(n, dtype=torch.int32, device=dev)
    base = torch.empty(n, dtype=torch.float32, device=dev)
    for it in range(10):
        x, x0 = sets[it % 6]
        torch.cuda.synchronize()
        L.dpz_debug_stamps(None, 1)
        bs = (ctypes.c_ulonglong * (16 * 4096))()
        codec.topk_encode(x, k, x0=x0, idx_out=idx, val_out=val, counter=cnt, workspace=ws,
                          asynchronous=True,
                          fold_base=(base, [0.5], 0.5) if fbase else None)
        torch.cuda.synchronize()
        arr = (ctypes.c_ulonglong * 64)()
        L.dpz_debug_stamps(ctypes.addressof(arr), 0)
        L.dpz_debug_block_stamps(ctypes.addressof(bs))
        t0 = arr[0]
        ball = np.frombuffer(bs, dtype=np.uint64).reshape(16, 4096).astype(np.int64)
        if it < 4:
            continue
        out = [f"iter {it}:"]
        for name, rows in ROWS:
            for r in rows:
                v = ball[r]
                v = v[v >= t0]  # this call's stamps only
                if len(v):
                    rel = (v - t0) / 100.0
                    out.append(f"{name}[{r}] {rel.min():.1f}/{np.median(rel):.1f}/{rel.max():.1f}")
        print("  ".join(out), flush=True)


if __name__ == "__main__":
    main()
