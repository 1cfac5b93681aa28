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
         4: "selA first-in", 5: "selA last-out", 6: "selB first-in", 7: "selB last-out",
         8: "selC start", 9: "selC loads done", 10: "selC gathered", 11: "selC radix done",
         12: "selC end", 13: "compact first-in"}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 11_000_000
    L = _lib.lib()
    L.dpz_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.dpz_debug_stamps.restype = ctypes.c_int
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(n, device=dev, generator=g)
    x0 = x - 0.01 * torch.randn(n, device=dev, generator=g)
    ws = codec.Workspace(dev)
    k = round(0.01 * n)
    idx = torch.empty(k, dtype=torch.int32, device=dev)
    val = torch.empty(k, dtype=torch.float32, device=dev)
    for it in range(6):
        torch.cuda.synchronize()
        L.dpz_debug_stamps(None, 1)
        codec.topk_encode(x, k, x0=x0, idx_out=idx, val_out=val, workspace=ws, asynchronous=True)
        torch.cuda.synchronize()
        arr = (ctypes.c_ulonglong * 64)()
        L.dpz_debug_stamps(ctypes.addressof(arr), 0)
        t0 = arr[0]
        line = "  ".join(f"{NAMES[i]}={(arr[i] - t0) / 100:.1f}" for i in sorted(NAMES) if 0 < arr[i] < 2**63)
        print(f"iter {it}: (us from sample start) {line}")


if __name__ == "__main__":
    main()
