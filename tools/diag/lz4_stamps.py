"""Phase timeline of lz4_decode_par_kernel (s_memrealtime stamps, 100 MHz) on a C2 index frame,
from the diagnostic build decentralizepy_amd/libdpzcodec_stamps.so (make -C
decentralizepy_amd/csrc stamps): per phase, the median over blocks of the time since the
block's first stamp (us).  Diagnostic only."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["DPZ_CODEC_LIB"] = os.path.join(ROOT, "decentralizepy_amd", "libdpzcodec_stamps.so")
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from decentralizepy_amd import _lib, codec  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(13)
idx = torch.sort(torch.randperm(11_000_000, device=dev, generator=g)[:110_000])[0].to(torch.int32)
ws = codec.Workspace(dev)
frame = codec.lz4_compress(codec.delta_i32(idx).view(torch.uint8), workspace=ws).cpu().numpy().tobytes()
L = _lib.lib()
L.dpz_debug_lz4_stamps.argtypes = [ctypes.c_void_p]
for _ in range(3):
    codec.lz4_decompress(frame, dev, workspace=ws)
torch.cuda.synchronize()
buf = np.zeros((10, 512), dtype=np.uint64)
L.dpz_debug_lz4_stamps(buf.ctypes.data)
st = buf.astype(np.int64)
nb = codec.lz4_frame_info(frame)[1]
st = st[:, :nb]
rel = (st - st[0]) / 100.0
print("blocks", nb, "kernel span us", (st[9].max() - st[0].min()) / 100.0)
for i in range(1, 10):
    print(f"phase<= {i}: median {np.median(rel[i]):.2f} us, max {rel[i].max():.2f}")
