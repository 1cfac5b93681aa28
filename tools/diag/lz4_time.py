"""Diagnostic: LZ4 decode breakdown on a C2 index payload (kernel time vs host call time)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from decentralizepy_amd import codec  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(13)
n, k = 11_000_000, 110_000
idx = torch.sort(torch.randperm(n, device=dev, generator=g)[:k])[0].to(torch.int32)
ws = codec.Workspace(dev)
gaps = codec.delta_i32(idx)
frame = codec.lz4_compress(gaps.view(torch.uint8), workspace=ws).cpu().numpy().tobytes()
print("frame", len(frame), "blocks", codec.lz4_frame_info(frame))
for _ in range(3):
    codec.lz4_decompress(frame, dev, workspace=ws)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    codec.lz4_decompress(frame, dev, workspace=ws)
torch.cuda.synchronize()
print("host call us", (time.perf_counter() - t0) / 20 * 1e6)
with codec.KernelTimer() as kt:
    for _ in range(20):
        codec.lz4_decompress(frame, dev, workspace=ws)
    torch.cuda.synchronize()
print({nm: (round(ms / c * 1e3, 1), c // 20) for nm, (ms, c) in kt.result.items()})
d = torch.frombuffer(bytearray(frame), dtype=torch.uint8)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    d.to(dev)
torch.cuda.synchronize()
print("h2d of the frame us", (time.perf_counter() - t0) / 20 * 1e6)
