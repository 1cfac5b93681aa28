"""Diagnostic: host costs of bringing a device byte stream (a full-share float stream, ~88 MB)
back as an owned numpy array: .cpu() (pageable) vs D2H into a kept pinned buffer + numpy copy."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np
import torch

from decentralizepy_amd import codec  # noqa: E402

dev = torch.device("cuda", 0)
x = torch.randn(25_000_009, device=dev)
ws = codec.Workspace(dev)
res = {}
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s = codec.fpz_encode(x, 0, workspace=ws)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    a = s.cpu().numpy()
    t2 = time.perf_counter()
    pin = torch.empty(s.numel(), dtype=torch.uint8, pin_memory=True) if rep == 0 else pin
    t3 = time.perf_counter()
    pin.copy_(s, non_blocking=True)
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    b = pin.numpy().copy()
    t5 = time.perf_counter()
    res[rep] = {"bytes": int(s.numel()), "fpz_encode_ms": (t1 - t0) * 1e3, "cpu_ms": (t2 - t1) * 1e3,
                "pinned_d2h_ms": (t4 - t3) * 1e3, "np_copy_ms": (t5 - t4) * 1e3}
print(json.dumps(res))
