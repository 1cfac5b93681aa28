"""The C4 gossip round (bench.gossip_case, all-gather mode, 1 GPU) with the library the
environment selects (DPZ_CODEC_LIB: e.g. tools/diag/variants/lib_r03.so built from an older
tree by build_variant.sh) — run once per library on the same box for a same-box A/B.
One JSON line: ms per round and the per-leg breakdown."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
# ENGINE_SLICED=1: the counters in bit-sliced form (gossip.py sliced_counter)
ekw = {"sliced_counter": True} if os.environ.get("ENGINE_SLICED") == "1" else None
r = bench.gossip_case(11_000_000, 0.01, dev, 0, 1, None, rounds=int(os.environ.get("ROUNDS", "10")),
                      warmup=2, engine_kw=ekw)
from decentralizepy_amd import codec  # noqa: E402
with codec.KernelTimer() as kt:
    bench.gossip_case(11_000_000, 0.01, dev, 0, 1, None, rounds=2, warmup=0, engine_kw=ekw)
    torch.cuda.synchronize()
kern = {nm: [round(ms / c * 1e3, 2), c] for nm, (ms, c) in kt.result.items()}
print(json.dumps({"lib": os.environ.get("DPZ_CODEC_LIB", "product"),
                  "ms_per_round": round(r["s_step"] * 1e3, 4), "legs_ms": r["legs_ms"],
                  "kernels_us_calls": kern}), flush=True)
