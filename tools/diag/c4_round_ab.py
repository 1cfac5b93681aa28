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
# ENGINE_SLICED=0: the int32 counters (gossip.py sliced_counter, default on)
ekw = {"sliced_counter": os.environ.get("ENGINE_SLICED", "1") == "1"}
# ENGINE_RING=0: no ring of rounds (gossip.py ring_counter, default on): the sliced / int32 form
if os.environ.get("ENGINE_RING"):
    ekw["ring_counter"] = os.environ["ENGINE_RING"] == "1"
# NODE_GROUP / STREAMS: the node-batched encodes' group size and stream count (gossip.py defaults 4 / 3)
if os.environ.get("NODE_GROUP"):
    ekw["node_group"] = int(os.environ["NODE_GROUP"])
if os.environ.get("STREAMS"):
    ekw["streams"] = int(os.environ["STREAMS"])
r = bench.gossip_case(11_000_000, 0.01, dev, 0, 1, None, rounds=int(os.environ.get("ROUNDS", "10")),
                      warmup=2, engine_kw=ekw)
from decentralizepy_amd import codec  # noqa: E402
with codec.KernelTimer() as kt:
    bench.gossip_case(11_000_000, 0.01, dev, 0, 1, None, rounds=2, warmup=0, engine_kw=ekw)
    torch.cuda.synchronize()
kern = {nm: [round(ms / c * 1e3, 2), c] for nm, (ms, c) in kt.result.items()}
print(json.dumps({"lib": os.environ.get("DPZ_CODEC_LIB", "product"), "engine_kw": ekw,
                  "ms_per_round": round(r["s_step"] * 1e3, 4), "legs_ms": r["legs_ms"],
                  "kernels_us_calls": kern}), flush=True)
