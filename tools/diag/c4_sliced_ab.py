"""The C4 gossip round (bench.gossip_case, all-gather mode, 1 GPU, 96_regular x 11M) with every
node's counter in bit-sliced form (DPZ_TOPK_SLICED: compact writes a selection mask and adds it to
the counter planes) and with the int32 counter (k scattered atomics per node), alternating on the
same box.  One JSON line per run."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
for rep in range(int(os.environ.get("REPS", "3"))):
    for sliced in (True, False):
        r = bench.gossip_case(11_000_000, 0.01, dev, 0, 1, None,
                              rounds=int(os.environ.get("ROUNDS", "10")), warmup=2,
                              engine_kw={"sliced_counter": sliced})
        print(json.dumps({"sliced_counter": sliced, "rep": rep, "ms_per_round": round(r["s_step"] * 1e3, 4),
                          "legs_ms": r["legs_ms"]}), flush=True)
        torch.cuda.empty_cache()
