"""The C4 gossip round (bench.gossip_case, all-gather mode, 1 GPU, 96_regular x 11M) with the
guarded round (no host wait between encodes and folds, gossip.py _step_guarded) and the
host-checked round (guarded=False), alternating on the same box.  One JSON line per run."""
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
    for guarded in (True, False):
        r = bench.gossip_case(11_000_000, 0.01, dev, 0, 1, None,
                              rounds=int(os.environ.get("ROUNDS", "10")), warmup=2,
                              engine_kw={"guarded": guarded})
        print(json.dumps({"guarded": guarded, "rep": rep, "ms_per_round": round(r["s_step"] * 1e3, 4),
                          "legs_ms": r["legs_ms"]}), flush=True)
        torch.cuda.empty_cache()
