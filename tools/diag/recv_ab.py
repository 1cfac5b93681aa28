"""Same-box A/B of the JWINS plugin round's receive leg: the asynchronous payload decode
(Elias.async_decode, one status check per round) against the synchronous one, alternating in one
process (bench_workloads.plugin_case, jwins).  One JSON line per run."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench_workloads as bw  # noqa: E402
from decentralizepy_amd.compression import Elias  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "jwins"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda", 0)
bw.plugin_case(dev, kind, rounds=1, warmup=1, cpu_rounds=0)
for rep in range(reps):
    for mode in (True, False):
        Elias.Elias.async_decode = mode
        r = bw.plugin_case(dev, kind, rounds=8, warmup=2, cpu_rounds=0)
        print(json.dumps({"rep": rep, "async_decode": mode, "round_ms": r["round_ms"],
                          "send_ms": r["send_ms"], "receive_ms": r["receive_ms"],
                          "wire_in_bytes": r["wire_in_bytes"]}), flush=True)
