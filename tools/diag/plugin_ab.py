"""Diagnostic: same-box A/B of the PartialModel + Elias plugin round (bench_workloads.plugin_case
"partial", C2) with the encode's round-5 flags (hint, keep_x) as PartialModel issues them and with
both forced off, alternating A / B / A / B so host-load drift shows.  One JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

import bench_workloads as bw  # noqa: E402
from decentralizepy_amd import codec  # noqa: E402
from decentralizepy_amd.sharing import PartialModel  # noqa: E402

_enc = codec.topk_encode


def _plain(*a, **kw):
    kw["hint"] = False
    kw["keep_x"] = False
    return _enc(*a, **kw)


dev = torch.device("cuda", 0)
res = {"A": "PartialModel as shipped (hint, keep_x)", "B": "hint and keep_x forced off"}
bw.plugin_case(dev, "partial", rounds=2, warmup=1, cpu_rounds=0)
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2):
    for tag in ("A", "B"):
        PartialModel.codec.topk_encode = _enc if tag == "A" else _plain
        r = bw.plugin_case(dev, "partial", rounds=8, warmup=2, cpu_rounds=0)
        res.setdefault(tag + "_round_ms", []).append(r["round_ms"])
        res.setdefault(tag + "_send_ms", []).append(r["send_ms"])
        res.setdefault(tag + "_receive_ms", []).append(r["receive_ms"])
print(json.dumps(res))
