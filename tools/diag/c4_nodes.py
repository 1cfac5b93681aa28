"""Diagnostic: the C4 round (96_regular, 96 x 11M) with node-batched encodes (argv[1] == "1",
dpz_topk_encode_nodes) or node-after-node streams ("0"); per-leg times.  For rocprofv3."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from decentralizepy_amd.gossip import GossipRound, read_edges  # noqa: E402

dev = torch.device("cuda", 0)
nb = len(sys.argv) < 2 or sys.argv[1] != "0"
adj = read_edges(os.path.join(ROOT, "tests", "golden", "96_regular.edges"))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 11_000_000
g = torch.Generator(device=dev).manual_seed(3)
x = torch.randn(len(adj), n, device=dev, generator=g)
eng = GossipRound(adj, x, 0.01, device=dev, node_batch=nb,
                  node_group=int(os.environ.get("DPZ_NODE_GROUP", "4")))
del x
noise = 0.01 * torch.randn(len(adj), n, device=dev, generator=g)
ts = []
for r in range(6):
    eng.x += noise
    torch.cuda.synchronize()
    eng.leg_times = {} if r >= 2 else None
    t0 = time.perf_counter()
    eng.step()
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
print(json.dumps({"node_batch": nb, "round_ms": [round(t * 1e3, 3) for t in ts],
                  "legs_ms": {k: round(v * 1e3 / 4, 3) for k, v in (eng.leg_times or {}).items()}}))
