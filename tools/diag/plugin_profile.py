"""Diagnostic: where the host time of a plugin round goes (bench_workloads.plugin_case's round,
PartialModel + Elias at C2, or JWINS + EliasFpzip at 25 M with argv[1] == "jwins"), cProfile of
the timed rounds, top entries by cumulative and by own time."""
import cProfile
import io
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench_workloads as bw  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "partial"
dev = torch.device("cuda", 0)
bw.plugin_case(dev, kind, rounds=2, warmup=2, cpu_rounds=0)  # warm (allocations, kernels)
pr = cProfile.Profile()
pr.enable()
r = bw.plugin_case(dev, kind, rounds=4, warmup=0, cpu_rounds=0)
pr.disable()
print(r)
for key in ("cumulative", "tottime"):
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats(key).print_stats(30)
    print(s.getvalue())
