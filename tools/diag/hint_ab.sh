#!/bin/bash
# Same-box A/B of the prior-round window (BENCH_HINT=1/0) on the bench line (64 MiB headline +
# C2 secondary, product path included), twice each, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for i in 1 2; do for h in 1 0; do
  BENCH_HINT=$h timeout -k 10 200 python bench.py --no-cpu --steps 100 > gpurun_out/hab_${h}_$i.json 2>>gpurun_out/hab.err || { echo "bench h=$h failed"; exit 1; }
done; done
