#!/bin/bash
# C4 round with sliced counters: node group size x stream count, alternating (same box).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
: > gpurun_out/c4_gs_ab.jsonl
for r in 1 2; do for gs in 4:3 2:3 8:3 4:4 8:4 4:2; do
  NODE_GROUP=${gs%:*} STREAMS=${gs#*:} ROUNDS=12 timeout -k 10 300 python tools/diag/c4_round_ab.py >> gpurun_out/c4_gs_ab.jsonl 2> gpurun_out/c4_gs.err || { echo "$gs rc=$?"; tail -3 gpurun_out/c4_gs.err; exit 1; }
  tail -1 gpurun_out/c4_gs_ab.jsonl | cut -c1-400
done; done
