#!/bin/bash
# C4 round: node-batched encodes in groups of G nodes over 3 streams (DPZ_NODE_GROUP) vs streams
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
: > gpurun_out/c4g.log
for G in 0 16 8 4 2 1; do
  if [ $G = 0 ]; then timeout -k 10 200 python3 tools/diag/c4_nodes.py 0 >> gpurun_out/c4g.log 2>>gpurun_out/c4g.err || exit 1
  else DPZ_NODE_GROUP=$G timeout -k 10 200 python3 tools/diag/c4_nodes.py 1 | sed "s/^/G=$G /" >> gpurun_out/c4g.log 2>>gpurun_out/c4g.err || exit 1; fi
done
