#!/bin/bash
# Round-6 final validation on one box: the full GPU suite and the smoke, the rocprofv3 trace +
# PMC passes of the headline / C2 / plugin-round commands (tools/prof_r06.sh), and the
# workloads not yet re-run this round.  Each step has its own time limit; the chain stops at the
# first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=tests TAG=fin bash tools/gpu_r06.sh || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/fin_smoke.log; exit 1; }
tail -1 gpurun_out/fin_smoke.log
MODES="${MODES:-mib64 c2 product}" bash tools/prof_r06.sh || exit 1
STEPS=workloads WORKLOADS="${WORKLOADS:-c5 shard wire}" TAG=fin bash tools/gpu_r06.sh || exit 1
echo final done
