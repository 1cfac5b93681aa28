#!/bin/bash
# Secondary workloads (bench.py --workload c3 | fft | wire), each under its own time limit, then
# the C3 rocprofv3 kernel-trace + PMC passes (tools/prof_c3.sh).  Outputs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in ${WORKLOADS:-c3 fft wire}; do
  timeout -k 10 300 python bench.py --workload $w --steps 30 > gpurun_out/wl_$w.json 2> gpurun_out/wl_$w.err || { echo "$w rc=$?"; tail -5 gpurun_out/wl_$w.err; exit 1; }
  echo "$w done"
done
if [ -n "$PROF_C3" ]; then bash tools/prof_c3.sh || exit 1; fi
exit 0
