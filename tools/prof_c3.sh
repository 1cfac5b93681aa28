#!/bin/bash
# C3 (JWINS 25M) profile: rocprofv3 kernel-trace summary, then separate FETCH_SIZE / WRITE_SIZE
# passes for the per-kernel HBM traffic.  Outputs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CMD="python3 bench.py --workload c3 --steps 20"
rm -rf gpurun_out/prof_c3 gpurun_out/pmc_c3_fetch gpurun_out/pmc_c3_write
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run -- $CMD > gpurun_out/prof_c3.log 2>&1 || { echo "trace rc=$?"; tail -5 gpurun_out/prof_c3.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_c3_fetch -o run -- $CMD > gpurun_out/pmc_c3_fetch.log 2>&1 || { echo "fetch rc=$?"; tail -5 gpurun_out/pmc_c3_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_c3_write -o run -- $CMD > gpurun_out/pmc_c3_write.log 2>&1 || { echo "write rc=$?"; tail -5 gpurun_out/pmc_c3_write.log; exit 1; }
find gpurun_out/prof_c3 gpurun_out/pmc_c3_fetch gpurun_out/pmc_c3_write -type f | head -20
