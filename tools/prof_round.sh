#!/bin/bash
# Round profile: rocprofv3 kernel-trace summary of the default bench, then separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) for the HBM traffic of each kernel.  Outputs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
# the one-stream step co-schedules the decode inside the encoder's launches; profiling with it
# off keeps every kernel's trace and PMC rows its own (sample / select / compact free of
# replace-decode traffic)
export DPZ_BATCH_COSCHED=${COSCHED:-0}
CMD="python3 bench.py --steps ${STEPS:-100} --warmup 10 --no-cpu --no-extra --streams 1"
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- $CMD > gpurun_out/prof.log 2>&1 || { echo "trace rc=$?"; tail -5 gpurun_out/prof.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- $CMD > gpurun_out/pmc_fetch.log 2>&1 || { echo "fetch rc=$?"; tail -5 gpurun_out/pmc_fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- $CMD > gpurun_out/pmc_write.log 2>&1 || { echo "write rc=$?"; tail -5 gpurun_out/pmc_write.log; exit 1; }
tail -1 gpurun_out/prof.log | cut -c1-200
find gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write -type f | head -20
