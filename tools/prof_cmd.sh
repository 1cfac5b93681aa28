#!/bin/bash
# rocprofv3 kernel-trace summary of "$@" and separate FETCH_SIZE / WRITE_SIZE passes, under
# gpurun_out/prof_$NAME*, then the per-kernel traffic JSON gpurun_out/pmc_$NAME.json.
# Usage: NAME=c3a01 tools/prof_cmd.sh python3 tools/diag/c3_encode.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
N=${NAME:?NAME}
rm -rf gpurun_out/prof_$N gpurun_out/prof_${N}_fetch gpurun_out/prof_${N}_write
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$N -o run -- "$@" > gpurun_out/prof_$N.log 2>&1 || { echo "trace rc=$?"; tail -5 gpurun_out/prof_$N.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_${N}_fetch -o run -- "$@" > gpurun_out/prof_${N}_fetch.log 2>&1 || { echo "fetch rc=$?"; tail -5 gpurun_out/prof_${N}_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_${N}_write -o run -- "$@" > gpurun_out/prof_${N}_write.log 2>&1 || { echo "write rc=$?"; tail -5 gpurun_out/prof_${N}_write.log; exit 1; }
F=$(find gpurun_out/prof_${N}_fetch -name '*counter_collection.csv' | head -1)
W=$(find gpurun_out/prof_${N}_write -name '*counter_collection.csv' | head -1)
python3 tools/pmc2json.py "$F" "$W" gpurun_out/pmc_$N.json "$N: $*"
S=$(find gpurun_out/prof_$N -name '*kernel_stats.csv' | head -1)
cp "$S" gpurun_out/kstats_$N.csv
echo "prof $N done"
