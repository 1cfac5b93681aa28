#!/bin/bash
# Round-4 measurement session: the default bench line, the 64 MiB line, every secondary
# workload, then the rocprofv3 passes (tools/prof_r04.sh).  Each step under its own time limit;
# outputs under gpurun_out/ (r04_*).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/r04_bench.json 2> gpurun_out/r04_bench.err || { echo "bench rc=$?"; exit 1; }
timeout -k 10 300 python bench.py --n 16777216 > gpurun_out/r04_bench_64mib.json 2> gpurun_out/r04_bench_64mib.err || { echo "bench64 rc=$?"; exit 1; }
for w in ${WORKLOADS:-c3 c4 c5 e2e shard fft wire plugin}; do
  timeout -k 10 400 python bench.py --workload $w --steps 30 > gpurun_out/r04_wl_$w.json 2> gpurun_out/r04_wl_$w.err || { echo "$w rc=$?"; tail -5 gpurun_out/r04_wl_$w.err; exit 1; }
  echo "$w done"
done
if [ -z "$NO_PROF" ]; then bash tools/prof_r04.sh || exit 1; fi
exit 0
