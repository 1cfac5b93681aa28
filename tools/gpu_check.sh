#!/bin/bash
# GPU-box session: parity tests, then (only if no crash) a short bench and a rocprofv3 summary.
# Each GPU step has its own time limit; any abort/segfault/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok_or_stop() {  # rc 0 = pass, 1 = test failures (still safe to continue); anything else stops
  local rc=$1 what=$2
  echo "[$what] rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $what (rc=$rc)"; exit "$rc"; fi
}
STAGE=${1:-all}
if [ "$STAGE" = all ] || [ "$STAGE" = test ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
  ok_or_stop $? pytest
  tail -5 gpurun_out/pytest_gpu.log
fi
if [ "$STAGE" = all ] || [ "$STAGE" = bench ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
  ok_or_stop $? bench
  tail -2 gpurun_out/bench.log
fi
if [ "$STAGE" = all ] || [ "$STAGE" = prof ]; then
  rm -rf gpurun_out/prof
  timeout -k 10 ${PROF_TIMEOUT:-400} rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 50 --warmup 10 --no-cpu --no-extra > gpurun_out/prof.log 2>&1
  ok_or_stop $? rocprof
  find gpurun_out/prof -name '*kernel_stats*' | head -3
fi
exit 0
