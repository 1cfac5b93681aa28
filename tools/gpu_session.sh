#!/bin/bash
# One GPU-box session: the GPU test suite, then the driver's bench command and the secondary
# workloads given in $WORKLOADS, each under its own time limit; any failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
fi
timeout -k 10 ${BENCH_TIMEOUT:-400} python -u bench.py --gpus 1 --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; [ $rc -eq 0 ] || { echo "bench rc=$rc"; tail -5 gpurun_out/bench.err; exit $rc; }
echo "bench done"
for w in ${WORKLOADS}; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 20 > gpurun_out/wl_$w.json 2> gpurun_out/wl_$w.err
  rc=$?; [ $rc -eq 0 ] || { echo "$w rc=$rc"; tail -5 gpurun_out/wl_$w.err; exit $rc; }
  echo "$w done"
done
for d in ${DIAG}; do
  b=$(basename $d .py)
  timeout -k 10 300 python -u $d > gpurun_out/diag_$b.jsonl 2> gpurun_out/diag_$b.err
  rc=$?; [ $rc -eq 0 ] || { echo "diag $b rc=$rc"; tail -5 gpurun_out/diag_$b.err; exit $rc; }
  echo "diag $b done"
done
exit 0
