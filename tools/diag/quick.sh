#!/bin/bash
# quick GPU check: topk + fold parity tests, then per-kernel timings on HBM-rotated inputs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K} > gpurun_out/pytest_q.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_q.log; [ $rc -ne 0 ] && exit $rc
for n in ${NS:-11000000 16777216}; do
  timeout -k 10 120 python tools/diag/filter_time.py $n 2>&1 | grep -v amdgpu.ids || exit 1
done
