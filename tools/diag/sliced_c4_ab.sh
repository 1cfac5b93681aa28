#!/bin/bash
# The C4 round's counters in bit-sliced form (gossip.py sliced_counter): the gossip GPU tests, then
# tools/diag/c4_sliced_ab.py (sliced / int32 counters alternating).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_gossip.py tests/test_gpu_rccl.py tests/test_gpu_batch.py tests/test_gpu_sliced.py > gpurun_out/slc_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/slc_tests.log; exit 1; }
tail -1 gpurun_out/slc_tests.log
REPS=3 ROUNDS=15 timeout -k 10 500 python tools/diag/c4_sliced_ab.py > gpurun_out/c4_sliced_ab.jsonl 2> gpurun_out/c4_sliced_ab.err || { echo "ab rc=$?"; tail -5 gpurun_out/c4_sliced_ab.err; exit 1; }
cat gpurun_out/c4_sliced_ab.jsonl
