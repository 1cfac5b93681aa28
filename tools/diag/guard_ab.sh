cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_gossip.py tests/test_gpu_rccl.py tests/test_gpu_fold_batch.py tests/test_gpu_batch.py > gpurun_out/guard_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/guard_tests.log; exit 1; }
tail -2 gpurun_out/guard_tests.log
timeout -k 10 400 python tools/diag/c4_guard_ab.py > gpurun_out/c4_guard_ab.jsonl 2> gpurun_out/c4_guard_ab.err || { echo "ab rc=$?"; tail -5 gpurun_out/c4_guard_ab.err; exit 1; }
cat gpurun_out/c4_guard_ab.jsonl
