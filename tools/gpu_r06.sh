#!/bin/bash
# Round-6 GPU session pieces; STEPS selects: tests (the full -m gpu suite), quick (TESTS=...),
# bench (the default bench line), workloads (WORKLOADS=...), prof (tools/prof_r06.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r06}
for s in ${STEPS:-tests}; do
  case $s in
    tests) timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_gputests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/${TAG}_gputests.log; exit 1; }; tail -3 gpurun_out/${TAG}_gputests.log ;;
    quick) timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_quick.log 2>&1 || { echo "quick tests failed"; tail -40 gpurun_out/${TAG}_quick.log; exit 1; }; tail -3 gpurun_out/${TAG}_quick.log ;;
    bench) timeout -k 10 300 python bench.py $BENCH_ARGS > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench rc=$?"; tail -5 gpurun_out/${TAG}_bench.err; exit 1; } ;;
    workloads) for w in ${WORKLOADS:-c3 c4 c5 e2e shard fft wire plugin}; do
        timeout -k 10 500 python bench.py --workload $w --steps 30 > gpurun_out/${TAG}_wl_$w.json 2> gpurun_out/${TAG}_wl_$w.err || { echo "$w rc=$?"; tail -5 gpurun_out/${TAG}_wl_$w.err; exit 1; }
        echo "$w done"; done ;;
    prof) bash tools/prof_r06.sh || exit 1 ;;
  esac
done
exit 0
