#!/bin/bash
# Round-5 GPU session pieces; STEP selects: tests (the full -m gpu suite), ab (plugin-path A/B),
# bench (the default bench line), workloads (every secondary workload), prof (tools/prof_r05.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in ${STEPS:-tests}; do
  case $s in
    tests) timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_gputests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r05_gputests.log; exit 1; }; tail -3 gpurun_out/r05_gputests.log ;;
    ab) for hk in 00 11; do AB_HINT=${hk:0:1} AB_KEEP_X=${hk:1:1} timeout -k 10 200 python tools/diag/product_ab.py > gpurun_out/r05_ab_$hk.jsonl 2>>gpurun_out/r05_ab.err || { echo "ab $hk failed"; exit 1; }; done ;;
    bench) timeout -k 10 300 python bench.py > gpurun_out/r05_bench.json 2> gpurun_out/r05_bench.err || { echo "bench rc=$?"; tail -5 gpurun_out/r05_bench.err; exit 1; } ;;
    workloads) for w in ${WORKLOADS:-c3 c4 c5 e2e shard fft wire plugin}; do
        timeout -k 10 500 python bench.py --workload $w --steps 30 > gpurun_out/r05_wl_$w.json 2> gpurun_out/r05_wl_$w.err || { echo "$w rc=$?"; tail -5 gpurun_out/r05_wl_$w.err; exit 1; }
        echo "$w done"; done ;;
    prof) bash tools/prof_r05.sh || exit 1 ;;
  esac
done
exit 0
