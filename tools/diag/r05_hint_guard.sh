#!/bin/bash
# Round-5 A/B session: the hint / sliced GPU tests, the C4 guarded-round A/B (REPS x ROUNDS),
# and the C3 workload with the sliced encode's prior window on and off (BENCH_HINT).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_hint.py tests/test_gpu_sliced.py tests/test_gpu_plugins.py > gpurun_out/hint_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/hint_tests.log; exit 1; }
tail -2 gpurun_out/hint_tests.log
REPS=${REPS:-5} ROUNDS=${ROUNDS:-20} timeout -k 10 500 python tools/diag/c4_guard_ab.py > gpurun_out/c4_guard_ab2.jsonl 2> gpurun_out/c4_guard_ab2.err || { echo "ab rc=$?"; tail -5 gpurun_out/c4_guard_ab2.err; exit 1; }
cat gpurun_out/c4_guard_ab2.jsonl
for h in 1 0 1 0; do
  BENCH_HINT=$h timeout -k 10 300 python bench.py --workload c3 --steps 30 > gpurun_out/c3_hint$h.json 2> gpurun_out/c3_hint.err || { echo "c3 rc=$?"; tail -5 gpurun_out/c3_hint.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/c3_hint$h.json'))
for r in d['result'][:3]: print('hint=$h', r.get('alpha'), r.get('workload','')[:22], round(r['ms_per_step'],4), round(r.get('encode_us',0),1), r.get('fell_back'), r.get('kernels_avg_us'))"
done
