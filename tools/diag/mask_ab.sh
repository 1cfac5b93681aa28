#!/bin/bash
# Walk-fold hit mask A/B (DPZ_WALK_MASK): the fold GPU tests on the product library, then
# fold_kinds.py (auto and forced walk) and the bench's product-path stage with the mask / tag
# variant libraries, alternating.  Each step under its own time limit; outputs in gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
    tests/test_gpu_codec.py tests/test_gpu_fold_batch.py tests/test_gpu_foldbase.py tests/test_gpu_gossip.py \
    tests/test_gpu_batch.py tests/test_gpu_plugins.py > gpurun_out/mask_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/mask_tests.log; exit 1; }
  tail -2 gpurun_out/mask_tests.log
fi
export FOLD_KINDS=${FOLD_KINDS:-"0 4"}
export FOLD_CASES=${FOLD_CASES:-"25000009:0.01:16:0 25000009:0.02:16:0 25000009:0.1:16:0 25000009:0.2:16:0 25000009:0.1:3:0 25000009:0.4:3:0 16777216:0.01:3:0 16777216:0.01:1:0 11000000:0.01:4:0"}
for r in 1 2; do
  for v in mask_d nomask_d; do
    DPZ_CODEC_LIB=$PWD/tools/diag/variants/lib_$v.so timeout -k 10 300 python tools/diag/fold_kinds.py > gpurun_out/maskab_${v}_$r.jsonl 2> gpurun_out/maskab_$v.err || { echo "$v rc=$?"; tail -3 gpurun_out/maskab_$v.err; exit 1; }
    echo "== $v run $r"
    python -c "
import json
for l in open('gpurun_out/maskab_${v}_$r.jsonl'):
    d=json.loads(l); print(d['m'], d['alpha'], d['npay'], {k: (v['call_us'], v['kernels_us_event_pair']) for k, v in d['kinds'].items()})"
  done
done
if [ -n "$BENCH_AB" ]; then
  for r in 1 2; do
    for v in product nomask; do
      if [ $v = product ]; then unset DPZ_CODEC_LIB; else export DPZ_CODEC_LIB=$PWD/tools/diag/variants/lib_$v.so; fi
      timeout -k 10 300 python bench.py --no-cpu --no-extra > gpurun_out/maskab_bench_${v}_$r.json 2> gpurun_out/maskab_bench.err || { echo "bench $v rc=$?"; tail -3 gpurun_out/maskab_bench.err; exit 1; }
      python -c "
import json; d=json.load(open('gpurun_out/maskab_bench_${v}_$r.json')); s=d['stages']
print('$v', d['value'], s.get('product_one_node'))" | cut -c1-700
    done
  done
  unset DPZ_CODEC_LIB
fi
exit 0
