#!/bin/bash
# The merge fold with kept payload windows (round 6) against the committed build (lib_base) and
# against itself with DPZ_MERGE_KEEP=0, alternating on one box (tools/diag/merge_time.py cases),
# after the merge fold's parity tests on the working tree's product library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fold_merge.py tests/test_gpu_codec.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/keep_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/keep_tests.log; exit 1; }
tail -1 gpurun_out/keep_tests.log
: > gpurun_out/merge_keep_ab.jsonl
for r in 1 2; do for v in base keep keep0; do
  lib=$v; env=""
  if [ $v = keep0 ]; then lib=keep; env="DPZ_MERGE_KEEP=0"; fi
  env $env DPZ_CODEC_LIB=$PWD/tools/diag/variants/lib_$lib.so timeout -k 10 200 python tools/diag/merge_time.py > gpurun_out/mk_tmp.jsonl 2> gpurun_out/mk.err || { echo "$v rc=$?"; tail -3 gpurun_out/mk.err; exit 1; }
  grep '^{' gpurun_out/mk_tmp.jsonl | sed "s/^{/{\"variant\": \"$v\", \"rep\": $r, /" >> gpurun_out/merge_keep_ab.jsonl
done; done
python3 -c "
import json
for l in open('gpurun_out/merge_keep_ab.jsonl'):
    d=json.loads(l); print(d['variant'], d['rep'], d['m'], d['alpha'], d['npay'], d['us']['merge8'])"
