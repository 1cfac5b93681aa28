#!/bin/bash
# The fold kernel's hit path without chains (counts + first hit + pool rows): the fold parity GPU
# tests on the product library, then fold_kinds.py (auto dispatch and forced kind 1 = the
# classic kernel) with the new / old (HEAD) diagnostic builds alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_codec.py tests/test_gpu_foldbase.py tests/test_gpu_fold_batch.py tests/test_gpu_plugins.py tests/test_gpu_gossip.py tests/test_gpu_fft.py tests/test_gpu_stc.py tests/test_gpu_choco.py > gpurun_out/hp_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/hp_tests.log; exit 1; }
tail -1 gpurun_out/hp_tests.log
export FOLD_KINDS="1" FOLD_CASES="25000009:0.005:16:0 25000009:0.01:16:0 25000009:0.015:16:0 25000009:0.01:8:0 25000009:0.03:16:0 11000000:0.01:3:0"
for r in 1 2; do for v in old new; do
  DPZ_CODEC_LIB=$PWD/tools/diag/variants/lib_$v.so timeout -k 10 200 python tools/diag/fold_kinds.py > gpurun_out/hp_${v}_$r.jsonl 2> gpurun_out/hp.err || { echo "$v rc=$?"; tail -3 gpurun_out/hp.err; exit 1; }
  echo "== $v $r"; python -c "
import json
for l in open('gpurun_out/hp_${v}_$r.jsonl'):
    d=json.loads(l); print(d['alpha'], d['npay'], {k: (v['call_us'], v['kernels_us_event_pair']) for k, v in d['kinds'].items()})"
done; done
