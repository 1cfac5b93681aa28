#!/bin/bash
# DPZ_WALK_GUESS was removed after the A/B (profiles/r05_fold_start_ab.txt): build lib_guess from
# commit ff7398b (tools/diag/build_variant.sh guess "-DDPZ_WALK_GUESS=1" ff7398b) to re-run it.
# The lone walk fold's start-up switches (DPZ_WALK4_LOCKSTEP / DPZ_WALK4_L_FIRST / DPZ_WALK_GUESS,
# build_variant.sh libraries base / ls / lf / lslf / guess): the fold parity tests on the guess
# library, then the bench's product-path stage (64 MiB, 1 and 3 payloads), alternating on one box.
# Outputs in gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
DPZ_CODEC_LIB=$PWD/tools/diag/variants/lib_guess.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_codec.py tests/test_gpu_fold_batch.py tests/test_gpu_foldbase.py tests/test_gpu_gossip.py tests/test_gpu_batch.py \
  > gpurun_out/fsab_tests.log 2>&1 || { echo "guess tests failed"; tail -30 gpurun_out/fsab_tests.log; exit 1; }
tail -1 gpurun_out/fsab_tests.log
for r in 1 2; do for v in base guess ls lf lslf; do
  DPZ_CODEC_LIB=$PWD/tools/diag/variants/lib_$v.so timeout -k 10 300 python bench.py --no-cpu --no-extra > gpurun_out/fsab_${v}_$r.json 2> gpurun_out/fsab.err || { echo "$v rc=$?"; tail -3 gpurun_out/fsab.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/fsab_${v}_$r.json')); p=d['stages']['product_one_node']
print('$v $r', {k: (p[k]['step_us'], p[k]['fold_us']) for k in p if isinstance(p[k], dict) and 'fold_us' in p[k]})"
done; done
