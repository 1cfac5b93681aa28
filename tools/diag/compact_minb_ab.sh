#!/bin/bash
# DPZ_NODES_CMINB was removed after the A/B (profiles/r05_c4_compact_minb_ab.jsonl); it was the
# nodes_compact_kernel launch bound's minimum blocks per CU (4 in the product).
# The node-batched compact's register bound (DPZ_NODES_CMINB: blocks per CU the compiler must fit;
# at 4 the body spills ~320 bytes per lane, at 2 it needs 194 VGPRs): the gossip parity tests on the
# mb2 / mb3 libraries, then the C4 round alternating base / mb3 / mb2 (build_variant.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for v in ${VARIANTS_T:-mb2 mb3}; do
  DPZ_CODEC_LIB=$PWD/tools/diag/variants/lib_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_gossip.py > gpurun_out/cminb_tests_$v.log 2>&1 || { echo "$v tests failed"; tail -30 gpurun_out/cminb_tests_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/cminb_tests_$v.log)"
done
: > gpurun_out/${OUT:-cminb_ab}.jsonl
for r in 1 2; do for v in ${VARIANTS:-base mb3 mb2}; do
  DPZ_CODEC_LIB=$PWD/tools/diag/variants/lib_$v.so ROUNDS=12 timeout -k 10 300 python tools/diag/c4_round_ab.py > gpurun_out/cminb_$v.json 2> gpurun_out/cminb.err || { echo "$v rc=$?"; tail -3 gpurun_out/cminb.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/cminb_$v.json')); d['variant']='$v'; d['rep']=$r
open('gpurun_out/${OUT:-cminb_ab}.jsonl','a').write(json.dumps(d)+'\n')
print('$v $r', d['ms_per_round'], d['legs_ms'], {k: v for k, v in d['kernels_us_calls'].items() if 'topk' in k})"
done; done
