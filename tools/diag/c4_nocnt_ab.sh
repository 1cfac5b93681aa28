#!/bin/bash
# Ablation (results differ, timing only): the C4 round with the node-batched compact's counter
# update removed, against the same build with it — the ceiling of a cheaper counter form.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for r in 1 2 3; do for v in base nocnt; do
  DPZ_CODEC_LIB=$PWD/tools/diag/variants/lib_$v.so ROUNDS=10 timeout -k 10 300 python tools/diag/c4_round_ab.py > gpurun_out/nocnt_${v}_$r.json 2> gpurun_out/nocnt.err || { echo "$v rc=$?"; tail -3 gpurun_out/nocnt.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/nocnt_${v}_$r.json')); print('$v $r', d['ms_per_round'], d['legs_ms'], {k: v for k, v in d['kernels_us_calls'].items() if 'compact' in k or 'filter' in k or 'select' in k})"
done; done
