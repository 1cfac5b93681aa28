#!/bin/bash
# Planes read per ripple step (DPZ_SL_PF 1 / 2 / 4) for the C4 round with sliced counters, and the
# int32-counter round beside them (pf4 library, ENGINE_SLICED=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for r in 1 2; do for v in pf4 pf1 pf2 dense; do
  lib=$v; sl=1; if [ $v = dense ]; then lib=pf4; sl=0; fi
  DPZ_CODEC_LIB=$PWD/tools/diag/variants/lib_$lib.so ENGINE_SLICED=$sl ROUNDS=12 timeout -k 10 300 python tools/diag/c4_round_ab.py > gpurun_out/slpf_${v}_$r.json 2> gpurun_out/slpf.err || { echo "$v rc=$?"; tail -3 gpurun_out/slpf.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/slpf_${v}_$r.json')); print('$v $r', d['ms_per_round'], d['legs_ms'], {k: v for k, v in d['kernels_us_calls'].items() if 'compact' in k})"
done; done
