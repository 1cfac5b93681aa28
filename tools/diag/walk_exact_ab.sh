#!/bin/bash
# Same-box A/B: the few-payload walk fold compiled per exact payload count (product build) against
# the 4-slot kernel with run-time slot tests (tools/diag/variants/lib_noexact.so, DPZ_WALK_EXACT=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in exact noexact; do
    if [ $v = exact ]; then L=$PWD/decentralizepy_amd/libdpzcodec.so; else L=$PWD/tools/diag/variants/lib_noexact.so; fi
    DPZ_CODEC_LIB=$L timeout -k 10 120 python tools/diag/fold_probe.py | sed "s/^{/{\"variant\": \"$v\", /" >> gpurun_out/walk_exact_ab.jsonl || { echo "$v failed"; exit 1; }
  done
done
