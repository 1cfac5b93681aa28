#!/bin/bash
# tools/diag/fold_probe.py under diagnostic-build variants of the walk fold
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export DPZ_CODEC_LIB=$PWD/decentralizepy_amd/libdpzcodec_diag.so
for v in base epl8 b512 b768 b2048; do
  unset DPZ_FOLD_WALK_EPL DPZ_WALK_BLOCKS
  case $v in epl8) export DPZ_FOLD_WALK_EPL=8;; b512) export DPZ_WALK_BLOCKS=512;; b768) export DPZ_WALK_BLOCKS=768;; b2048) export DPZ_WALK_BLOCKS=2048;; esac
  timeout -k 10 120 python tools/diag/fold_probe.py > gpurun_out/fp_$v.json 2>>gpurun_out/fp.err || { echo "$v failed"; exit 1; }
done
