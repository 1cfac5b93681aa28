#!/bin/bash
# A/B of the filter grid for a lone codec (diagnostic build knobs DPZ_WLONE / DPZ_FILTER_DEPTH)
# on the plugin path (tools/diag/product_ab.py, hint + keep_x).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export DPZ_CODEC_LIB=$PWD/decentralizepy_amd/libdpzcodec_diag.so
for v in base 4096 2048 4096d6 6144; do
  unset DPZ_WLONE DPZ_FILTER_DEPTH
  case $v in 4096) export DPZ_WLONE=4096;; 2048) export DPZ_WLONE=2048;; 4096d6) export DPZ_WLONE=4096 DPZ_FILTER_DEPTH=6;; 6144) export DPZ_WLONE=6144;; esac
  timeout -k 10 200 python tools/diag/product_ab.py > gpurun_out/fg_$v.jsonl 2>>gpurun_out/fg.err || { echo "$v failed"; exit 1; }
done
