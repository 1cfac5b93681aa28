#!/bin/bash
# time the sampled encode kernels of several library builds (DPZ_CODEC_LIB) on HBM-rotated inputs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for v in ${VARIANTS}; do
  for n in ${NS:-11000000 16777216}; do
    echo -n "$v n=$n "
    DPZ_CODEC_LIB=$PWD/decentralizepy_amd/libdpz_v_$v.so timeout -k 10 120 python tools/diag/filter_time.py $n 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
