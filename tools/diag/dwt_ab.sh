#!/bin/bash
# DWT A/B: time the DWT pair / IDWT at 25M for library variants (decentralizepy_amd/libdpz_v_<name>.so,
# built by tools/diag/build_variant.sh and copied there), then one SQ PMC pass on the product DWT.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${VARIANTS}; do
  echo -n "$v: "
  DPZ_CODEC_LIB=$PWD/decentralizepy_amd/libdpz_v_$v.so timeout -k 10 120 python tools/diag/dwt_time.py 2>&1 | grep -v amdgpu.ids || exit 1
done
if [ -n "$PMC" ]; then
  rm -rf gpurun_out/pmc_dwt
  timeout -s KILL 90 rocprofv3 --pmc $PMC --output-format csv -d gpurun_out/pmc_dwt -o run -- python3 tools/diag/dwt_time.py > gpurun_out/pmc_dwt.log 2>&1 || { echo "pmc rc=$?"; tail -3 gpurun_out/pmc_dwt.log; exit 1; }
  echo pmc done
fi
