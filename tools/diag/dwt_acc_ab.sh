#!/bin/bash
# Accumulating post-step DWT A/B (the tile-start accumulator prefetch, DPZ_DWT_ACC_PRE): the DWT /
# sliced / JWINS parity tests on the product library, then tools/diag/dwt_post.py with each
# variant library (VARIANTS), alternating twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_sliced.py tests/test_gpu_codec.py tests/test_gpu_shard.py tests/test_gpu_wavelet_generic.py tests/test_gpu_gossip.py tests/test_gpu_plugins.py > gpurun_out/dwt_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/dwt_tests.log; exit 1; }
tail -2 gpurun_out/dwt_tests.log
for r in 1 2; do for v in ${VARIANTS:-nopre pre4 pre3}; do
  DPZ_CODEC_LIB=$PWD/tools/diag/variants/lib_$v.so timeout -k 10 200 python tools/diag/dwt_post.py > gpurun_out/dwtacc_${v}_$r.json 2> gpurun_out/dwtacc.err || { echo "$v rc=$?"; tail -3 gpurun_out/dwtacc.err; exit 1; }
  echo "$v $r $(cat gpurun_out/dwtacc_${v}_$r.json)"
done; done
