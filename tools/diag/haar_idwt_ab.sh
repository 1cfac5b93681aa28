#!/bin/bash
# The haar accumulating pass (batched accumulator read-modify-write, DPZ_HAAR_ACC_BATCH) and the
# IDWT's branch-free coefficient loads (DPZ_IDWT_BF): parity tests on the product library, then
# new / old variant libraries alternating (dwt_post.py sym2 + haar, idwt_ab.py sym2 + haar).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_sliced.py tests/test_gpu_codec.py tests/test_gpu_shard.py tests/test_gpu_wavelet_generic.py tests/test_gpu_gossip.py tests/test_gpu_plugins.py > gpurun_out/hi_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/hi_tests.log; exit 1; }
tail -1 gpurun_out/hi_tests.log
for r in 1 2; do for v in old new; do
  for wv in haar sym2; do
    DPZ_CODEC_LIB=$PWD/tools/diag/variants/lib_$v.so timeout -k 10 200 python tools/diag/dwt_post.py $wv > gpurun_out/hi_post_${v}_${wv}_$r.json 2> gpurun_out/hi.err || { echo "$v rc=$?"; tail -3 gpurun_out/hi.err; exit 1; }
    echo "post $v $wv $r $(cat gpurun_out/hi_post_${v}_${wv}_$r.json)"
    DPZ_CODEC_LIB=$PWD/tools/diag/variants/lib_$v.so timeout -k 10 200 python tools/diag/idwt_ab.py $wv > gpurun_out/hi_idwt_${v}_${wv}_$r.json 2> gpurun_out/hi.err || { echo "$v rc=$?"; tail -3 gpurun_out/hi.err; exit 1; }
    echo "idwt $v $wv $r $(cat gpurun_out/hi_idwt_${v}_${wv}_$r.json | cut -c1-400)"
  done
done; done
