#!/bin/bash
# Select's counter prefetch (DPZ_SELECT_CPF): the top-k GPU tests on the product library, then
# the bench line (one node, product path, 3 codecs at 64 MiB) and the C4 round with the product
# library and the nocpf variant alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_codec.py tests/test_gpu_hint.py tests/test_gpu_fullsize.py tests/test_gpu_stale.py tests/test_gpu_batch.py tests/test_gpu_gossip.py tests/test_gpu_plugins.py > gpurun_out/cpf_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/cpf_tests.log; exit 1; }
tail -1 gpurun_out/cpf_tests.log
for r in 1 2 3; do for v in product nocpf; do
  if [ $v = product ]; then unset DPZ_CODEC_LIB; else export DPZ_CODEC_LIB=$PWD/tools/diag/variants/lib_$v.so; fi
  timeout -k 10 300 python bench.py --no-cpu --no-extra > gpurun_out/cpf_bench_${v}_$r.json 2> gpurun_out/cpf.err || { echo "bench $v rc=$?"; tail -3 gpurun_out/cpf.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/cpf_bench_${v}_$r.json')); s=d['stages']; k=s.get('kernels', {})
print('$v $r', d['value'], s['one_node_serial_ms_per_step'], s['product_one_node']['3_payload']['step_us'], s['product_one_node']['1_payload']['step_us'], {n: k[n] for n in k if 'select' in n or 'compact' in n})"
done; done
for r in 1 2; do for v in product nocpf; do
  if [ $v = product ]; then unset DPZ_CODEC_LIB; else export DPZ_CODEC_LIB=$PWD/tools/diag/variants/lib_$v.so; fi
  ROUNDS=10 timeout -k 10 300 python tools/diag/c4_round_ab.py > gpurun_out/cpf_c4_${v}_$r.json 2> gpurun_out/cpf.err || { echo "c4 $v rc=$?"; tail -3 gpurun_out/cpf.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/cpf_c4_${v}_$r.json')); print('c4 $v $r', d['ms_per_round'], d['legs_ms'])"
done; done
unset DPZ_CODEC_LIB
