#!/bin/bash
# A/B of the default bench line: the product library, then each variant library
# (decentralizepy_amd/libdpz_v_<name>.so via DPZ_CODEC_LIB), each run under its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for v in product ${VARIANTS}; do
  if [ "$v" = product ]; then unset DPZ_CODEC_LIB; else export DPZ_CODEC_LIB=$PWD/decentralizepy_amd/libdpz_v_$v.so; fi
  timeout -k 10 300 python bench.py ${BENCH_ARGS:---steps 200 --warmup 20 --no-cpu} > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo "$v rc=$?"; tail -3 gpurun_out/ab_$v.err; exit 1; }
  python -c "
import json,sys; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]); st=d['stages']; se=d.get('secondary') or {}
print('$v', d['value'], d['ms_per_step'], 'serial', st['one_node_serial_ms_per_step'], '64MiB', se.get('ms_per_step'), se.get('one_node_serial_ms_per_step'), {k:v['avg_us'] for k,v in st['kernels'].items()})"
done
