#!/bin/bash
# A/B of the default bench line over environment settings of ONE library build:
#   AB="base: sif0:DPZ_SCATTER_IN_FILTER=0" tools/diag/env_ab.sh
# each entry "name:VAR=v,VAR2=w" (empty after the colon = the defaults), each run under its own
# time limit; prints one summary line per entry.  Diagnostic only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for ent in ${AB}; do
  name=${ent%%:*}
  envs=${ent#*:}
  (
    IFS=','; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done; unset IFS
    timeout -k 10 300 python bench.py ${BENCH_ARGS:---steps 200 --warmup 20 --no-cpu} > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err
  ) || { echo "$name rc=$?"; tail -3 gpurun_out/ab_$name.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/ab_$name.json').read().strip().splitlines()[-1]); st=d['stages']; se=d.get('secondary') or {}
print('$name', d['value'], d['ms_per_step'], 'serial', st['one_node_serial_ms_per_step'], '64MiB', se.get('ms_per_step'), se.get('one_node_serial_ms_per_step'), {k:v['avg_us'] for k,v in st['kernels'].items()})"
done
