#!/bin/bash
# A/B of the walk fold's window settings on the C3 workload (diagnostic): fold tests with
# 128-entry windows, then C3 under each "name:VAR=v,..." entry of $AB.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
DPZ_FOLD_WIN=128 timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 120 --timeout-method thread -k fold > gpurun_out/pytest_fold_w128.log 2>&1 || { echo "pytest rc=$?"; tail -5 gpurun_out/pytest_fold_w128.log; exit 1; }
tail -1 gpurun_out/pytest_fold_w128.log
for ent in ${AB}; do
  name=${ent%%:*}
  envs=${ent#*:}
  (
    IFS=','; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done; unset IFS
    timeout -k 10 300 python -u bench.py --workload c3 --steps 20 > gpurun_out/c3_$name.json 2> gpurun_out/c3_$name.err
  ) || { echo "$name rc=$?"; tail -3 gpurun_out/c3_$name.err; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/c3_$name.json'):
    l=l.strip()
    if not l.startswith('{'): continue
    for r in json.loads(l)['result']:
        if r.get('alpha') == 0.1: print('$name', round(r['ms_per_step'],4), r['kernels_avg_us'].get('fold'))
"
done
