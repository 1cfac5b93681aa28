#!/bin/bash
# walk fold (forced, DPZ_FOLD_KIND 4) at 16 payloads over JWINS alphas: window size x tile size
# sweep; one fold_kinds.py run per "name:VAR=v,..." entry of $AB (diagnostic).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export FOLD_KINDS="4"
export FOLD_CASES="${FOLD_CASES:-25000009:0.02:16:0 25000009:0.035:16:0 25000009:0.05:16:0 25000009:0.075:16:0 25000009:0.1:16:0 25000009:0.15:16:0 25000009:0.2:16:0}"
for ent in ${AB}; do
  name=${ent%%:*}
  envs=${ent#*:}
  (
    IFS=','; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done; unset IFS
    timeout -k 10 200 python -u tools/diag/fold_kinds.py > gpurun_out/wws_$name.jsonl 2> gpurun_out/wws_$name.err
  ) || { echo "$name rc=$?"; tail -3 gpurun_out/wws_$name.err; exit 1; }
  python3 -c "
import json
print('$name', [(d['alpha'], d['kinds']) for d in map(json.loads, open('gpurun_out/wws_$name.jsonl'))])"
done
