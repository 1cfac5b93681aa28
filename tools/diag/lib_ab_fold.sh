#!/bin/bash
# fold_kinds.py (auto dispatch) with the product library and each variant library
# tools/diag/variants/lib_<name>.so (VARIANTS="a b"), each run under its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export FOLD_KINDS=${FOLD_KINDS:-0}
export FOLD_CASES=${FOLD_CASES:-"25000009:0.02:16:0 25000009:0.05:16:0 25000009:0.1:16:0 25000009:0.2:16:0 25000009:0.1:8:0 25000009:0.1:3:0 25000009:0.4:3:0"}
for v in product ${VARIANTS}; do
  if [ "$v" = product ]; then unset DPZ_CODEC_LIB; else export DPZ_CODEC_LIB=$PWD/tools/diag/variants/lib_$v.so; fi
  timeout -k 10 200 python tools/diag/fold_kinds.py > gpurun_out/foldab_$v.jsonl 2> gpurun_out/foldab_$v.err || { echo "$v rc=$?"; tail -3 gpurun_out/foldab_$v.err; exit 1; }
  echo "== $v"; python -c "
import json
for l in open('gpurun_out/foldab_$v.jsonl'):
    d=json.loads(l); print(d['alpha'], d['npay'], d['kinds'])"
done
