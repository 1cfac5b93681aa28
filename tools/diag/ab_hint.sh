#!/bin/bash
# Round 5: the prior-round window (hint) and keep-x A/B on the plugin path (product library),
# after the hint tests.  Outputs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_hint.py > gpurun_out/t_hint.log 2>&1 || { echo "hint tests failed"; tail -30 gpurun_out/t_hint.log; exit 1; }
for hk in 00 10 01 11; do
  AB_HINT=${hk:0:1} AB_KEEP_X=${hk:1:1} timeout -k 10 200 python tools/diag/product_ab.py > gpurun_out/ab_hint_$hk.jsonl 2>>gpurun_out/ab_hint.err || { echo "ab $hk failed"; exit 1; }
done
echo done
