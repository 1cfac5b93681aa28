#!/bin/bash
# rocprofv3 kernel-trace summary of the plugin path (tools/diag/product_ab.py) for the AB_HINT /
# AB_KEEP_X setting in the environment; summary CSV under gpurun_out/kstats_product_$TAG.csv
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-p}
rm -rf gpurun_out/prof_product_$T
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_product_$T -o run -- python3 tools/diag/product_ab.py > gpurun_out/prof_product_$T.log 2>&1 || { echo "trace rc=$?"; tail -5 gpurun_out/prof_product_$T.log; exit 1; }
S=$(find gpurun_out/prof_product_$T -name '*kernel_stats.csv' | head -1)
cp "$S" gpurun_out/kstats_product_$T.csv
rm -rf gpurun_out/prof_product_$T
