#!/bin/bash
# Same-box A/B of two library variants (tools/diag/build_variant.sh) on the plugin's device round,
# the fold kinds (merge_time.py) and the C4 round; VARIANTS="base clamp".
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${VARIANTS:-base clamp}
VARIANTS="$V" TAG=${TAG:-cab}_product bash tools/diag/variant_product_ab.sh || exit 1
for v in $V; do
  DPZ_CODEC_LIB=$PWD/tools/diag/variants/lib_$v.so timeout -k 10 240 python tools/diag/merge_time.py > gpurun_out/${TAG:-cab}_merge_$v.jsonl 2> gpurun_out/cab.err || { echo "merge $v rc=$?"; tail -3 gpurun_out/cab.err; exit 1; }
  echo "merge $v done"
done
for r in 1 2; do for v in $V; do
  DPZ_CODEC_LIB=$PWD/tools/diag/variants/lib_$v.so timeout -k 10 240 python tools/diag/c4_round_ab.py > gpurun_out/cab_c4.json 2> gpurun_out/cab.err || { echo "c4 $v rc=$?"; tail -3 gpurun_out/cab.err; exit 1; }
  echo "{\"variant\": \"$v\", \"rep\": $r, \"c4\": $(tail -1 gpurun_out/cab_c4.json)}" >> gpurun_out/${TAG:-cab}_c4.jsonl
done; done
echo ok
