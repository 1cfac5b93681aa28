#!/bin/bash
# A/B of library variants (tools/diag/build_variant.sh) on the plugin's device round
# (tools/diag/product_run.py: bench stages.product_one_node alone), alternating on one box.
#   VARIANTS="base lslf" N=16777216 bash tools/diag/variant_product_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-vab}.jsonl
: > $OUT
for r in 1 2; do for v in ${VARIANTS:-base}; do
  DPZ_CODEC_LIB=$PWD/tools/diag/variants/lib_$v.so timeout -k 10 200 python tools/diag/product_run.py ${N:-16777216} ${REPS:-100} > gpurun_out/vab_tmp.json 2> gpurun_out/vab.err || { echo "$v rc=$?"; tail -3 gpurun_out/vab.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/vab_tmp.json')); p=d['product_one_node']
row={'variant':'$v','rep':$r,'n':d['n']}
for k in ('1_payload','3_payload'):
    e=p[k]; row[k]={'step_us':e['step_us'],'encode_us':e['encode_us'],'fold_us':e['fold_us'],'frac':e['frac_of_hbm_peak'],'fold_kernel_us':e['kernels'].get('fold',{}).get('avg_us_event_pair')}
print(json.dumps(row))" | tee -a $OUT
done; done
