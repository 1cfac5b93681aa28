cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export FOLD_KINDS="0" FOLD_CASES="25000009:0.02:16:0 25000009:0.05:16:0 25000009:0.1:16:0 25000009:0.2:16:0 16777216:0.01:3:0"
for r in 1 2; do for v in $VARIANTS; do
  DPZ_CODEC_LIB=$PWD/tools/diag/variants/lib_$v.so timeout -k 10 200 python tools/diag/fold_kinds.py > gpurun_out/ab16_${v}_$r.jsonl 2> gpurun_out/ab16_$v.err || { echo "$v rc=$?"; tail -3 gpurun_out/ab16_$v.err; exit 1; }
  echo "== $v $r"; python -c "
import json
for l in open('gpurun_out/ab16_${v}_$r.jsonl'):
    d=json.loads(l); print(d['alpha'], d['npay'], {k: (v['call_us'], v['kernels_us_event_pair']) for k, v in d['kinds'].items()})"
done; done
