cd "${GRAFT_REPO_ROOT:-/root/repo}"
export DPZ_CODEC_LIB=$PWD/decentralizepy_amd/libdpzcodec_diag.so
for cfg in "0 x" "8 128" "8 64" "0 x" "8 128"; do
  set -- $cfg
  if [ "$2" = x ]; then unset DPZ_FOLD_WIN; else export DPZ_FOLD_WIN=$2; fi
  DPZ_FOLD_WALK_EPL=$1 timeout -k 10 300 python bench.py --workload c3 --steps 30 > gpurun_out/fab.json 2>gpurun_out/fab.err || exit 1
  python tools/diag/c3_summary.py "epl$1/win$2" gpurun_out/fab.json >> gpurun_out/fab.log
  python -c "
import json; d=json.loads(open('gpurun_out/fab.json').read().strip().splitlines()[-1]); print('epl$1/win$2 fold', d['result'][1]['kernels_avg_us']['fold'], 'idwt', d['result'][1]['kernels_avg_us']['idwt'])" >> gpurun_out/fab.log
done
cat gpurun_out/fab.log
