cd "${GRAFT_REPO_ROOT:-.}"
for i in 1 2 3; do
  for v in product base; do
    if [ $v = product ]; then unset DPZ_CODEC_LIB; else export DPZ_CODEC_LIB=$PWD/decentralizepy_amd/libdpz_v_base.so; fi
    echo "$v $(timeout -k 10 200 python bench.py --workload c4 --steps 10 --warmup 2 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"])')" || exit 1
  done
done
