#!/bin/bash
# A/B of a secondary workload (bench.py --workload $WL) across the product library and variants
# (decentralizepy_amd/libdpz_v_<name>.so): ms per step of every result entry.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for v in product ${VARIANTS}; do
  if [ "$v" = product ]; then unset DPZ_CODEC_LIB; else export DPZ_CODEC_LIB=$PWD/decentralizepy_amd/libdpz_v_$v.so; fi
  timeout -k 10 300 python bench.py --workload ${WL:-c3} --steps 20 > gpurun_out/wl_$v.json 2> gpurun_out/wl_$v.err || { echo "$v rc=$?"; tail -3 gpurun_out/wl_$v.err; exit 1; }
  python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open(f"gpurun_out/wl_{v}.json").read().strip().splitlines()[-1])
r = d["result"]
r = r if isinstance(r, list) else [r]
print(v, [(round(x.get("ms_per_step", 0), 4), x.get("fell_back")) for x in r])
PY
done
