#!/bin/bash
# default bench (C2, eager) per library build: value, ms/step and the per-kernel breakdown
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for v in ${VARIANTS}; do
  DPZ_CODEC_LIB=$PWD/decentralizepy_amd/libdpz_v_$v.so timeout -k 10 200 python bench.py --no-cpu ${BENCH_ARGS} > gpurun_out/bv_$v.log 2>&1 || { tail -3 gpurun_out/bv_$v.log; exit 1; }
  python3 - "$v" <<'PY'
import json, sys
l = [x for x in open(f"gpurun_out/bv_{sys.argv[1]}.log") if x.startswith("{")][-1]
d = json.loads(l)
sec = d.get("secondary") or {}
print(sys.argv[1], d["value"], d["ms_per_step"], sec.get("value"), {k: v["avg_us"] for k, v in d["stages"]["kernels"].items()})
PY
done
