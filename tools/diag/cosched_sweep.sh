#!/bin/bash
# bench (C2 + 64 MiB) per co-scheduling split of the decode over sample/select/resolve/compact
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for sh in ${SHARES:-0.2,0.3,0.35,0.15}; do
  DPZ_COSCHED=$sh timeout -k 10 200 python bench.py --no-cpu ${BENCH_ARGS} > gpurun_out/cs.log 2>&1 || { tail -3 gpurun_out/cs.log; exit 1; }
  python3 - "$sh" <<'PY'
import json, sys
d = json.loads([x for x in open("gpurun_out/cs.log") if x.startswith("{")][-1])
e, s = d.get("secondary") or {}, d["stages"]
print(sys.argv[1], "C2", d["value"], d["ms_per_step"], "serial", s["one_node_serial_ms_per_step"], "host", s["host_enqueue_ms_per_step"],
      "| 64MiB", e.get("value"), e.get("ms_per_step"), "serial", e.get("one_node_serial_ms_per_step"), e.get("fell_back"))
print("   ", {k: round(v["avg_us"], 1) for k, v in s["kernels"].items()})
PY
done
