#!/bin/bash
# A/B of the batched bench step with and without the co-scheduled decode (DPZ_BATCH_COSCHED).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for c in 0 1 0 1; do
  DPZ_BATCH_COSCHED=$c timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu > gpurun_out/cs_$c.json 2>/dev/null || exit 1
  python - "$c" <<'PY'
import json, sys
c = sys.argv[1]
d = json.loads(open(f"gpurun_out/cs_{c}.json").read().strip().splitlines()[-1])
st, se = d["stages"], d["secondary"]
print(f"cosched={c}", d["value"], d["ms_per_step"], "serial", st["one_node_serial_ms_per_step"],
      "64MiB", se["ms_per_step"], se["one_node_serial_ms_per_step"],
      st["encode"]["sampled_path_fell_back"], se["fell_back"])
PY
done
