"""One-line summaries of bench JSON for the late round-4 A/B script (tools/diag/ab_r04_late.sh):
`c3_summary.py <tag> <file>` for a --workload c3 line, `... product` for product_ab.py lines."""
import json
import sys

tag, path = sys.argv[1], sys.argv[2]
if len(sys.argv) > 3 and sys.argv[3] == "product":
    for line in open(path):
        d = json.loads(line)
        print(tag, d["n"], *[(k, d[k]["step_us"], d[k]["fold_us"]) for k in ("1_payload", "3_payload")])
else:
    d = json.loads(open(path).read().strip().splitlines()[-1])
    for r in d["result"][:2]:
        k = r["kernels_avg_us"]
        print(tag, r.get("alpha", ""), round(r["ms_per_step"] * 1e3, 1), "compact", k["topk_compact"],
              "filter", k["topk_filter"], "dwt", k.get("dwt"))
