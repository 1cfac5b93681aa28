"""Per-kernel average durations of a rocprofv3 ``--kernel-trace --stats`` summary (the
kernel_stats.csv) as JSON keyed by the bench's kernel names (tools/pmc2json.py short()), so the
bench line can quote the profile of its own command beside its live event-pair figure.
Usage: kstats2json.py kernel_stats.csv out.json ["source description"]; PMC_N = the tensor size."""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc2json import short  # noqa: E402


def main(path, out):
    calls = collections.Counter()
    total = collections.Counter()
    names = {}
    for r in csv.DictReader(open(path)):
        k = short(r["Name"])
        if not k:
            continue
        calls[k] += int(r["Calls"])
        total[k] += float(r["TotalDurationNs"])
        names.setdefault(k, r["Name"].split("(")[0].replace("void ", ""))
    kernels = {k: {"avg_us": round(total[k] / calls[k] / 1e3, 3), "calls": calls[k],
                   "kernel": names[k]} for k in sorted(calls)}
    doc = {"source": "rocprofv3 --kernel-trace --stats of "
                     + (sys.argv[3] if len(sys.argv) > 3 else "the bench command"),
           "kernels": kernels}
    if os.environ.get("PMC_N"):
        doc["n"] = int(os.environ["PMC_N"])
    with open(out, "w") as fh:
        json.dump(doc, fh, indent=1)
    for k, v in kernels.items():
        print(f"{k:22s} {v['avg_us']:9.3f} us x {v['calls']}")


if __name__ == "__main__":
    main(*sys.argv[1:3])
