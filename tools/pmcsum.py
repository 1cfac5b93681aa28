"""Average PMC counters per kernel from rocprofv3 counter_collection CSVs (one or more passes)."""
import collections
import csv
import sys


def main(paths):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for p in paths:
        for r in csv.DictReader(open(p)):
            name = r["Kernel_Name"]
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if "Start_Timestamp" in r and r.get("End_Timestamp"):
                dur[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for name, cs in acc.items():
        short = name.split("(")[0].replace("void ", "")[-40:]
        vals = {c: sum(v) / len(v) for c, v in cs.items()}
        print(short, " ".join(f"{c}={v:.4g}" for c, v in sorted(vals.items())))


if __name__ == "__main__":
    main(sys.argv[1:])
