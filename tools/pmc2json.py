"""Per-launch HBM traffic of the codec kernels from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of wide
coalesced reads (MI355X_MICROARCH.md § HBM), so traffic = 2 * FETCH_SIZE + WRITE_SIZE.
Usage: pmc2json.py fetch.csv write.csv out.json ["source description"]
The tensor size the pass ran at goes into the JSON's "n" when PMC_N is set (bench.py's
load_pmc attaches the traffic to the line only at a matching n).
"""
import collections
import csv
import json
import os
import sys

NAMES = {"sampled_sample_kernel": "topk_sample", "sampled_filter_kernel": "topk_filter", "sampled_filter_pipe_kernel": "topk_filter",
         "sampled_select_kernel": "topk_select", "sampled_resolve_kernel": "topk_resolve",
         "sampled_compact_kernel": "topk_compact", "fold_offsets_kernel": "fold_offsets",
         "fold_kernel": "fold", "fold_group_kernel": "fold_group", "fold_slots_kernel": "fold_slots",
         "fold_walk_kernel": "fold_walk", "fold_walk_groups_kernel": "fold_walk", "replace_kernel": "fold", "dwt_kernel": "dwt", "dwt4_kernel": "dwt",
         "haar_dwt_kernel": "haar_dwt", "haar_idwt_kernel": "haar_idwt",
         "idwt_kernel": "idwt", "counter_sweep_kernel": "counter_flush",
         "counter_bounds_kernel": "counter_bounds", "counter_scatter_kernel": "counter_flush",
         "fold_merge_kernel": "fold_merge", "ft_pass_kernel": "fft_pass", "ft_pass_ip_kernel": "fft_pass_ip",
         "ft_r2c_post_kernel": "fft_r2c_post", "ft_c2r_pre_kernel": "fft_c2r_pre"}


# sampled_filter_pipe_kernel<SRC, CP, D, OCC>: CP = 1 writes the fused decode's copy of x (the
# bench step, 12N bytes), 2 the fold base (12N), 0 neither (8N) — separate rows, since one average
# over the variants would mix 8N and 12N launches
FILTER_CP = {"0": "topk_filter_plain", "1": "topk_filter", "2": "topk_filter_foldbase"}


def short(name):
    head = name.split("(")[0].replace("void ", "").split("::")[-1]
    base = head.split("<")[0]
    if base == "sampled_filter_pipe_kernel" and "<" in head:
        cp = head.split("<")[1].split(",")[1].strip()
        return FILTER_CP.get(cp, "topk_filter")
    return NAMES.get(base)


def load(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = short(r["Kernel_Name"])
        if k:
            acc[k].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main(fetch, write, out):
    f, w = load(fetch, "FETCH_SIZE"), load(write, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(f) | set(w)):
        fk, wk = f.get(k, 0.0), w.get(k, 0.0)
        kernels[k] = {"FETCH_SIZE_KiB": round(fk, 2), "WRITE_SIZE_KiB": round(wk, 2),
                      "hbm_bytes_per_launch": int(round((2 * fk + wk) * 1024))}
    src = sys.argv[4] if len(sys.argv) > 4 else (
        "`python3 bench.py --steps 100 --warmup 10 --no-cpu --no-extra --streams 1 --serial`")
    doc = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of "
                     f"{src}; traffic = 2*FETCH_SIZE (gfx950 half-count correction) + WRITE_SIZE",
           "kernels": kernels}
    if os.environ.get("PMC_N"):
        doc["n"] = int(os.environ["PMC_N"])
    with open(out, "w") as fh:
        json.dump(doc, fh, indent=1)
    for k, v in kernels.items():
        print(f"{k:14s} {v['hbm_bytes_per_launch'] / 1e6:9.2f} MB/launch")


if __name__ == "__main__":
    main(*sys.argv[1:4])
