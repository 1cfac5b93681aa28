"""bench.py's stages.product_one_node alone (the drop-in PartialModel plugin's device round, 1
and 3 payloads) at one tensor size, for rocprofv3 passes over just that path.
Usage: python tools/diag/product_run.py [n] [reps]"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else bench.NORTH_STAR_N
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    dev = torch.device("cuda:0")
    k = round(0.01 * n)
    per_set = 4 * n * 4 + 8 * k
    R = max(6, math.ceil(2 * bench.L3_BYTES / per_set) + 1)
    g = torch.Generator(device=dev).manual_seed(1234)
    sets = []
    for _ in range(R):
        x = torch.randn(n, device=dev, generator=g)
        sets.append(dict(x=x, x0=x - 0.01 * torch.randn(n, device=dev, generator=g)))
    out = bench.product_one_node(sets, n, k, torch.cuda.Stream(dev), reps)
    print(json.dumps({"n": n, "k": k, "rotate": R, "product_one_node": out}), flush=True)


if __name__ == "__main__":
    main()
