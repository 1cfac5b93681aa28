#!/usr/bin/env python3
"""Generate the Choco golden fixtures (tests/golden/choco.npz + choco.json) from the UNMODIFIED
reference ``decentralizepy.sharing.Choco`` (sacs-epfl/decentralizepy, src/decentralizepy/sharing/
Choco.py).  Run in the build container only (the reference is not on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_choco.py

Scenario: one Choco node with three neighbours, three rounds: the node "trains" (fixed random
perturbation), get_data_to_send (threshold sparsification of x - x_hat, all ties kept, nonzero
entries sent), then _averaging of its neighbours' sparse messages (x_hat += q; s += w_i T_i;
s += (1 - sum w) q; x += step_size (s - x_hat)); a second run takes alpha's k = 0 branch (no sparsification) through a second node with alpha = 0.  Round 0 of both
quantises the model to steps of 0.05 and zeroes every 5th element (x_hat = 0, so d = x): ties at
the threshold and exact zeros.  Every input and
output is saved as plain numpy arrays (allow_pickle=False).
"""
import json
import os
import sys
import tempfile
from collections import OrderedDict, deque

import numpy as np

sys.dont_write_bytecode = True
REF = "/root/reference/src"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REF)
import torch  # noqa: E402

from decentralizepy.mappings.Linear import Linear  # noqa: E402
from decentralizepy.models.Model import Model  # noqa: E402
from decentralizepy.sharing.Choco import Choco  # noqa: E402


class Net(Model):
    def __init__(self, rows, cols, nb):
        super().__init__()
        self.weight = torch.nn.Parameter(torch.zeros(rows, cols))
        self.bias = torch.nn.Parameter(torch.zeros(nb))


class Graph:
    def __init__(self, nbrs):
        self.nbrs = set(nbrs)

    def neighbors(self, uid):
        return self.nbrs


def set_flat(model, flat):
    new, pos = {}, 0
    for key, v in model.state_dict().items():
        new[key] = torch.from_numpy(flat[pos:pos + v.numel()].reshape(v.shape).copy())
        pos += v.numel()
    model.load_state_dict(new)


def get_flat(model):
    return torch.cat([v.flatten() for v in model.state_dict().values()]).numpy().copy()


def run(tag, alpha, step_size, rows, cols, nb, seed, quantised, arrays, meta):
    rng = np.random.default_rng(seed)
    n = rows * cols + nb
    model = Net(rows, cols, nb)
    x0 = rng.standard_normal(n).astype(np.float32)
    set_flat(model, x0)
    mapping = Linear(1, 4)
    with tempfile.TemporaryDirectory() as tmp:
        node = Choco(0, 0, None, mapping, Graph([1, 2, 3]), model, None, tmp,
                     step_size=step_size, alpha=alpha)
    arrays[f"{tag}_x0"] = x0
    rounds = []
    for r in range(3):
        train = (0.01 * rng.standard_normal(n)).astype(np.float32)
        x_r = (get_flat(model) + train).astype(np.float32)
        if quantised and r == 0:  # x_hat = 0: d = x quantised -> ties at T, exact zeros
            x_r = (np.round(x_r * 20) / 20).astype(np.float32)
            x_r[::5] = 0.0
        set_flat(model, x_r)
        arrays[f"{tag}_r{r}_x"] = x_r
        data = node.get_data_to_send(degree=3)
        arrays[f"{tag}_r{r}_idx"] = np.asarray(data["indices"])
        arrays[f"{tag}_r{r}_vals"] = np.asarray(data["params"], dtype=np.float32)
        peers = OrderedDict()
        degs = []
        for j, uid in enumerate((1, 2, 3)):
            kk = max(1, round(alpha * n)) if alpha > 0 else n // 3
            idx = np.sort(rng.choice(n, size=kk, replace=False)).astype(np.int64)
            vals = (0.05 * rng.standard_normal(kk)).astype(np.float32)
            deg = int(rng.integers(2, 6))
            degs.append(deg)
            arrays[f"{tag}_r{r}_nbr{j}_idx"] = idx
            arrays[f"{tag}_r{r}_nbr{j}_vals"] = vals
            peers[uid] = deque([{"params": vals, "indices": idx, "send_partial": True,
                                 "degree": deg, "iteration": r, "CHANNEL": "DPSGD"}])
        node._averaging(peers)
        arrays[f"{tag}_r{r}_x_after"] = get_flat(model)
        arrays[f"{tag}_r{r}_x_hat"] = torch.cat([v.flatten() for v in node.model_hat.values()]).numpy().copy()
        arrays[f"{tag}_r{r}_s"] = torch.cat([v.flatten() for v in node.s.values()]).numpy().copy()
        rounds.append({"degrees": degs})
    meta[tag] = {"alpha": alpha, "step_size": step_size, "shape": [rows, cols, nb], "n": n,
                 "seed": seed, "rounds": rounds}


def main():
    arrays, meta = {}, {}
    run("a", 0.05, 0.5, 100, 199, 101, 21, True, arrays, meta)
    run("z", 0.0, 0.3, 40, 50, 7, 22, True, arrays, meta)
    np.savez_compressed(os.path.join(OUT, "choco.npz"), **arrays)
    with open(os.path.join(OUT, "choco.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote choco.npz", len(arrays), meta["a"]["n"], meta["z"]["n"])


if __name__ == "__main__":
    main()
