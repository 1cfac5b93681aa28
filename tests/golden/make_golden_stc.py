#!/usr/bin/env python3
"""Generate the STC golden fixtures (tests/golden/stc.npz + stc.json) from the UNMODIFIED
reference ``decentralizepy.sharing.STC`` (sacs-epfl/decentralizepy, src/decentralizepy/sharing/
STC.py).  Run in the build container only (the reference is not on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_stc.py

Scenario (the paper's Algorithm 2 as the reference implements it): a client STC node and a server
STC node.  Each round the client "trains" (fixed random perturbation), encodes with
get_data_to_send (top-k of model_change with residual error feedback), the server folds that
payload and two synthetic sparse payloads with _averaging_server, re-encodes with
server_broadcast, and the client applies the broadcast with process_received.  Every input and
output is saved as plain numpy arrays (allow_pickle=False).  compress=False: the reference's
default compressor EliasFpzipLossy needs fpzip, absent here.  Seeds whose k-th |model_change| key
ties are skipped (torch.topk's CPU tie order is implementation-defined).
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
from decentralizepy.sharing.STC import STC  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))
from oracle import topk as otopk  # noqa: E402


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


def make(rows, cols, nb, alpha, seed):
    rng = np.random.default_rng(seed)
    n = rows * cols + nb
    k = round(alpha * n)
    mapping = Linear(1, 4)
    with tempfile.TemporaryDirectory() as tmp:
        cm, sm = Net(rows, cols, nb), Net(rows, cols, nb)
        xc = rng.standard_normal(n).astype(np.float32)
        xs = rng.standard_normal(n).astype(np.float32)
        set_flat(cm, xc)
        set_flat(sm, xs)
        kw = dict(alpha=alpha, compress=False, compression_package=None, compression_class=None)
        client = STC(0, 0, None, mapping, Graph([1]), cm, None, tmp, **kw)
        server = STC(1, 0, None, mapping, Graph([0, 2, 3]), sm, None, tmp, **kw)
    arrays = {"xc0": xc, "xs0": xs}
    for r in range(2):
        x_r = (get_flat(cm) + (0.01 * rng.standard_normal(n)).astype(np.float32)).astype(np.float32)
        set_flat(cm, x_r)
        arrays[f"r{r}_x"] = x_r
        data = client.get_data_to_send()
        if otopk.kth_has_tie(otopk.keys_u32(client.model.model_change.numpy()), k):
            raise RuntimeError("tie")
        arrays[f"r{r}_idx"] = np.asarray(data["indices"], dtype=np.int32)
        arrays[f"r{r}_vals"] = np.asarray(data["params"], dtype=np.float32)
        arrays[f"r{r}_res"] = client.residuals.numpy().copy()
        peers = OrderedDict()
        msgs = [dict(data)]
        for j in range(2):
            idx = np.sort(rng.choice(n, size=k, replace=False)).astype(np.int32)
            vals = (0.05 * rng.standard_normal(k)).astype(np.float32)
            arrays[f"r{r}_nbr{j}_idx"] = idx
            arrays[f"r{r}_nbr{j}_vals"] = vals
            msgs.append({"alpha": alpha, "indices": idx, "params": vals, "iteration": r})
        for uid, m in zip((0, 2, 3), msgs):
            m = dict(m)
            m["degree"] = 1
            m["CHANNEL"] = "STC"
            peers[uid] = deque([m])
        total = server._averaging_server(peers)
        arrays[f"r{r}_total"] = total.numpy().copy()
        arrays[f"r{r}_server_change"] = server.model.model_change.numpy().copy()
        if otopk.kth_has_tie(otopk.keys_u32(server.model.model_change.numpy()), k):
            raise RuntimeError("tie")
        bdata = server.server_broadcast()
        arrays[f"r{r}_b_idx"] = np.asarray(bdata["indices"], dtype=np.int32)
        arrays[f"r{r}_b_vals"] = np.asarray(bdata["params"], dtype=np.float32)
        arrays[f"r{r}_server_res"] = server.residuals.numpy().copy()
        arrays[f"r{r}_server_model"] = get_flat(sm)
        b = {key: v for key, v in bdata.items() if key != "iteration"}
        client.process_received(dict(b))
        arrays[f"r{r}_client_model"] = get_flat(cm)
    return arrays, {"rows": rows, "cols": cols, "nb": nb, "n": n, "alpha": alpha, "k": k,
                    "seed": seed, "rounds": 2}


def main():
    for attempt in range(40):
        try:
            arrays, meta = make(100, 199, 101, 0.01, 11 + attempt)
            break
        except RuntimeError as e:
            print("retry:", e)
    np.savez_compressed(os.path.join(OUT, "stc.npz"), **arrays)
    with open(os.path.join(OUT, "stc.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote stc.npz", {k: v.shape for k, v in list(arrays.items())[:4]}, meta)


if __name__ == "__main__":
    main()
