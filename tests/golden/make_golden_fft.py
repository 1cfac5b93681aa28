#!/usr/bin/env python3
"""Golden fixtures of the reference FFT sharing plugin (sharing/JWINS/FFT.py) -> tests/golden/fft.npz
+ fft.json.  Run in the build container only (the reference is not present on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_fft.py

The UNMODIFIED reference ``FFT`` class (torch.fft on the CPU) replays two gossip rounds per
scenario, as make_golden.py does for PartialModel / Wavelet: the node's model is set, perturbed,
encoded with get_data_to_send and averaged through _averaging with synthetic complex64 neighbour
payloads.  Only sparse neighbour payloads: the reference's FFT.deserialized_model reads
m["indices"] for a full payload too (FFT.py:225-234) and raises KeyError, which the device plugin
reproduces (tests/test_gpu_fft.py).  Inputs and outputs (payload indices / complex params, counter,
complex accumulator, averaged model) are saved as plain numpy arrays.

The transform is floating-point and rocFFT rounds differently from pocketfft, so the consumers
compare with tolerances; a scenario is kept only if the k-th selection key is separated from the
(k+1)-th by a relative gap of at least 1e-3, so the index set is robust to that rounding.
"""
import json
import os
import sys
import tempfile
from collections import deque

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (puts the reference on sys.path)
import torch  # noqa: E402

from decentralizepy.sharing.JWINS.FFT import FFT  # noqa: E402

OUT = HERE
ROWS, COLS, NB = 40, 100, 98  # n = 4098 (even: the reference's irfft length is 2 (m - 1))


def complex_payloads(rng, m, kinds, rnd, alpha):
    msgs = []
    for kind in kinds:
        deg = int(rng.integers(2, 6))
        if kind == "full":
            v = (rng.standard_normal(m) + 1j * rng.standard_normal(m)).astype(np.complex64)
            msg = {"params": v}
        else:
            k = max(1, round(alpha * m))
            idx = np.sort(rng.choice(m, size=k, replace=False)).astype(np.int32)
            v = (0.05 * (rng.standard_normal(k) + 1j * rng.standard_normal(k))).astype(np.complex64)
            msg = {"alpha": alpha, "indices": idx, "params": v, "send_partial": True}
        msg.update(degree=deg, iteration=rnd, CHANNEL="DPSGD")
        msgs.append(msg)
    return msgs


class GapError(RuntimeError):
    pass


def kth_gap(key, k):
    s = np.sort(key.astype(np.float64))[::-1]
    if k >= len(s):
        return 1.0
    return float((s[k - 1] - s[k]) / max(s[k - 1], 1e-30))


def run(name, kwargs, rounds, seed, nbr_kinds=None):
    for attempt in range(60):
        try:
            return _run(name, kwargs, rounds, seed + 1000 * attempt, nbr_kinds)
        except GapError as e:
            print("retry:", e)
    raise RuntimeError(f"{name}: no well-separated seed")


def _run(name, kwargs, rounds, seed, nbr_kinds):
    rng = np.random.default_rng(seed)
    n = ROWS * COLS + NB
    m = n // 2 + 1
    model = mg.Net(ROWS, COLS, NB)
    x0 = rng.standard_normal(n).astype(np.float32)
    mg.set_flat(model, x0)
    nbrs = [1, 2, 3]
    with tempfile.TemporaryDirectory() as tmp:
        plugin = FFT(0, 0, None, mg.Linear(1, 4), mg.Graph(nbrs), model, None, tmp, **kwargs)
    arrays = {"x0": x0}
    meta = {"name": name, "class": "FFT", "kwargs": kwargs, "shape": [ROWS, COLS, NB], "n": n,
            "m": m, "seed": seed, "rounds": []}
    for r in range(rounds):
        cur = mg.get_flat(model)
        x_r = (cur + (0.01 * rng.standard_normal(n)).astype(np.float32)).astype(np.float32)
        mg.set_flat(model, x_r)
        arrays[f"r{r}_x"] = x_r
        data = plugin.get_data_to_send(degree=len(nbrs))
        rmeta = {"alpha": float(plugin.alpha), "partial": "send_partial" in data,
                 "degree": data["degree"]}
        if "send_partial" in data:
            k = len(data["indices"])
            sel = plugin.model.model_change if plugin.change_based_selection else \
                plugin.pre_share_model_transformed
            gap = kth_gap(sel.abs().numpy(), k)
            if gap < 1e-3:
                raise GapError(f"{name}: k-th gap {gap:.2e} in round {r} (seed {seed})")
            rmeta.update(k=k, kth_gap=gap)
            arrays[f"r{r}_indices"] = np.asarray(data["indices"])
        arrays[f"r{r}_params"] = np.asarray(data["params"])
        arrays[f"r{r}_counter_after_encode"] = plugin.model.shared_parameters_counter.numpy().copy()
        if plugin.model.accumulated_changes is not None:
            arrays[f"r{r}_acc_after_encode"] = plugin.model.accumulated_changes.numpy().copy()
        kinds = nbr_kinds[r] if nbr_kinds else ["partial"] * len(nbrs)
        msgs = complex_payloads(rng, m, kinds, r, 0.05)
        rmeta["neighbours"] = mg.record_msgs(f"r{r}", msgs, arrays)
        plugin._averaging({uid: deque([msg]) for uid, msg in zip(nbrs, msgs)})
        arrays[f"r{r}_model_after"] = mg.get_flat(model)
        if plugin.model.accumulated_changes is not None:
            arrays[f"r{r}_acc_after_avg"] = plugin.model.accumulated_changes.numpy().copy()
        meta["rounds"].append(rmeta)
    return meta, arrays


def main():
    torch.set_num_threads(4)
    base = {"dict_ordered": True, "alpha": 0.1}
    cases = [
        ("fft_plain", base, 2, 61, None),
        ("fft_acc", {**base, "accumulation": True}, 2, 62, None),
        ("fft_accavg", {**base, "accumulation": True, "accumulate_averaging_changes": True}, 2,
         63, None),
        ("fft_nochange_sel", {**base, "accumulation": True, "change_based_selection": False}, 2,
         64, None),
        ("fft_fullshare", {**base, "alpha": 0.6, "metadata_cap": 0.5, "accumulation": True}, 1,
         65, None),
    ]
    scen, arrays = [], {}
    for name, kw, rounds, seed, kinds in cases:
        meta, arr = run(name, kw, rounds, seed, kinds)
        scen.append(meta)
        arrays.update({f"{name}/{k}": v for k, v in arr.items()})
    np.savez_compressed(os.path.join(OUT, "fft.npz"), **arrays)
    with open(os.path.join(OUT, "fft.json"), "w") as f:
        json.dump({"scenarios": scen, "generator": "tests/golden/make_golden_fft.py",
                   "reference": "sacs-epfl/decentralizepy v1 (/root/reference/src)",
                   "torch": torch.__version__}, f, indent=1)
    print("wrote", len(scen), "FFT scenarios")


if __name__ == "__main__":
    main()
