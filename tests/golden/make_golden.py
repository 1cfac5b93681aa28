#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the UNMODIFIED reference.

Run in the build container only (the reference is not present on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports sacs-epfl/decentralizepy from /root/reference/src (Sharing, PartialModel, Wavelet,
JWINS, Elias, Linear mapping, Model) and replays multi-round gossip scenarios: a node's model is
set, "trained" (a fixed random perturbation), encoded with get_data_to_send, and averaged with
synthetic neighbour payloads through _averaging — twice, so the accumulation bookkeeping of
_pre_step/_post_step is exercised.  Every input and every output (payload indices/params,
shared_parameters_counter, accumulated_changes, averaged model) is saved as plain numpy arrays
(allow_pickle=False) together with the scenario description in JSON.

The reference's Wavelet imports PyWavelets, which exists in this image only for
/opt/conda/bin/python3.9 (PyWavelets 1.1.1).  A minimal in-process ``pywt`` module forwards the
four functions the reference calls (wavedec, coeffs_to_array, array_to_coeffs, waverec) to that
interpreter; the reference classes themselves run unmodified.

Scenarios are generated tie-free at the k-th key (checked on the reference's own model_change),
because torch.topk's CPU tie order is implementation-defined.
"""
import json
import os
import pickle
import subprocess
import sys
import tempfile
import types
from collections import deque

import numpy as np

sys.dont_write_bytecode = True
REF = "/root/reference/src"
OUT = os.path.dirname(os.path.abspath(__file__))
PY39 = "/opt/conda/bin/python3.9"

# ---------------------------------------------------------------------------------------------
# pywt bridge (forwards to PyWavelets 1.1.1 in python3.9)
_BRIDGE = r"""
import pickle, sys, warnings
warnings.filterwarnings("ignore")
import pywt
fn, args, kwargs = pickle.load(sys.stdin.buffer)
res = getattr(pywt, fn)(*args, **kwargs)
sys.stdout.buffer.write(pickle.dumps(res, protocol=4))
"""


def _call_pywt(fn, *args, **kwargs):
    p = subprocess.run([PY39, "-c", _BRIDGE], input=pickle.dumps((fn, args, kwargs), protocol=4),
                       capture_output=True, check=True)
    return pickle.loads(p.stdout)


def _np(x):
    try:
        import torch
        if isinstance(x, torch.Tensor):
            return x.numpy()
    except ImportError:
        pass
    return np.asarray(x)


pywt = types.ModuleType("pywt")
pywt.wavedec = lambda x, wavelet, level=None, **kw: _call_pywt("wavedec", _np(x), wavelet, level=level, **kw)
pywt.coeffs_to_array = lambda c, **kw: _call_pywt("coeffs_to_array", [_np(a) for a in c], **kw)
pywt.array_to_coeffs = lambda a, s, **kw: _call_pywt("array_to_coeffs", _np(a), s, **kw)
pywt.waverec = lambda c, wavelet, **kw: _call_pywt("waverec", [_np(a) for a in c], wavelet, **kw)
sys.modules["pywt"] = pywt

sys.path.insert(0, REF)
import torch  # noqa: E402

from decentralizepy.compression.Elias import Elias  # noqa: E402
from decentralizepy.mappings.Linear import Linear  # noqa: E402
from decentralizepy.models.Model import Model  # noqa: E402
from decentralizepy.sharing.JWINS.JWINS import JWINS  # noqa: E402
from decentralizepy.sharing.JWINS.Wavelet import Wavelet  # noqa: E402
from decentralizepy.sharing.PartialModel import PartialModel  # noqa: E402
from decentralizepy.sharing.Sharing import Sharing  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))
from oracle import topk as otopk  # noqa: E402


class Net(Model):
    """Two-tensor model: weight (rows, cols) and bias (nb,)."""

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
    sd = model.state_dict()
    pos = 0
    new = {}
    for k, v in sd.items():
        new[k] = torch.from_numpy(flat[pos:pos + v.numel()].reshape(v.shape).copy())
        pos += v.numel()
    model.load_state_dict(new)


def get_flat(model):
    return torch.cat([v.flatten() for v in model.state_dict().values()]).numpy().copy()


def neighbour_payloads(rng, length, kind, n_nbrs, rnd, alpha):
    """Synthetic neighbour messages in the reference wire format."""
    msgs = []
    for i in range(n_nbrs):
        deg = int(rng.integers(2, 6))
        if kind[i] == "full":
            m = {"params": rng.standard_normal(length).astype(np.float32)}
        else:
            k = max(1, round(alpha * length))
            idx = np.sort(rng.choice(length, size=k, replace=False)).astype(np.int32)
            m = {"alpha": alpha, "indices": idx,
                 "params": (0.05 * rng.standard_normal(k)).astype(np.float32), "send_partial": True}
        m["degree"] = deg
        m["iteration"] = rnd
        m["CHANNEL"] = "DPSGD"
        msgs.append(m)
    return msgs


def record_msgs(prefix, msgs, arrays):
    meta = []
    for i, m in enumerate(msgs):
        arrays[f"{prefix}_nbr{i}_params"] = np.asarray(m["params"])
        if "indices" in m:
            arrays[f"{prefix}_nbr{i}_indices"] = np.asarray(m["indices"])
        meta.append({"degree": m["degree"], "partial": "send_partial" in m,
                     "alpha": m.get("alpha")})
    return meta


def kth_tie(change, k):
    return otopk.kth_has_tie(otopk.keys_u32(change.numpy()), k)


class TieError(RuntimeError):
    pass


def run_scenario(name, cls, kwargs, rows, cols, nb, rounds, seed, wavelet=False, nbr_kinds=None,
                 averaging="_averaging", record_change=False):
    """Replay; on a tie at the k-th key (fp32 differences are quantised) retry with the next seed.
    ``averaging`` names the reference method the node calls on receive (``_averaging``, or the
    federated server's ``_averaging_server``)."""
    for attempt in range(40):
        try:
            meta = _run_scenario(name, cls, kwargs, rows, cols, nb, rounds, seed + 1000 * attempt,
                                 wavelet, nbr_kinds, averaging, record_change=record_change)
            meta["seed"] = seed + 1000 * attempt
            return meta
        except TieError as e:
            print("retry:", e)
    raise RuntimeError(f"{name}: no tie-free seed found")


def _run_scenario(name, cls, kwargs, rows, cols, nb, rounds, seed, wavelet, nbr_kinds,
                  averaging="_averaging", on_send=None, record_change=False):
    rng = np.random.default_rng(seed)
    n = rows * cols + nb
    model = Net(rows, cols, nb)
    x0 = rng.standard_normal(n).astype(np.float32)
    set_flat(model, x0)
    uid_nbrs = [1, 2, 3]
    mapping = Linear(1, 4)
    with tempfile.TemporaryDirectory() as tmp:
        plugin = cls(0, 0, None, mapping, Graph(uid_nbrs), model, None, tmp, **kwargs)
    arrays = {"x0": x0}
    meta = {"name": name, "class": cls.__name__, "kwargs": kwargs, "shape": [rows, cols, nb],
            "n": n, "rounds": []}
    if averaging != "_averaging":
        meta["averaging"] = averaging
    length = n
    for r in range(rounds):
        cur = get_flat(model)
        train = (0.01 * rng.standard_normal(n)).astype(np.float32)
        x_r = (cur + train).astype(np.float32)
        set_flat(model, x_r)
        arrays[f"r{r}_x"] = x_r
        data = plugin.get_data_to_send(degree=len(uid_nbrs))
        if on_send is not None:  # wire_main: records the payload and ends the replay
            on_send(r, data)
        change = plugin.model.model_change
        if record_change:  # PartialModel.py:331 (the reference's model.model_change after send)
            arrays[f"r{r}_model_change"] = change.numpy().copy()
        rmeta = {"alpha": float(plugin.alpha), "partial": "send_partial" in data}
        if wavelet:
            length = int(plugin.wt_shape[0])
            rmeta["coeff_len"] = length
        if "send_partial" in data:
            k = len(data["indices"])
            rmeta["k"] = k
            if plugin.change_based_selection if wavelet else True:
                if kth_tie(change, k):
                    raise TieError(f"{name}: tie at the k-th key in round {r} (seed {seed})")
            arrays[f"r{r}_indices"] = np.asarray(data["indices"])
        arrays[f"r{r}_params"] = np.asarray(data["params"])
        rmeta["degree"] = data["degree"]
        arrays[f"r{r}_counter_after_encode"] = plugin.model.shared_parameters_counter.numpy().copy()
        if plugin.model.accumulated_changes is not None:
            arrays[f"r{r}_acc_after_encode"] = plugin.model.accumulated_changes.numpy().copy()
        kinds = nbr_kinds[r] if nbr_kinds else ["partial"] * len(uid_nbrs)
        msgs = neighbour_payloads(rng, length, kinds, len(uid_nbrs), r, 0.05)
        rmeta["neighbours"] = record_msgs(f"r{r}", msgs, arrays)
        peer = {uid: deque([m]) for uid, m in zip(uid_nbrs, msgs)}
        getattr(plugin, averaging)(peer)
        arrays[f"r{r}_model_after"] = get_flat(model)
        if plugin.model.accumulated_changes is not None:
            arrays[f"r{r}_acc_after_avg"] = plugin.model.accumulated_changes.numpy().copy()
        meta["rounds"].append(rmeta)
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **arrays)
    return meta


def sharing_scenario(averaging="_averaging", name="sharing_full", seed=5):
    rng = np.random.default_rng(seed)
    rows, cols, nb = 31, 33, 7
    n = rows * cols + nb
    model = Net(rows, cols, nb)
    x0 = rng.standard_normal(n).astype(np.float32)
    set_flat(model, x0)
    with tempfile.TemporaryDirectory() as tmp:
        plugin = Sharing(0, 0, None, Linear(1, 4), Graph([1, 2, 3]), model, None, tmp)
    data = plugin.get_data_to_send(degree=3)
    msgs = neighbour_payloads(rng, n, ["full"] * 3, 3, 0, 1.0)
    arrays = {"x0": x0, "sent_params": np.asarray(data["params"])}
    meta = {"name": name, "class": "Sharing", "n": n, "shape": [rows, cols, nb],
            "neighbours": record_msgs("r0", msgs, arrays)}
    if averaging != "_averaging":
        meta["averaging"] = averaging
    getattr(plugin, averaging)({uid: deque([m]) for uid, m in zip([1, 2, 3], msgs)})
    arrays["r0_model_after"] = get_flat(model)
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **arrays)
    return meta


def server_main():
    """The federated server's plain average (reference Sharing.py:200-229 and
    sharing/JWINS/Wavelet.py:331-385, weight 1 / n, no self term) on Sharing, PartialModel and
    Wavelet, two rounds each with mixed sparse / full neighbour payloads ->
    tests/golden/server_*.npz + server_scenarios.json (the _averaging fixtures are untouched)."""
    torch.set_num_threads(4)
    srv = "_averaging_server"
    mixed = [["partial", "full", "partial"], ["full", "partial", "partial"]]
    scen = [
        run_scenario("server_pm", PartialModel, {"dict_ordered": True, "alpha": 0.1}, 40, 100,
                     99, 2, seed=51, nbr_kinds=mixed, averaging=srv),
        run_scenario("server_pm_acc", PartialModel,
                     {"dict_ordered": True, "alpha": 0.05, "accumulation": True,
                      "accumulate_averaging_changes": True}, 40, 100, 99, 2, seed=52,
                     averaging=srv),
        run_scenario("server_wv", Wavelet,
                     {"wavelet": "sym2", "level": 4, "alpha": 0.1, "metadata_cap": 0.5,
                      "accumulation": True}, 40, 100, 99, 2, seed=53, wavelet=True,
                     nbr_kinds=mixed, averaging=srv),
        sharing_scenario(averaging=srv, name="server_sharing", seed=54),
    ]
    with open(os.path.join(OUT, "server_scenarios.json"), "w") as f:
        json.dump({"scenarios": scen, "generator": "tests/golden/make_golden.py --server",
                   "reference": "sacs-epfl/decentralizepy v1 (/root/reference/src)",
                   "pywavelets": "1.1.1 (python3.9 bridge)", "torch": torch.__version__}, f,
                  indent=1)
    print("wrote", len(scen), "server scenarios")


def elias_vectors():
    rng = np.random.default_rng(9)
    cases = {"kat": np.array([10, 3, 6, 5], dtype=np.int32)}
    cases["consecutive"] = np.arange(100, 400, dtype=np.int32)
    cases["two"] = np.array([7, 2**31 - 1], dtype=np.int32)
    cases["pow2_gaps"] = np.cumsum(np.array([0] + [2**j for j in range(30)], dtype=np.int64)).astype(np.int32)
    for name, n, k in [("sparse_1pct", 1_000_000, 10_000), ("dense_40pct", 50_000, 20_000),
                       ("tiny", 1000, 17)]:
        cases[name] = rng.choice(n, size=k, replace=False).astype(np.int32)
    arrays = {}
    for name, a in cases.items():
        inp = a.copy()
        enc = Elias().compress(inp)           # sorts inp in place, as the reference does
        dec = Elias().decompress(enc)
        arrays[f"{name}_input"] = a
        arrays[f"{name}_sorted"] = inp
        arrays[f"{name}_bytes"] = np.asarray(enc, dtype=np.uint8)
        arrays[f"{name}_decoded"] = np.asarray(dec)
    np.savez_compressed(os.path.join(OUT, "elias.npz"), **arrays)
    return sorted(cases)


def pywt_vectors():
    """sym2 level-4 wavedec/coeffs_to_array and waverec straight from PyWavelets 1.1.1."""
    rng = np.random.default_rng(41)
    arrays = {}
    sizes = [64, 65, 66, 67, 101, 1001, 4099, 10000]
    for n in sizes:
        x = rng.standard_normal(n).astype(np.float32)
        arr, sl = pywt.coeffs_to_array(pywt.wavedec(x, "sym2", level=4))
        rec = pywt.waverec(pywt.array_to_coeffs(arr, sl, output_format="wavedec"), wavelet="sym2")
        arrays[f"n{n}_x"] = x
        arrays[f"n{n}_coeffs"] = np.asarray(arr, dtype=np.float32)
        arrays[f"n{n}_rec"] = np.asarray(rec, dtype=np.float32)
    np.savez_compressed(os.path.join(OUT, "wavelet_pywt.npz"), **arrays)
    return sizes


def main():
    torch.set_num_threads(4)
    scen = []
    pm_common = {"dict_ordered": True}
    scen.append(run_scenario("pm_a01_plain", PartialModel, {**pm_common, "alpha": 0.1},
                             40, 100, 99, 2, seed=11, nbr_kinds=[["partial", "full", "partial"]] * 2))
    scen.append(run_scenario("pm_a01_acc", PartialModel,
                             {**pm_common, "alpha": 0.1, "accumulation": True}, 40, 100, 99, 2,
                             seed=12))
    scen.append(run_scenario("pm_a02_accavg", PartialModel,
                             {**pm_common, "alpha": 0.2, "accumulation": True,
                              "accumulate_averaging_changes": True}, 40, 100, 99, 2, seed=13))
    scen.append(run_scenario("pm_a001_large", PartialModel, {**pm_common, "alpha": 0.01},
                             300, 333, 103, 1, seed=14))
    scen.append(run_scenario("pm_fullshare", PartialModel,
                             {**pm_common, "alpha": 0.6, "metadata_cap": 0.5, "accumulation": True},
                             40, 100, 99, 1, seed=15))
    wv = {"wavelet": "sym2", "level": 4, "alpha": 0.1, "metadata_cap": 0.5}
    scen.append(run_scenario("wv_plain", Wavelet, wv, 20, 50, 1, 2, seed=21, wavelet=True,
                             nbr_kinds=[["partial", "full", "partial"]] * 2))
    scen.append(run_scenario("wv_acc", Wavelet, {**wv, "accumulation": True}, 40, 100, 99, 2,
                             seed=22, wavelet=True))
    scen.append(run_scenario("wv_accavg", Wavelet,
                             {**wv, "accumulation": True, "accumulate_averaging_changes": True},
                             40, 100, 99, 2, seed=23, wavelet=True))
    scen.append(run_scenario("wv_nochange_sel", Wavelet,
                             {**wv, "accumulation": True, "change_based_selection": False},
                             40, 100, 99, 2, seed=24, wavelet=True))
    jw = {"alpha_list": "[0.1,0.15,0.2,0.25,0.3,0.4,1.0]", "wavelet": "sym2", "level": 4,
          "accumulation": True, "accumulate_averaging_changes": True, "metadata_cap": 0.5,
          "change_based_selection": True}
    scen.append(run_scenario("jwins_tutorial", JWINS, jw, 100, 100, 103, 4, seed=31,
                             wavelet=True))
    scen.append(sharing_scenario())
    elias = elias_vectors()
    wsizes = pywt_vectors()
    with open(os.path.join(OUT, "scenarios.json"), "w") as f:
        json.dump({"scenarios": scen, "elias_cases": elias, "wavelet_sizes": wsizes,
                   "generator": "tests/golden/make_golden.py",
                   "reference": "sacs-epfl/decentralizepy v1 (/root/reference/src)",
                   "pywavelets": "1.1.1 (python3.9 bridge)",
                   "torch": torch.__version__}, f, indent=1)
    print("wrote", len(scen), "scenarios")


class _WireDone(Exception):
    pass


def wire_main():
    """What the reference's TCP layer puts on the wire for a node's first outgoing message
    (communication/TCP.py:110-131, 215-232: pickle.dumps of the dict after DPSGDNode adds
    CHANNEL; total_data += len(pickle.dumps(params)), total_meta += the rest, total_bytes += the
    message length): for PartialModel, Wavelet and JWINS payloads, plain and with the reference
    Elias index compression -> tests/golden/wire.json (sha256 + lengths of the pickled dict)."""
    import hashlib
    torch.set_num_threads(4)
    with open(os.path.join(OUT, "scenarios.json")) as f:
        metas = {m["name"]: m for m in json.load(f)["scenarios"]}
    classes = {"PartialModel": PartialModel, "Wavelet": Wavelet, "JWINS": JWINS}
    cases = []
    for name, compression in [("pm_a01_plain", None), ("pm_a01_plain", "Elias"),
                              ("wv_plain", None), ("wv_acc", "Elias"),
                              ("jwins_tutorial", "Elias"), ("pm_fullshare", None)]:
        m = metas[name]
        kwargs = dict(m["kwargs"])
        if compression:
            kwargs.update(compress=True, compression_package="decentralizepy.compression." +
                          compression, compression_class=compression)
        rec = {}

        def on_send(r, data, rec=rec):
            msg = dict(data)
            msg["CHANNEL"] = "DPSGD"  # node/DPSGDNode.py adds the channel before send
            out = pickle.dumps(msg)
            data_len = len(pickle.dumps(msg["params"])) if "params" in msg else 0
            rec.update(keys=list(msg), pickle_len=len(out), data_len=data_len,
                       meta_len=len(out) - data_len, sha256=hashlib.sha256(out).hexdigest())
            raise _WireDone()

        rows, cols, nb = m["shape"]
        try:
            _run_scenario(name, classes[m["class"]], kwargs, rows, cols, nb, 1, m["seed"],
                          m["class"] != "PartialModel", None, on_send=on_send)
        except _WireDone:
            pass
        cases.append({"scenario": name, "compression": compression, **rec})
    with open(os.path.join(OUT, "wire.json"), "w") as f:
        json.dump({"cases": cases, "generator": "tests/golden/make_golden.py --wire",
                   "python": sys.version.split()[0], "numpy": np.__version__,
                   "pickle_protocol": pickle.DEFAULT_PROTOCOL}, f, indent=1)
    print("wrote", len(cases), "wire cases")


FULLSIZE = [  # (name, class, model shape (rows, cols, nb), kwargs): BASELINE.json's sizes
    ("c2_pm_11M", "PartialModel", (1000, 10999, 1000), {"dict_ordered": True, "alpha": 0.01}),
    ("pm_16M", "PartialModel", (4096, 4095, 4096), {"dict_ordered": True, "alpha": 0.01}),
    ("pm_64MiB_acc", "PartialModel", (4096, 4095, 4096),
     {"dict_ordered": True, "alpha": 0.01, "accumulation": True}),
    ("pm_67M", "PartialModel", (8192, 8191, 8192), {"dict_ordered": True, "alpha": 0.001}),
    ("c3_wv_25M", "Wavelet", (5000, 4999, 5000),
     {"wavelet": "sym2", "level": 4, "alpha": 0.01, "metadata_cap": 0.5}),
]


def fullsize_inputs(n, seed):
    """The full-size inputs, regenerated bit-identically by tests/test_gpu_fullsize.py: torch's
    CPU generator, x0 = randn(n), x1 = x0 + 0.01 * randn(n) in fp32."""
    g = torch.Generator().manual_seed(seed)
    x0 = torch.randn(n, generator=g)
    x1 = x0 + 0.01 * torch.randn(n, generator=g)
    return x0, x1


def fullsize_main():
    """SHA-256 of what the unmodified reference sends at BASELINE.json's full sizes (SURVEY.md §8c
    item 5): one get_data_to_send of PartialModel (sharing/PartialModel.py:164-255) at N = 11M,
    16.8M (64 MiB, plain and with accumulation) and 67M, and of Wavelet
    (sharing/JWINS/Wavelet.py:142-231) on a 25M-parameter model — indices int32, params fp32 and
    shared_parameters_counter int32 -> tests/golden/fullsize.json.  The k-th key is checked
    tie-free (else the next seed), so the index set is determined by the values alone."""
    import hashlib
    torch.set_num_threads(8)
    classes = {"PartialModel": PartialModel, "Wavelet": Wavelet}
    sha = lambda a, dt: hashlib.sha256(np.ascontiguousarray(a, dtype=dt).tobytes()).hexdigest()
    cases = []
    for name, cls_name, shape, kwargs in FULLSIZE:
        rows, cols, nb = shape
        n = rows * cols + nb
        for seed in range(100, 140):
            x0, x1 = fullsize_inputs(n, seed)
            model = Net(rows, cols, nb)
            set_flat(model, x0.numpy())
            with tempfile.TemporaryDirectory() as tmp:
                plugin = classes[cls_name](0, 0, None, Linear(1, 4), Graph([1, 2, 3]), model,
                                           None, tmp, **kwargs)
            set_flat(model, x1.numpy())
            data = plugin.get_data_to_send(degree=3)
            k = len(data["indices"])
            if kth_tie(plugin.model.model_change, k):
                print(name, "tie at seed", seed)
                continue
            rec = {"name": name, "class": cls_name, "shape": list(shape), "n": n, "seed": seed,
                   "kwargs": kwargs, "k": k, "alpha": float(plugin.alpha),
                   "indices_sha256": sha(data["indices"], np.int32),
                   "params_sha256": sha(data["params"], np.float32),
                   "counter_sha256": sha(plugin.model.shared_parameters_counter.numpy(), np.int32),
                   "indices_head": np.asarray(data["indices"][:4]).tolist()}
            if cls_name == "Wavelet":
                rec["coeff_len"] = int(plugin.wt_shape[0])
            if plugin.model.accumulated_changes is not None:
                rec["acc_sha256"] = sha(plugin.model.accumulated_changes.numpy(), np.float32)
            print(rec, flush=True)
            cases.append(rec)
            break
        else:
            raise RuntimeError(f"{name}: no tie-free seed")
    with open(os.path.join(OUT, "fullsize.json"), "w") as f:
        json.dump({"cases": cases, "generator": "tests/golden/make_golden.py --fullsize",
                   "inputs": "torch CPU Generator(seed): x0 = randn(n), x1 = x0 + 0.01*randn(n)",
                   "reference": "sacs-epfl/decentralizepy v1 (/root/reference/src)",
                   "pywavelets": "1.1.1 (python3.9 bridge)", "torch": torch.__version__}, f,
                  indent=1)
    print("wrote", len(cases), "full-size cases")


def haar_main():
    """The reference Wavelet plugin with its DEFAULT wavelet, haar (sharing/JWINS/Wavelet.py:56):
    pywt 1.1.1 haar wavedec / waverec vectors (odd and even sizes, levels 1-8) and multi-round
    Wavelet scenarios (plain, accumulation, accumulate-averaging, level 6, mixed full payloads)
    -> tests/golden/wavelet_haar_pywt.npz, haar_*.npz, haar_scenarios.json."""
    torch.set_num_threads(4)
    rng = np.random.default_rng(71)
    arrays, cases = {}, []
    for n, level in [(1, 1), (2, 1), (3, 1), (17, 4), (64, 4), (65, 4), (101, 4), (1001, 8),
                     (4099, 4), (10000, 6), (65537, 8)]:
        x = rng.standard_normal(n).astype(np.float32)
        arr, sl = pywt.coeffs_to_array(pywt.wavedec(x, "haar", level=level))
        rec = pywt.waverec(pywt.array_to_coeffs(arr, sl, output_format="wavedec"), wavelet="haar")
        key = f"n{n}_l{level}"
        arrays[f"{key}_x"] = x
        arrays[f"{key}_coeffs"] = np.asarray(arr, dtype=np.float32)
        arrays[f"{key}_rec"] = np.asarray(rec, dtype=np.float32)
        cases.append([n, level])
    np.savez_compressed(os.path.join(OUT, "wavelet_haar_pywt.npz"), **arrays)
    wv = {"alpha": 0.1, "metadata_cap": 0.5}  # wavelet / level: the reference defaults
    mixed = [["partial", "full", "partial"], ["full", "partial", "partial"]]
    scen = [
        run_scenario("haar_plain", Wavelet, wv, 20, 50, 1, 2, seed=81, wavelet=True,
                     nbr_kinds=mixed),
        run_scenario("haar_acc", Wavelet, {**wv, "accumulation": True}, 40, 100, 99, 2,
                     seed=82, wavelet=True),
        run_scenario("haar_accavg", Wavelet,
                     {**wv, "accumulation": True, "accumulate_averaging_changes": True},
                     40, 100, 99, 2, seed=83, wavelet=True),
        run_scenario("haar_l6_nochange", Wavelet,
                     {**wv, "level": 6, "accumulation": True, "change_based_selection": False},
                     40, 100, 99, 2, seed=84, wavelet=True),
        run_scenario("haar_server", Wavelet, {**wv, "accumulation": True}, 40, 100, 99, 2,
                     seed=85, wavelet=True, nbr_kinds=mixed, averaging="_averaging_server"),
    ]
    with open(os.path.join(OUT, "haar_scenarios.json"), "w") as f:
        json.dump({"scenarios": scen, "pywt_cases": cases,
                   "generator": "tests/golden/make_golden.py --haar",
                   "reference": "sacs-epfl/decentralizepy v1 (/root/reference/src)",
                   "pywavelets": "1.1.1 (python3.9 bridge)", "torch": torch.__version__}, f,
                  indent=1)
    print("wrote", len(scen), "haar scenarios,", len(cases), "pywt cases")


def generic_main():
    """The reference Wavelet plugin with wavelets other than sym2 / haar (any pywt name reaches
    pywt.wavedec / waverec, sharing/JWINS/Wavelet.py:12-32, 311-316): multi-round scenarios
    (plain with mixed full payloads, accumulation, accumulate-averaging, no change-based
    selection, the federated server, sym2 past level 4) -> tests/golden/wg_*.npz +
    wavelet_generic_scenarios.json (the pywt vectors: make_golden_wavelets.py)."""
    torch.set_num_threads(4)
    wv = {"alpha": 0.1, "metadata_cap": 0.5}
    mixed = [["partial", "full", "partial"], ["full", "partial", "partial"]]
    scen = [
        run_scenario("wg_db4_plain", Wavelet, {**wv, "wavelet": "db4", "level": 4}, 20, 50, 1, 2,
                     seed=91, wavelet=True, nbr_kinds=mixed),
        run_scenario("wg_coif3_acc", Wavelet,
                     {**wv, "wavelet": "coif3", "level": 3, "accumulation": True},
                     40, 100, 99, 2, seed=92, wavelet=True),
        run_scenario("wg_sym5_accavg", Wavelet,
                     {**wv, "wavelet": "sym5", "level": 4, "accumulation": True,
                      "accumulate_averaging_changes": True}, 40, 100, 99, 2, seed=93,
                     wavelet=True),
        run_scenario("wg_bior35_nochange", Wavelet,
                     {**wv, "wavelet": "bior3.5", "level": 4, "accumulation": True,
                      "change_based_selection": False}, 40, 100, 99, 2, seed=94, wavelet=True),
        run_scenario("wg_dmey_plain", Wavelet, {**wv, "wavelet": "dmey", "level": 2},
                     40, 100, 99, 2, seed=95, wavelet=True),
        run_scenario("wg_sym2_l6_acc", Wavelet,
                     {**wv, "wavelet": "sym2", "level": 6, "accumulation": True},
                     40, 100, 99, 2, seed=96, wavelet=True),
        run_scenario("wg_db8_server", Wavelet,
                     {**wv, "wavelet": "db8", "level": 3, "accumulation": True},
                     40, 100, 99, 2, seed=97, wavelet=True, nbr_kinds=mixed,
                     averaging="_averaging_server"),
    ]
    with open(os.path.join(OUT, "wavelet_generic_scenarios.json"), "w") as f:
        json.dump({"scenarios": scen, "generator": "tests/golden/make_golden.py --generic",
                   "reference": "sacs-epfl/decentralizepy v1 (/root/reference/src)",
                   "pywavelets": "1.1.1 (python3.9 bridge)", "torch": torch.__version__}, f,
                  indent=1)
    print("wrote", len(scen), "generic-wavelet scenarios")


def model_change_main():
    """``model.model_change`` as the reference leaves it after get_data_to_send
    (PartialModel.py:317-331: T(x - init), with accumulation the accumulated change before the
    rewind) for PartialModel plain / accumulation / accumulate_averaging_changes and Wavelet
    with accumulate_averaging_changes -> tests/golden/mc_*.npz + model_change_scenarios.json
    (the other fixtures are untouched)."""
    torch.set_num_threads(4)
    pm = {"dict_ordered": True}
    wv = {"wavelet": "sym2", "level": 4, "alpha": 0.1, "metadata_cap": 0.5}
    scen = [
        run_scenario("mc_pm_plain", PartialModel, {**pm, "alpha": 0.1}, 40, 100, 99, 2, seed=61,
                     record_change=True),
        run_scenario("mc_pm_acc", PartialModel, {**pm, "alpha": 0.1, "accumulation": True},
                     40, 100, 99, 2, seed=62, record_change=True),
        run_scenario("mc_pm_accavg", PartialModel,
                     {**pm, "alpha": 0.2, "accumulation": True,
                      "accumulate_averaging_changes": True}, 40, 100, 99, 2, seed=63,
                     record_change=True),
        run_scenario("mc_wv_accavg", Wavelet,
                     {**wv, "accumulation": True, "accumulate_averaging_changes": True},
                     40, 100, 99, 2, seed=64, wavelet=True, record_change=True),
    ]
    with open(os.path.join(OUT, "model_change_scenarios.json"), "w") as f:
        json.dump({"scenarios": scen, "generator": "tests/golden/make_golden.py --model-change",
                   "reference": "sacs-epfl/decentralizepy v1 (/root/reference/src)",
                   "pywavelets": "1.1.1 (python3.9 bridge)", "torch": torch.__version__}, f,
                  indent=1)
    print("wrote", len(scen), "model_change scenarios")


if __name__ == "__main__":
    if "--model-change" in sys.argv:
        model_change_main()
    elif "--haar" in sys.argv:
        haar_main()
    elif "--generic" in sys.argv:
        generic_main()
    elif "--fullsize" in sys.argv:
        fullsize_main()
    elif "--wire" in sys.argv:
        wire_main()
    elif "--server" in sys.argv:
        server_main()
    else:
        main()
