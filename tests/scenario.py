"""Replay the golden multi-round gossip scenarios (tests/golden/make_golden.py) against a backend.

Two backends:
  * OracleNode — the numpy restatement (oracle/) of the reference Sharing logic, to pin the
    oracle against the reference's recorded outputs (CPU tests);
  * the device plugin classes of decentralizepy_amd (GPU tests), driven exactly like the Node
    drives the reference: get_data_to_send(), then _averaging(peer_deques).
"""
import json
import os
import random
from collections import deque

import numpy as np

from oracle import fold as ofold
from oracle import topk as otopk
from oracle import wavelet as owav

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_meta():
    """scenarios.json plus the federated-server scenarios (server_scenarios.json), merged."""
    with open(os.path.join(GOLDEN, "scenarios.json")) as f:
        meta = json.load(f)
    for extra in ("server_scenarios.json", "haar_scenarios.json", "model_change_scenarios.json",
                  "wavelet_generic_scenarios.json"):
        with open(os.path.join(GOLDEN, extra)) as f:
            meta["scenarios"] = meta["scenarios"] + json.load(f)["scenarios"]
    return meta


def scenario_names(cls_filter=None):
    return [s["name"] for s in load_meta()["scenarios"]
            if "rounds" in s and (cls_filter is None or s["class"] in cls_filter)]


def load(name):
    meta = next(s for s in load_meta()["scenarios"] if s["name"] == name)
    arrays = dict(np.load(os.path.join(GOLDEN, f"{name}.npz")))
    return meta, arrays


def neighbour_msgs(meta_round, arrays, r):
    msgs = []
    for i, nm in enumerate(meta_round["neighbours"]):
        m = {"params": arrays[f"r{r}_nbr{i}_params"].copy()}
        if nm["partial"]:
            m = {"alpha": nm["alpha"], "indices": arrays[f"r{r}_nbr{i}_indices"].copy(),
                 "params": arrays[f"r{r}_nbr{i}_params"].copy(), "send_partial": True}
        m["degree"] = nm["degree"]
        m["iteration"] = r
        m["CHANNEL"] = "DPSGD"
        msgs.append(m)
    return msgs


class OracleNode:
    """numpy mirror of reference PartialModel / Wavelet / JWINS round logic (fp32 exact)."""

    def __init__(self, meta, x0):
        kw = meta["kwargs"]
        self.cls = meta["class"]
        self.wavelet = self.cls in ("Wavelet", "JWINS")
        self.level = int(kw.get("level", 4))
        self.wname = kw.get("wavelet", "haar")  # the reference Wavelet's default
        self.alpha = kw.get("alpha", 1.0)
        self.cap = kw.get("metadata_cap", 1.0)
        self.accumulation = kw.get("accumulation", False)
        self.aac = kw.get("accumulate_averaging_changes", False)
        self.cbs = kw.get("change_based_selection", True)
        self.n = x0.shape[0]
        self.init = x0.copy()
        self.model = x0.copy()
        self.L = owav.coeff_len(self.n, self.level, self.wname) if self.wavelet else self.n
        self.acc = np.zeros(self.L, np.float32) if self.accumulation else None
        self.prev = self.init
        self.counter = np.zeros(self.L, np.int32)
        if self.cls == "JWINS":
            self.alpha_list = eval(kw["alpha_list"])
            random.seed(0)  # uid of rank 0 / machine 0

    def T(self, v):
        return owav.wavedec_array(v, self.level, self.wname) if self.wavelet else v

    def get_data_to_send(self):
        if self.cls == "JWINS":
            self.alpha = random.choice(self.alpha_list)
        x = self.model.copy()
        self.xT = self.T(x)
        if self.wavelet:
            change = owav.wavedec_array(x - self.init, self.level, self.wname)
            x0 = None
        else:
            change, x0 = x, self.init
        mode = otopk.ACC_NONE
        if self.accumulation:
            mode = otopk.ACC_ADD if self.aac else otopk.ACC_ACCUMULATE
        # model.model_change (PartialModel.py:317-331): the change, with accumulation the
        # accumulated change before the rewind
        if mode == otopk.ACC_ACCUMULATE:
            self.model_change = self.acc + ((change - x0) if x0 is not None else change)
        elif mode == otopk.ACC_ADD:
            self.model_change = ((change - x0) if x0 is not None else change) + self.acc
        else:
            self.model_change = (change - x0) if x0 is not None else change.copy()
        if self.alpha >= self.cap:
            if self.accumulation:
                if mode == otopk.ACC_ACCUMULATE:  # pre-step accumulation happens before the zeroing
                    self.acc += (change - x0) if x0 is not None else change
                self.acc[:] = 0
            return {"params": self.xT.copy()}
        k = round(self.alpha * self.L)
        if self.wavelet and not self.cbs:
            if mode == otopk.ACC_ACCUMULATE:
                self.acc += change
            idx, val = otopk.encode(self.xT, None, None, otopk.ACC_NONE, k, vals_src=self.xT,
                                    counter=self.counter)
            if self.acc is not None:
                self.acc[idx] = 0
        else:
            idx, val = otopk.encode(change, x0, self.acc, mode, k, vals_src=self.xT,
                                    counter=self.counter)
        return {"alpha": self.alpha, "indices": idx, "params": val, "send_partial": True}

    def averaging(self, msgs, server=False):
        """Metro-Hastings fold (reference Sharing.py:156-190); ``server``: the plain 1/n average
        with no self term of _averaging_server (Sharing.py:200-229, Wavelet.py:331-385)."""
        pays, degs = [], []
        for m in msgs:
            pays.append((m["indices"], m["params"]) if "send_partial" in m else (None, m["params"]))
            degs.append(m["degree"])
        local = self.xT if self.wavelet else self.model
        if server:
            total = ofold.fold(local, pays, [1 / len(msgs)] * len(msgs), None)
        else:
            w = [ofold.mh_weight(len(msgs), d) for d in degs]
            wt = 0
            for v in w:
                wt += v
            total = ofold.fold(local, pays, w, 1 - wt)
        self.model = (owav.waverec_array(total, self.n, self.level, self.wname) if self.wavelet
                      else total)
        # post step
        new = self.model.copy()
        if self.accumulation and self.aac:
            d = new - self.prev
            self.acc += self.T(d) if self.wavelet else d
        self.init = new
        if self.accumulation:
            self.prev = new


def check_round(got, arrays, r, meta_round, bits=True):
    """Compare one round's outputs: got = dict(payload, counter_enc, acc_enc, model, acc_avg)."""
    pay = got["payload"]
    if meta_round["partial"]:
        np.testing.assert_array_equal(np.asarray(pay["indices"]), arrays[f"r{r}_indices"])
    np.testing.assert_array_equal(np.asarray(pay["params"]).view(np.uint32),
                                  arrays[f"r{r}_params"].view(np.uint32))
    np.testing.assert_array_equal(np.asarray(got["counter_enc"]),
                                  arrays[f"r{r}_counter_after_encode"])
    if f"r{r}_acc_after_encode" in arrays:
        np.testing.assert_array_equal(np.asarray(got["acc_enc"]).view(np.uint32),
                                      arrays[f"r{r}_acc_after_encode"].view(np.uint32))
    np.testing.assert_array_equal(np.asarray(got["model"]).view(np.uint32),
                                  arrays[f"r{r}_model_after"].view(np.uint32))
    if f"r{r}_acc_after_avg" in arrays:
        np.testing.assert_array_equal(np.asarray(got["acc_avg"]).view(np.uint32),
                                      arrays[f"r{r}_acc_after_avg"].view(np.uint32))
    if f"r{r}_model_change" in arrays:
        np.testing.assert_array_equal(np.asarray(got["model_change"]).view(np.uint32),
                                      arrays[f"r{r}_model_change"].view(np.uint32))


def replay_oracle(name):
    meta, arrays = load(name)
    node = OracleNode(meta, arrays["x0"])
    for r, mr in enumerate(meta["rounds"]):
        node.model = arrays[f"r{r}_x"].copy()
        pay = node.get_data_to_send()
        got = {"payload": pay, "counter_enc": node.counter.copy(),
               "acc_enc": None if node.acc is None else node.acc.copy(),
               "model_change": node.model_change}
        node.averaging(neighbour_msgs(mr, arrays, r),
                       server=meta.get("averaging") == "_averaging_server")
        got["model"] = node.model
        got["acc_avg"] = None if node.acc is None else node.acc.copy()
        check_round(got, arrays, r, mr)


# ---- device plugin backend ---------------------------------------------------------------------
class _Mapping:
    def __init__(self, procs=4):
        self.procs = procs

    def get_uid(self, rank, machine_id):
        return machine_id * self.procs + rank


class _Graph:
    def __init__(self, nbrs):
        self.nbrs = set(nbrs)

    def neighbors(self, uid):
        return self.nbrs


def make_model(shape):
    import torch

    class Net(torch.nn.Module):
        """Stand-in for the reference Model (models/Model.py:15-25 codec fields)."""

        def __init__(self, rows, cols, nb):
            super().__init__()
            self.weight = torch.nn.Parameter(torch.zeros(rows, cols))
            self.bias = torch.nn.Parameter(torch.zeros(nb))
            self.model_change = None
            self.accumulated_changes = None
            self.shared_parameters_counter = None

    return Net(*shape)


def set_flat(model, flat):
    import torch
    sd = model.state_dict()
    pos, new = 0, {}
    for k, v in sd.items():
        new[k] = torch.from_numpy(flat[pos:pos + v.numel()].reshape(v.shape).copy())
        pos += v.numel()
    model.load_state_dict(new)


def get_flat(model):
    import torch
    return torch.cat([v.flatten() for v in model.state_dict().values()]).numpy().copy()


def _elias_wire(msgs, check_cls):
    """Neighbour messages as an Elias(-Fpzip) sender puts them on the wire (oracle encoder)."""
    from oracle import elias as oelias
    from oracle import fpz as ofpz
    out = []
    for m in msgs:
        m = dict(m)
        if check_cls == "Lz4Wrapper":  # liblz4 frames, as a reference node's lz4.frame sends
            from oracle import lz4 as olz4
            if "indices" in m:
                m["indices"] = olz4.wrapper_compress(np.array(m["indices"], dtype=np.int32))
            out.append(m)
            continue
        if "indices" in m:
            m["indices"] = oelias.encode(m["indices"])
        if check_cls == "EliasFpzip" and "params" in m:
            m["params"] = ofpz.encode(m["params"], 0)
        out.append(m)
    return out


def replay_plugin(name, tmpdir, compression_class=None, config=None):
    """Drive the device plugin through the scenario; with ``compression_class`` ("Elias",
    "EliasFpzip" or "Lz4Wrapper" of decentralizepy_amd.compression) the wire payloads are
    compressed and the outgoing index stream is checked against the oracle's reference-pinned
    Elias bytes (Lz4Wrapper: decoded by liblz4 and by the oracle's frame decoder; the neighbour
    messages arrive as liblz4 frames).
    ``config`` = (package, class, kwargs) from sharing_section(): the plugin is built the way
    Node.init_sharing builds it (importlib, keyword arguments from the config file)."""
    import torch  # noqa: F401
    from oracle import elias as oelias

    from decentralizepy_amd.sharing.JWINS.JWINS import JWINS
    from decentralizepy_amd.sharing.JWINS.Wavelet import Wavelet
    from decentralizepy_amd.sharing.PartialModel import PartialModel
    classes = {"PartialModel": PartialModel, "Wavelet": Wavelet, "JWINS": JWINS}
    meta, arrays = load(name)
    model = make_model(meta["shape"])
    set_flat(model, arrays["x0"])
    kwargs = dict(meta["kwargs"])
    if compression_class:
        kwargs.update(compress=True, compression_class=compression_class,
                      compression_package=f"decentralizepy_amd.compression.{compression_class}")
    if config is not None:
        import importlib
        package, cls_name, kwargs = config
        cls = getattr(importlib.import_module(package), cls_name)
        compression_class = kwargs.get("compression_class") if kwargs.get("compress") else None
    else:
        cls = classes[meta["class"]]
    plugin = cls(0, 0, None, _Mapping(), _Graph([1, 2, 3]), model, None, str(tmpdir), **kwargs)
    for r, mr in enumerate(meta["rounds"]):
        set_flat(model, arrays[f"r{r}_x"])
        data = plugin.get_data_to_send(degree=3)
        if compression_class:
            data = dict(data)
            if "indices" in data and compression_class == "Lz4Wrapper":
                from oracle import lz4 as olz4
                np.testing.assert_array_equal(olz4.wrapper_decompress(data["indices"]),
                                              arrays[f"r{r}_indices"])
                assert olz4.ref_decompress(data["indices"]) == olz4.decode_frame(data["indices"])
            elif "indices" in data:
                np.testing.assert_array_equal(np.asarray(data["indices"]),
                                              oelias.encode(arrays[f"r{r}_indices"]))
            if compression_class == "EliasFpzip" and "params" in data:
                from oracle import fpz as ofpz
                np.testing.assert_array_equal(np.asarray(data["params"]),
                                              ofpz.encode(arrays[f"r{r}_params"], 0))
            data = plugin.decompress_data(data)
        acc = getattr(model, "accumulated_changes", None)
        mc = getattr(model, "model_change", None)
        got = {"payload": data, "counter_enc": model.shared_parameters_counter.numpy().copy(),
               "acc_enc": None if acc is None else acc.cpu().numpy().copy(),
               "model_change": None if mc is None else mc.cpu().numpy().copy()}
        assert data["degree"] == mr["degree"]
        msgs = neighbour_msgs(mr, arrays, r)
        if compression_class:
            msgs = _elias_wire(msgs, compression_class)
        peer = {uid: deque([m]) for uid, m in zip([1, 2, 3], msgs)}
        getattr(plugin, meta.get("averaging", "_averaging"))(peer)
        got["model"] = get_flat(model)
        acc = getattr(model, "accumulated_changes", None)
        got["acc_avg"] = None if acc is None else acc.cpu().numpy().copy()
        check_round(got, arrays, r, mr)
    return plugin


# ---- config.ini drop-in ---------------------------------------------------------------------------
def localconfig_value(v):
    """The scalar coercion the reference's config reader (the absent ``localconfig`` package)
    applies, as inferred from its call sites (JWINS.py:88 evals alpha_list, so
    lists stay strings): int, then float, then booleans / None, else the string."""
    s = v.strip()
    for conv in (int, float):
        try:
            return conv(s)
        except ValueError:
            pass
    low = s.lower()
    if low in ("true", "yes", "on"):
        return True
    if low in ("false", "no", "off"):
        return False
    if low == "none":
        return None
    return s


def sharing_section(path, to_build=True):
    """[SHARING] of a reference config.ini as Node.init_sharing sees it (node/Node.py:303-328):
    package, class and the remaining keyword arguments; with ``to_build`` the reference's
    package paths point at this build (decentralizepy. -> decentralizepy_amd.), nothing else."""
    import configparser
    cp = configparser.ConfigParser()
    cp.read(path)
    sec = {k: localconfig_value(v) for k, v in cp.items("SHARING")}
    if to_build:
        for key in ("sharing_package", "compression_package"):
            if key in sec and str(sec[key]).startswith("decentralizepy."):
                sec[key] = "decentralizepy_amd." + sec[key][len("decentralizepy."):]
    package, cls = sec.pop("sharing_package"), sec.pop("sharing_class")
    return package, cls, sec


# ---- FFT plugin (tolerance parity: the device fp32 FFT / numpy vs torch's CPU pocketfft) -----------------------
def fft_tol(what, n, scale):
    """Absolute tolerance of an FFT-plugin quantity against the reference (torch float32
    pocketfft): 4 x the float32 FFT error bound eps * log2(n) * |x|, times sqrt(n) for the
    frequency-domain arrays (params, accumulators), with |x| = max |x0| of the scenario.
    Measured oracle-vs-reference errors sit 3-10x inside it (float64 numpy FFT)."""
    eps = float(np.finfo(np.float32).eps)
    base = 4 * eps * np.log2(n) * scale
    return base if what == "model" else base * np.sqrt(n)


def load_fft(name):
    with open(os.path.join(GOLDEN, "fft.json")) as f:
        meta = next(s for s in json.load(f)["scenarios"] if s["name"] == name)
    z = np.load(os.path.join(GOLDEN, "fft.npz"))
    arrays = {k.split("/", 1)[1]: z[k] for k in z.files if k.startswith(name + "/")}
    return meta, arrays


def fft_names():
    with open(os.path.join(GOLDEN, "fft.json")) as f:
        return [s["name"] for s in json.load(f)["scenarios"]]


def _close(got, ref, what, n, scale):
    got, ref = np.asarray(got), np.asarray(ref)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    np.testing.assert_allclose(got, ref, rtol=0, atol=fft_tol(what, n, scale), err_msg=what)


def check_fft_round(got, arrays, r, meta_round):
    """One FFT round: indices and counters exactly (the fixtures keep the k-th key separated by a
    relative gap >= 1e-3), complex values, accumulators and the averaged model within fft_tol."""
    pay = got["payload"]
    n, scale = arrays["x0"].shape[0], float(np.max(np.abs(arrays["x0"])))
    if meta_round["partial"]:
        np.testing.assert_array_equal(np.asarray(pay["indices"]), arrays[f"r{r}_indices"])
    _close(pay["params"], arrays[f"r{r}_params"], "params", n, scale)
    np.testing.assert_array_equal(np.asarray(got["counter_enc"]),
                                  arrays[f"r{r}_counter_after_encode"])
    if f"r{r}_acc_after_encode" in arrays:
        _close(got["acc_enc"], arrays[f"r{r}_acc_after_encode"], "acc_enc", n, scale)
    _close(got["model"], arrays[f"r{r}_model_after"], "model", n, scale)
    if f"r{r}_acc_after_avg" in arrays:
        _close(got["acc_avg"], arrays[f"r{r}_acc_after_avg"], "acc_avg", n, scale)


def replay_fft_oracle(name):
    from oracle import fft as offt
    meta, arrays = load_fft(name)
    node = offt.FFTNode(meta["kwargs"], arrays["x0"])
    for r, mr in enumerate(meta["rounds"]):
        node.model = arrays[f"r{r}_x"].copy()
        pay = node.get_data_to_send()
        got = {"payload": pay, "counter_enc": node.counter.copy(),
               "acc_enc": None if node.acc is None else node.acc.copy()}
        node.averaging(neighbour_msgs(mr, arrays, r))
        got["model"] = node.model
        got["acc_avg"] = None if node.acc is None else node.acc.copy()
        check_fft_round(got, arrays, r, mr)


def replay_fft_plugin(name, tmpdir):
    from decentralizepy_amd.sharing.JWINS.FFT import FFT
    meta, arrays = load_fft(name)
    model = make_model(meta["shape"])
    set_flat(model, arrays["x0"])
    plugin = FFT(0, 0, None, _Mapping(), _Graph([1, 2, 3]), model, None, str(tmpdir),
                 **meta["kwargs"])
    for r, mr in enumerate(meta["rounds"]):
        set_flat(model, arrays[f"r{r}_x"])
        data = plugin.get_data_to_send(degree=3)
        assert data["degree"] == mr["degree"]
        assert list(data) == (["alpha", "params", "indices", "send_partial", "degree", "iteration"]
                              if mr["partial"] else ["params", "degree", "iteration"])
        assert data["params"].dtype == np.complex64
        acc = getattr(model, "accumulated_changes", None)
        mc = getattr(model, "model_change", None)
        got = {"payload": data, "counter_enc": model.shared_parameters_counter.numpy().copy(),
               "acc_enc": None if acc is None else acc.cpu().numpy().copy(),
               "model_change": None if mc is None else mc.cpu().numpy().copy()}
        peer = {uid: deque([m]) for uid, m in zip([1, 2, 3], neighbour_msgs(mr, arrays, r))}
        plugin._averaging(peer)
        got["model"] = get_flat(model)
        acc = getattr(model, "accumulated_changes", None)
        got["acc_avg"] = None if acc is None else acc.cpu().numpy().copy()
        check_fft_round(got, arrays, r, mr)
    return plugin
