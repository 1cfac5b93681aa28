"""GPU: the drop-in plugin classes replay the reference's recorded multi-round scenarios
bit-exactly (payload indices/params, counters, accumulators, averaged models)."""
import os
from collections import deque

import numpy as np
import pytest
import torch

from tests import scenario

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", scenario.scenario_names())
def test_plugin_replays_reference_scenario(name, dev, tmp_path):
    scenario.replay_plugin(name, tmp_path)


@pytest.mark.parametrize("name", ["sharing_full", "server_sharing"])
def test_sharing_full_model_fold(dev, tmp_path, name):
    """Full-model Sharing: _averaging (Metro-Hastings) and the federated server's
    _averaging_server (1/n, no self term) against the reference's recorded outputs."""
    from decentralizepy_amd.sharing.Sharing import Sharing
    meta = next(s for s in scenario.load_meta()["scenarios"] if s["name"] == name)
    a = dict(np.load(os.path.join(scenario.GOLDEN, f"{name}.npz")))
    model = scenario.make_model(meta["shape"])
    scenario.set_flat(model, a["x0"])
    plugin = Sharing(0, 0, None, scenario._Mapping(), scenario._Graph([1, 2, 3]), model, None,
                     str(tmp_path))
    data = plugin.get_data_to_send(degree=3)
    np.testing.assert_array_equal(data["params"], a["sent_params"])
    msgs = []
    for i, nb in enumerate(meta["neighbours"]):
        msgs.append({"params": a[f"r0_nbr{i}_params"], "degree": nb["degree"], "iteration": 0,
                     "CHANNEL": "DPSGD"})
    getattr(plugin, meta.get("averaging", "_averaging"))(
        {uid: deque([m]) for uid, m in zip([1, 2, 3], msgs)})
    np.testing.assert_array_equal(scenario.get_flat(model).view(np.uint32),
                                  a["r0_model_after"].view(np.uint32))


def test_counter_dump_like_the_node(dev, tmp_path):
    """DPSGDNode.py:186-194 dumps model.shared_parameters_counter.numpy().tolist()."""
    plugin = scenario.replay_plugin("pm_a01_plain", tmp_path)
    counts = plugin.model.shared_parameters_counter.numpy().tolist()
    assert isinstance(counts, list) and sum(counts) == 2 * 410


def test_jwins_built_from_tutorial_config_replays_reference(dev, tmp_path):
    """JWINS built from the UNCHANGED tutorial/JWINS/config.ini [SHARING] section (package paths
    swapped), the way Node.init_sharing builds it, with the EliasFpzip wire compression the
    config names: the tutorial scenario replays bit-exactly, the outgoing index streams match
    the reference-pinned Elias bytes."""
    cfg = scenario.sharing_section(os.path.join(scenario.GOLDEN, "jwins_tutorial_config.ini"))
    meta = next(s for s in scenario.load_meta()["scenarios"] if s["name"] == "jwins_tutorial")
    # the fixture was generated with the config's algorithm keywords (no compression)
    for key, v in meta["kwargs"].items():
        assert cfg[2][key] == v, key
    scenario.replay_plugin("jwins_tutorial", tmp_path, config=cfg)


def _wire_cases():
    import json
    with open(os.path.join(scenario.GOLDEN, "wire.json")) as f:
        return json.load(f)["cases"]


@pytest.mark.parametrize("case", _wire_cases(), ids=lambda c: f"{c['scenario']}-{c['compression']}")
def test_outgoing_message_pickles_like_the_reference(dev, tmp_path, case):
    """TCP wire (communication/TCP.py:110-131, 215-232): the node's first outgoing dict, with the
    CHANNEL key DPSGDNode adds, pickles to the reference's exact bytes (same keys, order, dtypes
    and values), so total_bytes / total_data / total_meta count the same."""
    import hashlib
    import pickle

    from decentralizepy_amd.sharing.JWINS.JWINS import JWINS
    from decentralizepy_amd.sharing.JWINS.Wavelet import Wavelet
    from decentralizepy_amd.sharing.PartialModel import PartialModel
    classes = {"PartialModel": PartialModel, "Wavelet": Wavelet, "JWINS": JWINS}
    meta, arrays = scenario.load(case["scenario"])
    kwargs = dict(meta["kwargs"])
    if case["compression"]:
        c = case["compression"]
        kwargs.update(compress=True, compression_class=c,
                      compression_package=f"decentralizepy_amd.compression.{c}")
    model = scenario.make_model(meta["shape"])
    scenario.set_flat(model, arrays["x0"])
    plugin = classes[meta["class"]](0, 0, None, scenario._Mapping(), scenario._Graph([1, 2, 3]),
                                    model, None, str(tmp_path), **kwargs)
    scenario.set_flat(model, arrays["r0_x"])
    msg = dict(plugin.get_data_to_send(degree=3))
    msg["CHANNEL"] = "DPSGD"
    out = pickle.dumps(msg)
    data_len = len(pickle.dumps(msg["params"])) if "params" in msg else 0
    assert list(msg) == case["keys"]
    assert (len(out), data_len, len(out) - data_len) == (
        case["pickle_len"], case["data_len"], case["meta_len"])
    assert hashlib.sha256(out).hexdigest() == case["sha256"]


def test_save_accumulated_behaves_like_reference(dev, tmp_path):
    """save_accumulated (reference PartialModel.py:122-131, 350-390): the constructor creates
    model_change/<rank> and model_val/<rank>; _post_step clears model.model_change and then
    save_change() dumps it, i.e. calls None.tolist() -> AttributeError, as the reference does."""
    from decentralizepy_amd.sharing.PartialModel import PartialModel
    meta, arrays = scenario.load("pm_a01_plain")
    model = scenario.make_model(meta["shape"])
    scenario.set_flat(model, arrays["x0"])
    plugin = PartialModel(0, 0, None, scenario._Mapping(), scenario._Graph([1, 2, 3]), model,
                          None, str(tmp_path), alpha=0.1, save_accumulated="yes")
    assert (tmp_path / "model_change" / "0").is_dir() and (tmp_path / "model_val" / "0").is_dir()
    plugin.get_data_to_send(degree=3)
    msgs = scenario.neighbour_msgs(meta["rounds"][0], arrays, 0)
    with pytest.raises(AttributeError, match="tolist"):
        plugin._averaging({uid: deque([m]) for uid, m in zip([1, 2, 3], msgs)})


def test_staging_over_cap_falls_back_to_pageable_copies(dev):
    import numpy as np
    import torch

    from decentralizepy_amd._device import Staging, h2d_array, to_device_flat, to_host
    st = Staging(cap_bytes=4096)
    x = torch.randn(100_000)
    assert torch.equal(to_device_flat(x, dev, st, "local").cpu(), x)
    a = np.arange(50_000, dtype=np.int32)
    assert np.array_equal(h2d_array(a, np.int32, dev, st, "idx").cpu().numpy(), a)
    assert np.array_equal(to_host(torch.from_numpy(a).to(dev), st, "out"), a)
    small = to_device_flat(torch.ones(100), dev, st, "small")  # within the cap: pinned
    assert st.total == 400 and torch.equal(small.cpu(), torch.ones(100))


@pytest.mark.parametrize("chunk", [1000, 1 << 22])
def test_load_flat_pipelined_equals_load_state_dict(dev, chunk):
    """The averaged model's D2H pipelined against its copy into the model (_device.load_flat:
    chunked DMAs, each state tensor filled range by range as its chunks land) leaves every state
    tensor — fp32 parameters and BatchNorm's int64 counter — exactly as load_state_dict of the
    unflattened vector does (reference sharing/Sharing.py:186-190)."""
    import copy

    from decentralizepy_amd._device import Staging, load_flat
    torch.manual_seed(3)
    model = torch.nn.Sequential(torch.nn.Linear(300, 200), torch.nn.BatchNorm1d(200),
                                torch.nn.Linear(200, 7))
    ref = copy.deepcopy(model)
    sd = ref.state_dict()
    n = sum(v.numel() for v in sd.values())
    flat = torch.randn(n)
    out, s = {}, 0
    for key, v in sd.items():
        if v.dtype == torch.int64:
            flat[s:s + v.numel()] = 41.0
        out[key] = flat[s:s + v.numel()].view(v.shape)
        s += v.numel()
    ref.load_state_dict(out)
    load_flat(model, flat.to(dev), Staging(), "result", chunk=chunk)
    for (k1, a), (k2, b) in zip(model.state_dict().items(), ref.state_dict().items()):
        assert k1 == k2 and a.dtype == b.dtype
        assert torch.equal(a, b), k1
