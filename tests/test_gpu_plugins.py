"""GPU: the drop-in plugin classes replay the reference's recorded multi-round scenarios
bit-exactly (payload indices/params, counters, accumulators, averaged models)."""
import os
from collections import deque

import numpy as np
import pytest

from tests import scenario

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", scenario.scenario_names())
def test_plugin_replays_reference_scenario(name, dev, tmp_path):
    scenario.replay_plugin(name, tmp_path)


def test_sharing_full_model_fold(dev, tmp_path):
    from decentralizepy_amd.sharing.Sharing import Sharing
    meta = next(s for s in scenario.load_meta()["scenarios"] if s["name"] == "sharing_full")
    a = dict(np.load(os.path.join(scenario.GOLDEN, "sharing_full.npz")))
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
    plugin._averaging({uid: deque([m]) for uid, m in zip([1, 2, 3], msgs)})
    np.testing.assert_array_equal(scenario.get_flat(model).view(np.uint32),
                                  a["r0_model_after"].view(np.uint32))


def test_counter_dump_like_the_node(dev, tmp_path):
    """DPSGDNode.py:186-194 dumps model.shared_parameters_counter.numpy().tolist()."""
    plugin = scenario.replay_plugin("pm_a01_plain", tmp_path)
    counts = plugin.model.shared_parameters_counter.numpy().tolist()
    assert isinstance(counts, list) and sum(counts) == 2 * 410
