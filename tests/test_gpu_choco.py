"""GPU: the Choco plugin (decentralizepy_amd/sharing/Choco.py) replays the reference's own Choco
runs (tests/golden/choco.npz from the unmodified reference sharing/Choco.py) bit-exactly through
the HIP kernels, and the threshold selection (every tie kept, nonzero filter) matches the oracle
at sizes the sampled top-k never sees."""
import json
import os
from collections import OrderedDict, deque

import numpy as np
import pytest

from tests import scenario

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def _flat(sd):
    import torch
    return torch.cat([v.flatten() for v in sd.values()]).numpy()


@pytest.mark.parametrize("tag", ["a", "z"])
def test_choco_rounds_match_reference(dev, tmp_path, tag):
    from decentralizepy_amd.sharing.Choco import Choco
    meta = json.load(open(os.path.join(scenario.GOLDEN, "choco.json")))[tag]
    g = np.load(os.path.join(scenario.GOLDEN, "choco.npz"))
    model = scenario.make_model(meta["shape"])
    scenario.set_flat(model, g[f"{tag}_x0"])
    node = Choco(0, 0, None, scenario._Mapping(), scenario._Graph([1, 2, 3]), model, None,
                 str(tmp_path), step_size=meta["step_size"], alpha=meta["alpha"])
    for r, rm in enumerate(meta["rounds"]):
        scenario.set_flat(model, g[f"{tag}_r{r}_x"])
        data = node.get_data_to_send(degree=3)
        assert data["indices"].dtype == np.int64
        np.testing.assert_array_equal(data["indices"], g[f"{tag}_r{r}_idx"])
        np.testing.assert_array_equal(_bits(data["params"]), _bits(g[f"{tag}_r{r}_vals"]))
        peers = OrderedDict()
        for j, uid in enumerate((1, 2, 3)):
            peers[uid] = deque([{"params": g[f"{tag}_r{r}_nbr{j}_vals"],
                                 "indices": g[f"{tag}_r{r}_nbr{j}_idx"], "send_partial": True,
                                 "degree": rm["degrees"][j], "iteration": r,
                                 "CHANNEL": "DPSGD"}])
        node._averaging(peers)
        np.testing.assert_array_equal(_bits(scenario.get_flat(model)),
                                      _bits(g[f"{tag}_r{r}_x_after"]))
        np.testing.assert_array_equal(_bits(_flat(node.model_hat)), _bits(g[f"{tag}_r{r}_x_hat"]))
        np.testing.assert_array_equal(_bits(_flat(node.s)), _bits(g[f"{tag}_r{r}_s"]))


@pytest.mark.parametrize("n,alpha,quant", [(1_000_003, 0.01, False), (1_000_003, 0.05, True),
                                           (4_000_000, 0.0, True), (11_000_000, 0.01, False)])
def test_threshold_select_matches_oracle(dev, n, alpha, quant):
    import torch

    from decentralizepy_amd import codec
    from oracle import choco as ochoco
    rng = np.random.default_rng(n)
    d = (0.01 * rng.standard_normal(n)).astype(np.float32)
    if quant:
        d = (np.round(d * 400) / 400).astype(np.float32)  # heavy ties, exact zeros
        d[::9] = -0.0
    k = round(alpha * n)
    q = ochoco.sparsify(d, k)
    oi, ov = ochoco.serialize(q)
    td = torch.from_numpy(d).to(dev)
    ws = codec.Workspace(dev)
    idx, vals = codec.topk_threshold(td, k, workspace=ws)
    np.testing.assert_array_equal(idx.cpu().numpy().astype(np.int64), oi)
    np.testing.assert_array_equal(_bits(vals.cpu().numpy()), _bits(ov))
    gq = codec.mask_below_threshold(td, ws, out=torch.empty_like(td)).cpu().numpy()
    np.testing.assert_array_equal(_bits(gq), _bits(q))
