"""GPU: the STC plugin (decentralizepy_amd/sharing/STC.py) replays the reference's own STC run
(tests/golden/stc.npz from the unmodified reference sharing/STC.py, see make_golden_stc.py)
bit-exactly through the HIP kernels: client payload + residuals, server _averaging_server total
+ model_change, server_broadcast payload + residuals + server model, client process_received."""
import json
import os
from collections import OrderedDict, deque

import numpy as np
import pytest

from tests import scenario

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def test_stc_client_server_rounds_match_reference(dev, tmp_path):
    from decentralizepy_amd.sharing.STC import STC
    meta = json.load(open(os.path.join(scenario.GOLDEN, "stc.json")))
    g = np.load(os.path.join(scenario.GOLDEN, "stc.npz"))
    shape = [meta["rows"], meta["cols"], meta["nb"]]
    cm, sm = scenario.make_model(shape), scenario.make_model(shape)
    scenario.set_flat(cm, g["xc0"])
    scenario.set_flat(sm, g["xs0"])
    kw = dict(alpha=meta["alpha"], compress=False, compression_package=None,
              compression_class=None)
    client = STC(0, 0, None, scenario._Mapping(), scenario._Graph([1]), cm, None, str(tmp_path),
                 **kw)
    server = STC(1, 0, None, scenario._Mapping(), scenario._Graph([0, 2, 3]), sm, None,
                 str(tmp_path), **kw)
    for r in range(meta["rounds"]):
        scenario.set_flat(cm, g[f"r{r}_x"])
        data = client.get_data_to_send()
        np.testing.assert_array_equal(data["indices"], g[f"r{r}_idx"])
        np.testing.assert_array_equal(_bits(data["params"]), _bits(g[f"r{r}_vals"]))
        np.testing.assert_array_equal(_bits(client.residuals.cpu().numpy()), _bits(g[f"r{r}_res"]))
        assert data["iteration"] == client.communication_round
        msgs = [dict(data)] + [{"alpha": meta["alpha"], "indices": g[f"r{r}_nbr{j}_idx"],
                                "params": g[f"r{r}_nbr{j}_vals"], "iteration": r}
                               for j in range(2)]
        peers = OrderedDict()
        for uid, m in zip((0, 2, 3), msgs):
            m = dict(m)
            m["degree"] = 1
            m["CHANNEL"] = "STC"
            peers[uid] = deque([m])
        total = server._averaging_server(peers)
        np.testing.assert_array_equal(_bits(total.numpy()), _bits(g[f"r{r}_total"]))
        np.testing.assert_array_equal(_bits(server.model.model_change.cpu().numpy()),
                                      _bits(g[f"r{r}_server_change"]))
        b = server.server_broadcast()
        np.testing.assert_array_equal(b["indices"], g[f"r{r}_b_idx"])
        np.testing.assert_array_equal(_bits(b["params"]), _bits(g[f"r{r}_b_vals"]))
        np.testing.assert_array_equal(_bits(server.residuals.cpu().numpy()),
                                      _bits(g[f"r{r}_server_res"]))
        np.testing.assert_array_equal(_bits(scenario.get_flat(sm)), _bits(g[f"r{r}_server_model"]))
        client.process_received({k: v for k, v in b.items() if k != "iteration"})
        np.testing.assert_array_equal(_bits(scenario.get_flat(cm)), _bits(g[f"r{r}_client_model"]))


@pytest.mark.parametrize("n,k", [(1000, 10), (1_000_003, 10_000), (11_000_000, 110_000)])
def test_zero_base_fold_and_add_scatter_match_oracle(dev, n, k):
    """DPZ_FOLD_ZERO_BASE (STC's total = sum w T_i) and DPZ_FOLD_ADD_ONLY (flat + T) vs the
    oracle, including -0.0 locals (fl(-0 + +0) = +0 as the reference's dense add)."""
    import torch

    from decentralizepy_amd import codec
    from oracle import stc as ostc
    rng = np.random.default_rng(n)
    local = rng.standard_normal(n).astype(np.float32)
    local[::7] = -0.0
    pays = []
    for j in range(3):
        idx = np.sort(rng.choice(n, size=k, replace=False)).astype(np.int32)
        pays.append((idx, rng.standard_normal(k).astype(np.float32)))
    tl = torch.from_numpy(local).to(dev)
    tp = [(torch.from_numpy(i).to(dev), torch.from_numpy(v).to(dev)) for i, v in pays]
    tot = codec.decode_average(tl, tp, [1 / 3] * 3, None, zero_base=True).cpu().numpy()
    ref, _ = ostc.averaging_server(np.zeros(n, np.float32), pays)
    np.testing.assert_array_equal(_bits(tot), _bits(ref))
    out = codec.decode_average(tl, tp[:1], add_only=True).cpu().numpy()
    np.testing.assert_array_equal(_bits(out), _bits(ostc.process_received(local, *pays[0])))
    empty = (torch.empty(0, dtype=torch.int32, device=dev), torch.empty(0, device=dev))
    out0 = codec.decode_average(tl, [empty], add_only=True).cpu().numpy()
    np.testing.assert_array_equal(_bits(out0), _bits(local + np.float32(0)))
