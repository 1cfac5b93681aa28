"""GPU: the bench's ``stages.product_one_node`` times exactly the device work the drop-in
PartialModel plugin enqueues for a node's round (bench.plugin_device_round drives the plugin's own
methods): the same kernel launches as a full host-to-host round through get_data_to_send and
_averaging (reference sharing/PartialModel.py:188-331, sharing/Sharing.py:156-190), and the
same payload and averaged model."""
from collections import deque

import numpy as np
import pytest
import torch

import bench

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("deg", [1, 3])
def test_bench_round_launches_what_the_plugin_round_launches(dev, tmp_path, deg):
    from decentralizepy_amd import codec
    from decentralizepy_amd.sharing.PartialModel import PartialModel
    n, alpha = 1_000_003, 0.01
    k = round(alpha * n)
    g = torch.Generator().manual_seed(5)
    x0 = torch.randn(n, generator=g)
    xs = [x0 + 0.01 * torch.randn(n, generator=g) for _ in range(2)]
    rng = np.random.default_rng(6)
    pays = [[(np.sort(rng.choice(n, size=k, replace=False)).astype(np.int32),
              rng.standard_normal(k).astype(np.float32)) for _ in range(deg)] for _ in range(2)]

    # the plugin, host to host (Node's calls)
    model = bench._bench_model(n)
    with torch.no_grad():
        model.weight.copy_(x0)
    plugin = PartialModel(0, 0, None, bench._BenchMapping(), bench._BenchGraph(deg), model, None,
                          str(tmp_path), alpha=alpha)
    host_counts, host_out = None, None
    for r in range(2):
        with torch.no_grad():
            model.weight.copy_(xs[r])
        with codec.KernelTimer() as kt:
            data = plugin.get_data_to_send(degree=deg)
            peer = {u: deque([{"alpha": alpha, "indices": i, "params": v, "send_partial": True,
                               "degree": deg, "iteration": r, "CHANNEL": "DPSGD"}])
                    for u, (i, v) in zip(range(1, deg + 1), pays[r])}
            plugin._averaging(peer)
        host_counts = {nm: c for nm, (_, c) in kt.result.items()}
        host_out = model.weight.detach().numpy().copy()
        host_idx = np.asarray(data["indices"]).copy()

    # the bench's device round (same inputs, already in HBM)
    bp = bench.make_bench_plugins(1, n, alpha, deg, dev)[0]
    init = x0.to(dev)
    for r in range(2):
        dpays = [(torch.from_numpy(i).to(dev), torch.from_numpy(v).to(dev)) for i, v in pays[r]]
        torch.cuda.synchronize()
        with codec.KernelTimer() as kt:
            idx, _, out = bench.plugin_device_round(bp, xs[r].to(dev), init, dpays, [deg] * deg)
            torch.cuda.synchronize()
        init = out
    dev_counts = {nm: c for nm, (_, c) in kt.result.items()}
    assert dev_counts == host_counts  # (a prior window that missed re-runs in both alike)
    np.testing.assert_array_equal(idx.cpu().numpy(), host_idx)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), host_out.view(np.uint32))
    # the counters agree too (the host plugin's is read through its ring)
    np.testing.assert_array_equal(bp.model.shared_parameters_counter.numpy(),
                                  plugin.model.shared_parameters_counter.numpy())
