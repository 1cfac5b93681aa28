"""GPU: one- and multi-round gossip over the reference topologies with the HIP codec, bit-exact
against the same engine driven by the oracle on the CPU."""
import numpy as np
import pytest
import torch

from tests.test_cpu_gossip import EDGES16, EDGES96, _models, _oracle_encode, _oracle_fold, _train

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("path,n,alpha", [(EDGES16, 300_000, 0.01), (EDGES96, 40_000, 0.02)])
def test_gossip_round_device_matches_oracle(dev, path, n, alpha):
    from decentralizepy_amd.gossip import GossipRound, read_edges
    adj = read_edges(path)
    x = _models(len(adj), n)
    ref = GossipRound(adj, x, alpha, encode=_oracle_encode, fold=_oracle_fold)
    eng = GossipRound(adj, x.to(dev), alpha)
    for r in range(2):
        _train(ref, r)
        g = torch.Generator().manual_seed(100 + r)
        eng.x += (0.01 * torch.randn(len(adj), n, generator=g)).to(dev)
        ref.step()
        eng.step()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(eng.x.cpu().numpy().view(np.uint32),
                                      ref.x.numpy().view(np.uint32))
        np.testing.assert_array_equal(eng.counter.cpu().numpy(), ref.counter.numpy())
