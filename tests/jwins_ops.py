"""The numpy oracle behind decentralizepy_amd.gossip_jwins.JwinsRound — TEST INFRASTRUCTURE ONLY.

Same interface as ``HipJwinsOps``; every operation is the oracle restatement pinned by the
reference fixtures (oracle/wavelet.py, oracle/topk.py, oracle/fold.py), applied in place to CPU
torch tensors (their numpy views share memory), so the engine's round logic — alpha draws,
payload layout, all-gather offsets, neighbour order, post-step — runs unchanged on the CPU.
"""
import numpy as np
import torch

from oracle import fold as ofold
from oracle import topk as otopk
from oracle import wavelet as owav


def _np(t):
    return t.detach().cpu().numpy()


class OracleJwinsOps:
    def __init__(self, wavelet="sym2", level=4):
        self.wavelet, self.level = wavelet, level

    def transform_pair(self, x, x0, wx, wc):
        xn = _np(x)
        wx.copy_(torch.from_numpy(owav.wavedec_array(xn, self.level, self.wavelet)))
        wc.copy_(torch.from_numpy(owav.wavedec_array(xn - _np(x0), self.level, self.wavelet)))

    def encode(self, wc, k, acc, wx, counter, idx_out, val_out, status=None):
        a, c = acc.numpy(), counter.numpy()  # shared memory: mutated in place
        idx, val = otopk.encode(_np(wc), None, a, otopk.ACC_ADD, k, vals_src=_np(wx), counter=c)
        idx_out.copy_(torch.from_numpy(idx))
        val_out.copy_(torch.from_numpy(val))

    encode_exact = encode

    def missed(self, status):
        return []

    def fold_all(self, jobs, m_len):
        for local, pays, w, w_self, out in jobs:
            p = [(None if i is None else _np(i), _np(v)) for i, v in pays]
            out.copy_(torch.from_numpy(ofold.fold(_np(local), p, w, w_self)))

    def inverse(self, tot, n, out):
        out.copy_(torch.from_numpy(owav.waverec_array(_np(tot), n, self.level, self.wavelet)))

    def accumulate(self, acc, new, prev):
        a = acc.numpy()
        a += owav.wavedec_array(_np(new) - _np(prev), self.level, self.wavelet)


def coeff_len(n, level=4, wavelet="sym2"):
    return owav.coeff_len(n, level, wavelet)


def direct_round_nodes(adj, x, alpha_list, rounds, train, cap=0.5, level=4, wavelet="sym2"):
    """The reference JWINS semantics node by node with tests/scenario.OracleNode (pinned by the
    reference's own JWINS / Wavelet fixtures): every node draws alpha from random.Random(uid),
    encodes, and folds its neighbours' messages in neighbour-set order."""
    import random

    from tests.scenario import OracleNode
    meta = {"class": "Wavelet", "kwargs": {"wavelet": wavelet, "level": level,
                                           "metadata_cap": cap, "accumulation": True,
                                           "accumulate_averaging_changes": True,
                                           "change_based_selection": True}}
    nodes = [OracleNode(meta, np.asarray(x[i], np.float32).copy()) for i in range(len(adj))]
    rngs = [random.Random(u) for u in range(len(adj))]
    for r in range(rounds):
        for i, nd in enumerate(nodes):
            nd.model = nd.model + train(r, i)
        msgs = []
        for i, nd in enumerate(nodes):
            nd.alpha = rngs[i].choice(alpha_list)
            m = nd.get_data_to_send()
            m["degree"] = len(adj[i])
            msgs.append(m)
        for i, nd in enumerate(nodes):
            nd.averaging([msgs[q] for q in adj[i]])
    return nodes
