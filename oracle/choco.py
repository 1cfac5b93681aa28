"""Oracle: Choco-SGD sharing — TEST INFRASTRUCTURE ONLY.

CPU restatement (numpy fp32, one rounding per operation) of the reference's
``sharing/Choco.py`` (sacs-epfl/decentralizepy), only ever imported by tests/:

* ``topk_sparsification_tensor`` Choco.py:117-140  k = round(alpha n); if k > 0:
                                   cutoff = kthvalue(-|d|, k); d[|d| < -cutoff] = 0
* ``serialize_sparse_tensor``   Choco.py:148-161  indices = nonzero(q), values = q[indices]
* ``_pre_step``                 Choco.py:362-370  q = sparsify(x - x_hat)
* ``_averaging``                Choco.py:412-447  x_hat += q; s += w_i T_i (payload order,
                                   w_i = 1/(max(#nbrs, deg_i)+1)); s += (1 - sum w) q;
                                   x = x + step_size (s - x_hat)
"""
import numpy as np

from . import topk as otopk


def sparsify(d, k):
    """q = d with |d| < T zeroed (+0.0), T = the k-th largest |d| (all ties kept)."""
    q = np.array(d, dtype=np.float32, copy=True)
    if k > 0:
        keys = otopk.keys_u32(q)
        t = np.partition(keys, keys.shape[0] - k)[keys.shape[0] - k]
        q[keys < t] = np.float32(0.0)
    return q


def serialize(q):
    idx = np.flatnonzero(q)
    return idx.astype(np.int64), q[idx].copy()


def scatter_zero(n, idx, vals):
    t = np.zeros(n, dtype=np.float32)
    if len(idx):
        t[np.asarray(idx, dtype=np.int64)] = np.asarray(vals, dtype=np.float32)
    return t


def averaging(x, x_hat, s, q, payloads, degrees, step_size):
    """One ``_averaging``: returns (x_new, x_hat_new, s_new)."""
    x = np.asarray(x, dtype=np.float32)
    n = x.shape[0]
    x_hat = x_hat + np.float32(1.0) * q
    wt = 0
    for (idx, vals), deg in zip(payloads, degrees):
        w = 1 / (max(len(payloads), deg) + 1)
        wt += w
        s = s + scatter_zero(n, idx, vals) * np.float32(w)
    s = s + np.float32(1 - wt) * q
    x_new = x + np.float32(step_size) * (s - x_hat)
    return x_new, x_hat, s
