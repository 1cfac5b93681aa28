"""Oracle: decode (replace) + Metro-Hastings weighted fold — TEST INFRASTRUCTURE ONLY.

Restates the receive side of the reference in fp32 with the reference's operation order:

* ``PartialModel.deserialized_model``  reference ``sharing/PartialModel.py:257-303``:
  ``T = cat(local); T[idx] = params`` (REPLACE, not add).
* ``Sharing._averaging``               reference ``sharing/Sharing.py:156-190``:
  ``w_i = 1/(max(#nbrs, deg_i)+1)`` (Python double, rounded to fp32 by the tensor multiply);
  ``total = T_0*w_0`` then ``total += T_i*w_i`` in payload order, then
  ``total += (1 - sum w)*local``.
* ``Sharing._averaging_server``        reference ``sharing/Sharing.py:200-229``: ``w = 1/n``, no
  self term.
* ``Wavelet._averaging``               reference ``sharing/JWINS/Wavelet.py:269-309``: the same fold
  on wavelet coefficients (full payloads replace every coefficient).

Every product and sum is a single fp32 rounding (numpy float32 ops never contract to FMA).
"""
import numpy as np


def mh_weight(n_neighbors, degree):
    """Metro-Hastings weight as the reference computes it (Python double)."""
    return 1 / (max(n_neighbors, degree) + 1)


def replace(local, idx, vals):
    """``T = local.copy(); T[idx] = vals`` (``PartialModel.py:292-295``)."""
    t = np.array(local, dtype=np.float32, copy=True)
    if idx is None:
        return np.asarray(vals, dtype=np.float32).copy()
    t[np.asarray(idx, dtype=np.int64)] = np.asarray(vals, dtype=np.float32)
    return t


def fold(local, payloads, weights, w_self=None):
    """Weighted fold of replaced payloads.

    payloads : list of ``(idx or None, vals)``; ``idx=None`` means a dense (full-model) payload.
    weights  : per-payload weights (Python floats; rounded to fp32 here as torch does).
    w_self   : weight of the local term (``1 - sum(weights)`` computed in double by the caller),
               or None for the server variant (no self term).
    """
    local = np.asarray(local, dtype=np.float32)
    total = None
    for (idx, vals), w in zip(payloads, weights):
        term = replace(local, idx, vals) * np.float32(w)
        total = term if total is None else total + term
    if total is None:
        total = np.zeros_like(local)
    if w_self is not None:
        total = total + local * np.float32(w_self)
    return total
