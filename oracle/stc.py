"""Oracle: STC sharing (sparse top-k with residual error feedback) — TEST INFRASTRUCTURE ONLY.

CPU restatement (numpy fp32, one rounding per operation, no FMA) of the reference's
``sharing/STC.py`` (sacs-epfl/decentralizepy), only ever imported by tests/:

* ``_pre_step``            STC.py:243-254  model_change = (flat - prev) + residuals; prev = flat
* ``extract_top_gradients`` STC.py:158-174 top-k of |model_change| (sorted=True), index sorted,
                                            values model_change[index]
* ``get_data_to_send``     STC.py:305-315  residuals = model_change - T(data)
* ``deserialized_model``   STC.py:207-241  T = zeros(n); T[idx] = params
* ``process_received``     STC.py:270-303  model = flat + T   (flat + 0 without a message)
* ``_averaging_server``    STC.py:333-362  total = zeros; total += (1/n) * T_i (payload order);
                                            model_change = residuals + total
* ``server_broadcast``     STC.py:317-331  top-k of the current model_change, residual update,
                                            process_received of its own message
"""
import numpy as np

from . import topk as otopk


def scatter_zero(n, idx, vals):
    """``T = zeros(n); T[idx] = params`` (STC.py:236-239)."""
    t = np.zeros(n, dtype=np.float32)
    if idx is not None and len(idx):
        t[np.asarray(idx, dtype=np.int64)] = np.asarray(vals, dtype=np.float32)
    return t


def encode(flat, prev, residuals, k):
    """One client encode: returns (idx int32, vals fp32, model_change, new residuals)."""
    flat = np.asarray(flat, dtype=np.float32)
    change = (flat - np.asarray(prev, dtype=np.float32)) + np.asarray(residuals, dtype=np.float32)
    return encode_change(change, k)


def encode_change(change, k):
    """top-k of an existing model_change (server_broadcast, STC.py:317-331)."""
    change = np.asarray(change, dtype=np.float32)
    idx = otopk.topk_select(otopk.keys_u32(change), k)
    vals = change[idx].copy()
    res = change - scatter_zero(change.shape[0], idx, vals)
    return idx.astype(np.int32), vals, change, res


def process_received(flat, idx=None, vals=None):
    """``flat + T`` (or ``flat + 0`` when no message arrived)."""
    flat = np.asarray(flat, dtype=np.float32)
    return flat + scatter_zero(flat.shape[0], idx, vals)


def averaging_server(residuals, payloads):
    """(total, model_change) of ``_averaging_server`` over ``payloads = [(idx, vals), ...]``."""
    residuals = np.asarray(residuals, dtype=np.float32)
    n = residuals.shape[0]
    total = np.zeros(n, dtype=np.float32)
    w = np.float32(1.0 / len(payloads))
    for idx, vals in payloads:
        total = total + w * scatter_zero(n, idx, vals)
    return total, residuals + total
