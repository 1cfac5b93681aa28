"""Oracle: top-k magnitude selection of the model change — TEST INFRASTRUCTURE ONLY.

Restates, in numpy, what the reference computes on the encode side:

* ``PartialModel._pre_step``          reference ``sharing/PartialModel.py:305-331``
  change = T(x - x0); with accumulation either ``acc += change; change = acc`` (:321-325)
  or ``change += acc`` (accumulate_averaging_changes, :326-329).
* ``PartialModel.extract_top_gradients``  reference ``sharing/PartialModel.py:164-186``
  ``topk(|change|, round(alpha*N))`` then ``sort(index)``.
* ``PartialModel.serialized_model``   reference ``sharing/PartialModel.py:205-246``
  ``shared_parameters_counter[idx] += 1``, ``rewind_accumulation(idx)`` (``models/Model.py:53-64``),
  values ``pre_share_model[idx]``.
* ``Wavelet.apply_wavelet``           reference ``sharing/JWINS/Wavelet.py:142-172`` (same selection
  on the wavelet-domain change, values from W(x)).

Ordering rule.  Keys are the fp32 bit patterns of |change| with the sign cleared, so unsigned
integer order is magnitude order; every NaN is canonicalised to 0x7FC00000 so NaNs rank above
+inf and tie with each other (torch.topk treats NaN as the largest value).  torch's CPU topk
breaks ties at the k-th key in an implementation-defined way; this
build's rule — shared by this oracle and the HIP kernels — is *lowest index wins*.  On inputs
with no tie at the k-th key the selected set is identical to torch's.
"""
import numpy as np

ACC_NONE = 0        # change = x - x0                  (accumulation off)
ACC_ACCUMULATE = 1  # acc += change; key = |acc|        (PartialModel.py:321-325)
ACC_ADD = 2         # key = |change + acc|, acc as-is   (PartialModel.py:326-329)

NAN_KEY = np.uint32(0x7FC00000)


def keys_u32(change):
    """|change| as order-preserving uint32 keys (sign cleared, NaNs canonicalised)."""
    b = np.ascontiguousarray(change, dtype=np.float32).view(np.uint32) & np.uint32(0x7FFFFFFF)
    return np.where(b > np.uint32(0x7F800000), NAN_KEY, b).astype(np.uint32)


def topk_select(keys, k):
    """Ascending int64 indices of the k largest keys; ties at the k-th key -> lowest index."""
    n = keys.shape[0]
    if k <= 0:
        return np.zeros(0, dtype=np.int64)
    if k >= n:
        return np.arange(n, dtype=np.int64)
    t = np.partition(keys, n - k)[n - k]          # the k-th largest key
    gt = np.flatnonzero(keys > t)
    ties = np.flatnonzero(keys == t)[: k - gt.shape[0]]
    return np.sort(np.concatenate([gt, ties])).astype(np.int64)


def kth_has_tie(keys, k):
    """True when the k-th largest key is shared by >1 element (torch parity undefined there)."""
    n = keys.shape[0]
    if k <= 0 or k >= n:
        return False
    t = np.partition(keys, n - k)[n - k]
    return int(np.count_nonzero(keys == t)) > 1


def encode(x, x0, acc, acc_mode, k, vals_src=None, counter=None):
    """One PartialModel/Wavelet partial-share encode.

    Mutates ``acc`` (accumulate + rewind) and ``counter`` in place exactly as the reference
    mutates ``model.accumulated_changes`` and ``model.shared_parameters_counter``.
    Returns ``(idx int32[k] ascending, val fp32[k])``.
    """
    x = np.asarray(x, dtype=np.float32)
    change = (x - np.asarray(x0, dtype=np.float32)) if x0 is not None else x.copy()
    if acc_mode == ACC_ACCUMULATE:
        acc += change
        key_src = acc
    elif acc_mode == ACC_ADD:
        key_src = change + acc
    else:
        key_src = change
    idx = topk_select(keys_u32(key_src), k)
    src = x if vals_src is None else np.asarray(vals_src, dtype=np.float32)
    val = src[idx].copy()
    if counter is not None:
        counter[idx] += 1
    if acc is not None and acc_mode != ACC_NONE:
        acc[idx] = 0.0
    return idx.astype(np.int32), val
