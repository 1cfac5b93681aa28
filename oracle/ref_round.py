"""The reference's CPU op sequences for whole node rounds — TEST/BASELINE INFRASTRUCTURE ONLY.

``bench_workloads.py`` times these as the ``cpu_baseline`` of its workloads (kind "port"): the
ATen-CPU calls the reference issues, on torch CPU tensors, with pywt (absent from this image's
python3.10) replaced by this repo's NumPy restatement of its sym2 transforms (oracle/wavelet.py,
pinned to PyWavelets 1.1.1's outputs).  Nothing here is imported by the product package.

* :func:`partial_node` — a PartialModel node's round (C4 node / C2 / C5): encode
  (``sharing/PartialModel.py:164-246``, oracle/ref_ops.py) and ``Sharing._averaging`` over the
  neighbours' payloads, each deserialized as ``T = cat(local); T[idx] = params``
  (``PartialModel.py:257-303``, ``Sharing.py:156-190``), optionally with fp16 values
  (``params.half()``, BASELINE config 5's value packing).
* :func:`wavelet_node` — a JWINS / Wavelet node's round with the tutorial settings
  (change_based_selection, accumulation, accumulate_averaging_changes): ``_pre_step``
  (``PartialModel.py:305-331`` with the wavelet transform, ``Wavelet.py:12-32``: W(x), W(x - x0),
  change += acc), ``apply_wavelet`` (``Wavelet.py:142-172``: topk(sorted=False), sort), the
  counter and the rewind (``Wavelet.py:194-197``), ``_averaging`` (``Wavelet.py:269-329``: per
  payload clone + fill, the MH sums, waverec) and ``_post_step``'s accumulation
  (``PartialModel.py:340-350``: acc += W(x_new - prev)).
"""
import numpy as np
import torch

from oracle import ref_ops
from oracle import wavelet as owav


def partial_node(x, x0, alpha, counter, payloads, weights, fp16=False):
    """One node: encode its model, then fold the neighbours' (idx, params) payloads over it."""
    idx, vals = ref_ops.encode(x, x0, alpha, counter)                  # PartialModel.py:164-246
    if fp16:
        vals = torch.from_numpy(vals).half().numpy()                   # value packing (C5)
    total = None
    weight_total = 0
    for (pi, pv), w in zip(payloads, weights):                         # Sharing.py:156-190
        pv = np.asarray(pv, dtype=np.float32)
        t = ref_ops.decode(x, pi, pv)                                  # PartialModel.py:283-295
        weight_total += w
        total = t * w if total is None else total + t * w
    total += (1 - weight_total) * x
    return idx, vals, total


def wavelet_node(x, x0, acc, alpha, counter, payloads, weights, level=4, wavelet="sym2"):
    """One JWINS node round (tutorial settings); returns the new model and updates acc / counter
    in place (torch CPU tensors)."""
    wx = torch.from_numpy(owav.wavedec_array(x.numpy(), level, wavelet))       # Wavelet.py:12-32
    change = torch.from_numpy(owav.wavedec_array((x - x0).numpy(), level, wavelet))
    change += acc                                                       # PartialModel.py:322-327
    k = round(alpha * change.shape[0])
    _, index = torch.topk(change.abs(), k, dim=0, sorted=False)        # Wavelet.py:158-170
    index, _ = torch.sort(index)
    vals = wx[index]                                                    # Wavelet.py:172
    counter[index] += 1                                                 # Wavelet.py:194
    acc[index] = 0.0                                                    # Model.py:53-64 rewind
    total = None
    weight_total = 0
    for (pi, pv), w in zip(payloads, weights):                         # Wavelet.py:269-310
        t = wx.clone().detach()
        t[torch.as_tensor(pi, dtype=torch.long)] = torch.as_tensor(pv)
        weight_total += w
        total = w * t if total is None else total + w * t
    total += (1 - weight_total) * wx
    new = torch.from_numpy(owav.waverec_array(total.numpy(), x.shape[0], level, wavelet))
    acc += torch.from_numpy(owav.wavedec_array((new - x0).numpy(), level, wavelet))  # :340-350
    return index, vals, new
