"""Oracle: the FFT sharing plugin's round — TEST INFRASTRUCTURE ONLY.

Restates in numpy what the reference ``sharing/JWINS/FFT.py`` computes per round:

* ``change_transformer_fft``   FFT.py:12-25        ``torch.fft.rfft(x)`` (complex64, n // 2 + 1)
* ``PartialModel._pre_step``   PartialModel.py:305-331 with T = rfft: F(x), change = F(x - x0),
  complex accumulation (``acc += change; change = acc`` or ``change += acc``)
* ``FFT.apply_fft``            FFT.py:132-156      ``topk(|change|)`` (or ``|F(x)|`` without
  change-based selection), sorted indices, values ``F(x)[index]``
* ``FFT.serialized_model``     FFT.py:158-211      full share at alpha >= metadata_cap (acc
  zeroed), else counter += 1 and the complex rewind at the indices
* ``FFT._averaging``           FFT.py:252-302      per payload ``topkf = F(local); topkf[idx] =
  params``, Metro-Hastings fold in payload order plus the self term, ``irfft``
* ``PartialModel._post_step``  PartialModel.py:333-353  ``acc += rfft(new - prev)``

The transforms are computed in float64 (numpy's pocketfft) and rounded to complex64 / float32;
torch's CPU path runs pocketfft in float32, so this oracle — like the device path, whose own fp32
mixed-radix kernels round differently again — agrees with the reference to a tolerance, not
bit-for-bit.  The selection, the fold order
(each complex entry as its (re, im) fp32 pair, one rounding per operation) and the bookkeeping
are the reference's.
"""
import numpy as np

from . import fold as ofold
from . import topk as otopk


def rfft(x):
    return np.fft.rfft(np.asarray(x, dtype=np.float64)).astype(np.complex64)


def irfft(c, n):
    return np.fft.irfft(np.asarray(c, dtype=np.complex128), n).astype(np.float32)


def cabs(c):
    """fp32 |c| = sqrt(re^2 + im^2), one rounding per operation."""
    c = np.asarray(c, dtype=np.complex64)
    re, im = c.real.astype(np.float32), c.imag.astype(np.float32)
    return np.sqrt(re * re + im * im).astype(np.float32)


def pair_indices(idx):
    idx = np.asarray(idx, dtype=np.int64)
    return np.stack([2 * idx, 2 * idx + 1], axis=1).reshape(-1)


class FFTNode:
    """numpy mirror of the reference FFT plugin's round logic."""

    def __init__(self, kwargs, x0):
        self.alpha = kwargs.get("alpha", 1.0)
        self.cap = kwargs.get("metadata_cap", 1.0)
        self.accumulation = kwargs.get("accumulation", False)
        self.aac = kwargs.get("accumulate_averaging_changes", False)
        self.cbs = kwargs.get("change_based_selection", True)
        self.n = x0.shape[0]
        self.m = self.n // 2 + 1
        self.init = np.asarray(x0, dtype=np.float32).copy()
        self.model = self.init.copy()
        self.prev = self.init
        self.acc = np.zeros(self.m, np.complex64) if self.accumulation else None
        self.counter = np.zeros(self.m, np.int32)

    def get_data_to_send(self):
        x = self.model.copy()
        self.fx = rfft(x)
        change = rfft(x - self.init)
        if self.accumulation:
            if not self.aac:
                self.acc += change
                change = self.acc.copy()
            else:
                change = change + self.acc
        if self.alpha >= self.cap:
            if self.acc is not None:
                self.acc[:] = 0
            return {"params": self.fx.copy()}
        k = round(self.alpha * self.m)
        key = cabs(change) if self.cbs else cabs(self.fx)
        idx = otopk.topk_select(otopk.keys_u32(key), k)
        self.counter[idx] += 1
        if self.acc is not None:
            self.acc[idx] = 0
        return {"alpha": self.alpha, "params": self.fx[idx].copy(),
                "indices": idx.astype(np.int32), "send_partial": True}

    def averaging(self, msgs):
        local_fx = rfft(self.model)
        pays, w = [], []
        for msg in msgs:
            vals = np.asarray(msg["params"], dtype=np.complex64).view(np.float32)
            pays.append((pair_indices(msg["indices"]), vals))
            w.append(ofold.mh_weight(len(msgs), msg["degree"]))
        wt = 0
        for v in w:
            wt += v
        total = ofold.fold(local_fx.view(np.float32), pays, w, 1 - wt)
        self.model = irfft(total.view(np.complex64), 2 * (self.m - 1))
        new = self.model.copy()
        if self.accumulation and self.aac:
            self.acc += rfft(new - self.prev)
        self.init = new
        if self.accumulation:
            self.prev = new
