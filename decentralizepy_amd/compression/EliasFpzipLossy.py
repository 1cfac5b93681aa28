"""Elias indices + lossy block-floating values (reference compression/EliasFpzipLossy.py:8-58).

The reference calls ``fpzip.compress(arr, precision=float_precision)`` (16 by default): fpzip
keeps the ``float_precision`` most significant bits of every value.  fpzip is absent here; this
build's device codec (csrc/dpz_fpz.hip) keeps the same top bits of each fp32 bit pattern
(truncated; from 10 bits on a NaN stays a NaN) in its own block-floating format — ~62 % below raw
fp32 at 16 bits.  The plugins pass ``float_precision=None`` when a config names none (reference
sharing/Sharing.py:75); that selects the class default, 16.  Parity of the bytes with fpzip is
unpinned.
"""
from .EliasFpzip import EliasFpzip


class EliasFpzipLossy(EliasFpzip):
    """Elias-gamma indices, fp32 values truncated to ``float_precision`` bits."""

    def __init__(self, float_precision=16, *args, **kwargs):
        super().__init__(*args, **kwargs)
        if float_precision is None:
            float_precision = 16
        if int(float_precision) < 0:
            raise ValueError("float_precision must be >= 0 (0 = lossless)")
        self.float_precision = int(float_precision)
        self.precision = self.float_precision
