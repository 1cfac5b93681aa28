"""Elias indices + lossless float values (reference compression/EliasFpzip.py:8-51).

The reference codes values with ``fpzip.compress(arr, precision=0)``; fpzip is not available in
this image, so the lossless value leg here is the raw little-endian fp32 bytes.
Values round-trip bit-exactly, as with fpzip precision 0; the value byte format is this build's
own (parity of the float bytes with fpzip is unpinned).  The index leg is the device Elias codec.
"""
import numpy as np

from .Elias import Elias


class EliasFpzip(Elias):
    """Elias-gamma indices, lossless fp32 values."""

    def compress_float(self, arr):
        return np.ascontiguousarray(arr, dtype=np.float32).view(np.uint8).copy()

    def decompress_float(self, bytes):
        return np.frombuffer(memoryview(bytes), dtype=np.float32).copy().squeeze()
