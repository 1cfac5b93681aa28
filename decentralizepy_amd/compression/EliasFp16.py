"""Elias indices + fp16 values packed on the device (this build's codec for large-N configs).

Stands in for the reference's lossy fpzip leg (compression/EliasFpzipLossy.py:14-58), which is
not reproducible here (fpzip absent): values are rounded to IEEE half (round-to-nearest-even) by
``dpz_pack_fp16`` and widened back by ``dpz_unpack_fp16``.  Not byte-compatible with fpzip.
"""
import numpy as np
import torch

from .. import codec
from .Elias import Elias


class EliasFp16(Elias):
    """Elias-gamma indices, fp16 values."""

    def compress_float(self, arr):
        x = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.float32)).to(self._dev())
        return codec.pack_fp16(x).cpu().numpy().view(np.uint8)

    def decompress_float(self, bytes):
        h = np.frombuffer(memoryview(bytes), dtype=np.float16).copy()
        x = codec.unpack_fp16(torch.from_numpy(h).to(self._dev()))
        return x.cpu().numpy().squeeze()
