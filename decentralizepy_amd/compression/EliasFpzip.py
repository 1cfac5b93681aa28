"""Elias indices + lossless block-floating values (reference compression/EliasFpzip.py:8-51).

The reference codes values with ``fpzip.compress(arr, precision=0)``.  fpzip is not in this image
(SURVEY.md §8c), so the value leg is this build's own lossless format, coded on the device by
``dpz_fpz_encode`` / ``dpz_fpz_decode`` (csrc/dpz_fpz.hip): per 256 values a shared exponent base
and width, sign / exponent / mantissa bit planes — every fp32 bit pattern round-trips, and top-k
payload values come out ~12 % below raw fp32.  Parity of the bytes with fpzip is unpinned; the
index leg is the byte-identical device Elias codec.
"""
import numpy as np
import torch

from .. import codec
from .._device import host_copy_into, host_owned
from .Elias import Elias, _grown, stage_up

_MAGIC = 0x5A465044
_BLOCK = 256


def parse_float_header(buf):
    """(n, precision) of a block-floating stream; ValueError when ``buf`` is not one."""
    b = np.frombuffer(memoryview(buf), dtype=np.uint8)
    if b.size < 16 or b.size % 4:
        raise ValueError("float stream: truncated header")
    magic, n, prec, nblk = (int(v) for v in b[:16].view("<u4"))
    if magic != _MAGIC or nblk != (n + _BLOCK - 1) // _BLOCK or b.size < 4 * (5 + 2 * nblk):
        raise ValueError("float stream: bad header")
    return n, prec


class EliasFpzip(Elias):
    """Elias-gamma indices, lossless fp32 values."""

    precision = 0

    def compress_float_device(self, vals):
        """Device fp32 values -> host stream bytes (np.uint8, owned).  The stream comes down
        through a pinned buffer kept with the compressor (one DMA, then one host copy): a
        pageable ``.cpu()`` of a full share's 88 MB stream took 12-16 ms against 1.6 + 7-9.5 ms
        (tools/diag/d2h_probe.py on MI355X)."""
        self._dev(vals.device)
        x = vals.reshape(-1)
        if not x.is_contiguous():
            x = x.contiguous()
        s = codec.fpz_encode(x, self.precision, workspace=self._ws)
        pin = _grown(self._ws, "fpz_out_pin", s.numel(), dict(pin_memory=True))[:s.numel()]
        pin.copy_(s, non_blocking=True)
        torch.cuda.current_stream(s.device).synchronize()
        return host_owned(pin)

    def value_count(self, bytes):
        """The number of values a float stream holds (its header), without decoding it."""
        return parse_float_header(bytes)[0]

    def decompress_float_device(self, bytes, device=None, status=None):
        """Host stream bytes -> device fp32 values.  Up through a pinned buffer and into a
        device buffer, both kept with the compressor (fpz_decode synchronises before it returns,
        so both are free for the next call): one host copy into page-locked memory and a DMA —
        a fresh copy of the stream (page faults) plus a pageable transfer had cost ~4 ms per
        JWINS payload (tools/diag/plugin_breakdown.py).  With ``status`` (a device int32 word)
        the call does not synchronise: the stream goes up through the compressor's pinned ring
        and a malformed stream ORs the word nonzero."""
        dev = self._dev(device)
        n, prec = parse_float_header(bytes)
        b = np.frombuffer(memoryview(bytes), dtype=np.uint8)
        nb = b.size
        if status is not None:
            return codec.fpz_decode(stage_up(self, b, nb, dev, "vals"), n, prec, status=status)
        ws = self._ws
        pin = _grown(ws, "fpz_pin", nb, dict(pin_memory=True))
        dbuf = _grown(ws, "fpz_dev", nb, dict(device=dev))
        host_copy_into(pin[:nb], b)
        dbuf[:nb].copy_(pin[:nb], non_blocking=True)
        return codec.fpz_decode(dbuf[:nb], n, prec)

    def compress_float(self, arr):
        x = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.float32).reshape(-1))
        return self.compress_float_device(x.to(self._dev()))

    def decompress_float(self, bytes):
        return self.decompress_float_device(bytes).cpu().numpy().squeeze()
