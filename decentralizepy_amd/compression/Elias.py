"""Elias-gamma index compressor on the MI355X codec (byte-identical to the reference).

Drop-in for ``decentralizepy.compression.Elias.Elias`` (compression/Elias.py:15-97): the same
host surface (``compress(np.int32[k]) -> np.uint8[...]`` sorting its argument in place,
``decompress(bytes) -> np.int64[k]``), with the bit packing and the code-boundary chase running as
HIP kernels (``dpz_elias_encode`` / ``dpz_elias_decode``).  The sharing plugins call the device
entry points ``compress_device`` / ``decompress_device`` directly, so a payload's indices go
device -> stream -> host once instead of through a host round trip.
"""
import numpy as np
import torch

from .. import codec
from .._device import host_copy_into, host_owned, pick_device
from .Compression import Compression


def parse_trailer(buf):
    """(nbits, first) from the last 16 bytes (int64 LE each, reference Elias.py:48-51, 72-76)."""
    b = np.frombuffer(memoryview(buf), dtype=np.uint8)
    if b.size < 16:
        raise ValueError("Elias stream shorter than its 16-byte trailer")
    first = int(b[-16:-8].view("<i8")[0])
    nbits = int(b[-8:].view("<i8")[0])
    return nbits, first


def _grown(ws, name, n, kw):
    """A uint8 buffer of at least n bytes kept on the workspace object under ``name``; grown
    geometrically (payload sizes vary round to round: JWINS draws alpha per round), so pinned
    allocations stay rare."""
    buf = getattr(ws, name, None)
    if buf is None or buf.numel() < n:
        size = max(n, 4096, 0 if buf is None else min(2 * buf.numel(), n + (n >> 1)))
        buf = torch.empty(size, dtype=torch.uint8, **kw)
        setattr(ws, name, buf)
    return buf


class Elias(Compression):
    """Elias-gamma coding of sorted index gaps."""

    def __init__(self, *args, **kwargs):
        self.device = None
        self._ws = None

    # ---- device ----------------------------------------------------------------------------------
    def _dev(self, device=None):
        if device is not None:
            self.device = torch.device(device)
        if self.device is None:
            self.device = pick_device(0)
        if self._ws is None or self._ws.device != self.device:
            self._ws = codec.Workspace(self.device)
        return self.device

    def compress_device(self, idx_dev):
        """Strictly increasing device int32 indices -> host uint8 stream."""
        self._dev(idx_dev.device)
        enc = codec.elias_encode(idx_dev, workspace=self._ws)
        # down through a kept pinned buffer, then one host copy (no pageable transfer)
        pin = _grown(self._ws, "elias_out_pin", enc.numel(), dict(pin_memory=True))[:enc.numel()]
        pin.copy_(enc, non_blocking=True)
        torch.cuda.current_stream(enc.device).synchronize()
        return host_owned(pin)

    def decompress_device(self, buf, dtype=torch.int32, device=None):
        """Host stream -> device index tensor (int32 for the fold kernels, or int64)."""
        dev = self._dev(device)
        b = np.frombuffer(memoryview(buf), dtype=np.uint8)
        nbits, first = parse_trailer(b)
        nbytes = b.size
        need = ((nbytes + 3) // 4) * 4 + 16
        # up through a pinned buffer into a device buffer, both kept with the compressor (the
        # decode synchronizes before it returns, so both are free again for the next call)
        ws = self._ws
        pin = _grown(ws, "elias_pin", need, dict(pin_memory=True))
        dbuf = _grown(ws, "elias_dev", need, dict(device=dev))
        host_copy_into(pin[:nbytes], b)
        pin[nbytes:need].zero_()
        dbuf[:need].copy_(pin[:need], non_blocking=True)
        dbuf = dbuf[:need]
        count = max(nbits - 128, 0) + 1
        return codec.elias_decode(dbuf, nbytes, nbits, first, count, dtype=dtype,
                                  workspace=self._ws)

    # ---- reference host surface ----------------------------------------------------------------
    def compress(self, arr):
        """reference Elias.py:20-52: sorts ``arr`` in place, returns the packed stream."""
        if arr.size < 2:
            raise IndexError("index 0 is out of bounds" if arr.size == 0 else
                             "list index out of range")
        if np.any(arr[1:] < arr[:-1]):
            arr.sort()
        idx = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.int32)).to(self._dev())
        return self.compress_device(idx)

    def decompress(self, bytes):
        """reference Elias.py:54-97: int64 values."""
        return self.decompress_device(bytes, dtype=torch.int64).cpu().numpy()
