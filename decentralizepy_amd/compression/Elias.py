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
from .._device import PayloadNames, Staging, host_copy_into, host_owned, pick_device
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


def stage_up(comp, b, need, device, leg):
    """Host stream bytes ``b`` -> a fresh device uint8 buffer of ``need`` bytes (zero padded),
    through a ring of pinned buffers kept with the compressor ``comp``: the DMA is asynchronous and
    a pinned slot is reused only after its own earlier DMA has completed, so the host copy of the
    next payload's stream overlaps this one's DMA and decode.  The device buffer comes from torch's
    caching allocator: freed, it is reused only by later work on the same stream."""
    if comp._staging is None:
        comp._staging = Staging()
        comp._names = PayloadNames(slots=3)
    name = comp._names(leg)  # a ring per leg kind: an index slot never grows to a value leg's size
    pin = comp._staging.get(name, need, torch.uint8)
    if pin is None:  # over the pinned cap: a pageable copy
        pad = np.zeros(need, dtype=np.uint8)
        pad[:b.size] = b
        return torch.from_numpy(pad).to(device)
    host_copy_into(pin[:b.size], b)
    pin[b.size:need].zero_()
    dbuf = torch.empty(need, dtype=torch.uint8, device=device)
    dbuf.copy_(pin, non_blocking=True)
    comp._staging.mark(name, torch.uint8, torch.cuda.current_stream(device))
    return dbuf


class Elias(Compression):
    """Elias-gamma coding of sorted index gaps."""

    # decompress_device takes (count, status): the asynchronous receive path of
    # PartialModel.decompress_data
    async_decode = True

    def __init__(self, *args, **kwargs):
        self.device = None
        self._ws = None
        self._staging = None
        self._names = None

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

    def decompress_device(self, buf, dtype=torch.int32, device=None, count=None, status=None):
        """Host stream -> device index tensor (int32 for the fold kernels, or int64).  With
        ``count`` (the payload's value count) and ``status`` (a device int32 word) the decode is
        asynchronous: no host synchronisation, the status word OR-ed nonzero when the stream is
        malformed or does not hold ``count`` values (``codec.elias_decode_async``)."""
        dev = self._dev(device)
        b = np.frombuffer(memoryview(buf), dtype=np.uint8)
        nbits, first = parse_trailer(b)
        nbytes = b.size
        need = ((nbytes + 3) // 4) * 4 + 16
        if status is not None:
            dbuf = stage_up(self, b, need, dev, "idx")
            return codec.elias_decode_async(dbuf, nbytes, nbits, first, int(count), status,
                                            dtype=dtype, workspace=self._ws)
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
