"""LZ4 frame compressor on the MI355X codec.

Drop-in for ``decentralizepy.compression.Lz4Wrapper.Lz4Wrapper`` (compression/Lz4Wrapper.py):
the same constructor (``compress_metadata=True, compress_data=False``) and host surface —
``compress(np.int32[k])`` sorts its argument in place and returns an LZ4 frame of the int32 gaps
``np.diff(arr, prepend=0)``; ``decompress(frame)`` returns their running sum as int64;
``compress_float`` / ``decompress_float`` frame the fp32 bytes when ``compress_data`` (else they
pass the array through).  The frames are LZ4 frames any decoder reads (python-lz4 on a reference
node included): the gaps, the frame encode / decode and the running sum are HIP kernels
(csrc/dpz_lz4.hip).  The sharing plugins call the device entry points directly, so a payload's
indices go device -> frame -> host once.  Byte parity with python-lz4's own match finder is
unpinned (the frame FORMAT is pinned against liblz4 1.9.3, tests/test_gpu_lz4.py).
"""
import numpy as np
import torch

from .. import codec
from .._device import pick_device
from .Compression import Compression


class Lz4Wrapper(Compression):
    """Compression API"""

    def __init__(self, compress_metadata=True, compress_data=False, *args, **kwargs):
        self.compress_metadata = compress_metadata
        self.compress_data = compress_data
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
        """Sorted device int32 indices -> host LZ4 frame of their gaps (or, without
        compress_metadata, the host array as the reference returns it)."""
        self._dev(idx_dev.device)
        if not self.compress_metadata:
            return idx_dev.cpu().numpy()
        gaps = codec.delta_i32(idx_dev)
        frame = codec.lz4_compress(gaps.view(torch.uint8), workspace=self._ws)
        return frame.cpu().numpy().tobytes()

    def decompress_device(self, buf, dtype=torch.int32, device=None):
        """Host frame -> device running sum of the gaps (int32 for the fold kernels, or int64)."""
        dev = self._dev(device)
        if not self.compress_metadata:
            return torch.as_tensor(np.asarray(buf)).to(dev, dtype)
        raw = codec.lz4_decompress(buf, dev, workspace=self._ws)
        if raw.numel() % 4:
            raise ValueError("LZ4 index payload is not a whole number of int32 values")
        return codec.running_sum_i32(raw.view(torch.int32), dtype=dtype, workspace=self._ws)

    def compress_float_device(self, val_dev):
        self._dev(val_dev.device)
        if not self.compress_data:
            return val_dev.cpu().numpy()
        frame = codec.lz4_compress(val_dev.contiguous().view(torch.uint8), workspace=self._ws)
        return frame.cpu().numpy().tobytes()

    def decompress_float_device(self, buf, device=None):
        dev = self._dev(device)
        if not self.compress_data:
            return torch.as_tensor(np.asarray(buf, dtype=np.float32)).to(dev)
        raw = codec.lz4_decompress(buf, dev, workspace=self._ws)
        if raw.numel() % 4:
            raise ValueError("LZ4 value payload is not a whole number of fp32 values")
        return raw.view(torch.float32)

    # ---- reference host surface ----------------------------------------------------------------
    def compress(self, arr):
        """reference Lz4Wrapper.py:20-41: sorts ``arr`` in place."""
        if self.compress_metadata:
            arr.sort()
            idx = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.int32)).to(self._dev())
            return self.compress_device(idx)
        return arr

    def decompress(self, bytes):
        """reference Lz4Wrapper.py:43-61: int64 running sum of the decoded int32 gaps."""
        if self.compress_metadata:
            return self.decompress_device(bytes, dtype=torch.int64).cpu().numpy()
        return bytes

    def compress_float(self, arr):
        """reference Lz4Wrapper.py:63-80"""
        if self.compress_data:
            v = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.float32)).to(self._dev())
            return self.compress_float_device(v)
        return arr

    def decompress_float(self, bytes):
        """reference Lz4Wrapper.py:82-98"""
        if self.compress_data:
            return self.decompress_float_device(bytes).cpu().numpy()
        return bytes
