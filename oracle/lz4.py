"""Oracle: LZ4 frames — TEST INFRASTRUCTURE ONLY.

The reference's ``compression/Lz4Wrapper.py:20-98`` calls python-lz4's ``lz4.frame.compress`` /
``decompress`` (third-party, absent in this image).  python-lz4 is a binding of the C liblz4; its
``lz4.frame.compress`` defaults are: block_size = LZ4F_default (64 KB max), block_linked = True,
content_checksum = False, block_checksum = False, store_size = True, compression_level = 0
(LZ4F_compressFrame with acceleration 1).  This module

* ``ref_compress`` / ``ref_decompress``: the C liblz4 1.9.3 that ships in this image's conda
  (``/opt/conda/lib/liblz4.so.1.9.3``, NOT part of the reference) through ctypes, with those
  preferences — the frames a reference node would put on / accept from the wire, modulo the
  liblz4 version python-lz4 bundles (parity of the FORMAT, which the LZ4 frame spec fixes);
* ``decode_frame``: a pure-Python restatement of the LZ4 frame and block format (magic, FLG/BD,
  content size, header checksum = xxh32 >> 8, size-prefixed blocks with the uncompressed flag,
  end mark; sequences = token, literal length, literals, 16-bit offset, match length), pinned
  against ``ref_compress`` by tests/test_oracle_lz4.py;
* ``wrapper_compress`` / ``wrapper_decompress``: Lz4Wrapper's index leg on top of them.
"""
import ctypes
import os

import numpy as np

LIBLZ4 = "/opt/conda/lib/liblz4.so.1.9.3"
_lib = None


class _FrameInfo(ctypes.Structure):
    _fields_ = [("blockSizeID", ctypes.c_int), ("blockMode", ctypes.c_int),
                ("contentChecksumFlag", ctypes.c_int), ("frameType", ctypes.c_int),
                ("contentSize", ctypes.c_ulonglong), ("dictID", ctypes.c_uint),
                ("blockChecksumFlag", ctypes.c_int)]


class _Prefs(ctypes.Structure):
    _fields_ = [("frameInfo", _FrameInfo), ("compressionLevel", ctypes.c_int),
                ("autoFlush", ctypes.c_uint), ("favorDecSpeed", ctypes.c_uint),
                ("reserved", ctypes.c_uint * 3)]


def available():
    return os.path.exists(LIBLZ4)


def _l():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(LIBLZ4)
        _lib.LZ4F_compressFrameBound.restype = ctypes.c_size_t
        _lib.LZ4F_compressFrameBound.argtypes = [ctypes.c_size_t, ctypes.POINTER(_Prefs)]
        _lib.LZ4F_compressFrame.restype = ctypes.c_size_t
        _lib.LZ4F_compressFrame.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                            ctypes.c_size_t, ctypes.POINTER(_Prefs)]
        _lib.LZ4F_isError.restype = ctypes.c_uint
        _lib.LZ4F_isError.argtypes = [ctypes.c_size_t]
        _lib.LZ4F_createDecompressionContext.restype = ctypes.c_size_t
        _lib.LZ4F_createDecompressionContext.argtypes = [ctypes.POINTER(ctypes.c_void_p),
                                                         ctypes.c_uint]
        _lib.LZ4F_freeDecompressionContext.argtypes = [ctypes.c_void_p]
        _lib.LZ4F_decompress.restype = ctypes.c_size_t
        _lib.LZ4F_decompress.argtypes = [ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.POINTER(ctypes.c_size_t), ctypes.c_void_p,
                                         ctypes.POINTER(ctypes.c_size_t), ctypes.c_void_p]
    return _lib


def ref_compress(data, block_linked=True, block_size_id=0, store_size=True):
    """``lz4.frame.compress(data)`` with python-lz4's default preferences (liblz4 1.9.3)."""
    lib = _l()
    src = bytes(data)
    p = _Prefs()
    p.frameInfo.blockSizeID = block_size_id
    p.frameInfo.blockMode = 0 if block_linked else 1
    p.frameInfo.contentSize = len(src) if store_size else 0
    bound = lib.LZ4F_compressFrameBound(len(src), ctypes.byref(p))
    dst = ctypes.create_string_buffer(bound)
    r = lib.LZ4F_compressFrame(dst, bound, src, len(src), ctypes.byref(p))
    if lib.LZ4F_isError(r):
        raise RuntimeError("LZ4F_compressFrame failed")
    return dst.raw[:r]


def ref_decompress(frame, max_size=1 << 28):
    """``lz4.frame.decompress(frame)`` through liblz4 1.9.3."""
    lib = _l()
    ctx = ctypes.c_void_p()
    if lib.LZ4F_isError(lib.LZ4F_createDecompressionContext(ctypes.byref(ctx), 100)):
        raise RuntimeError("LZ4F context")
    src = bytes(frame)
    out = bytearray()
    chunk = ctypes.create_string_buffer(1 << 20)
    pos = 0
    try:
        while True:
            dn = ctypes.c_size_t(len(chunk))
            sn = ctypes.c_size_t(len(src) - pos)
            r = lib.LZ4F_decompress(ctx, chunk, ctypes.byref(dn),
                                    ctypes.c_char_p(src[pos:]), ctypes.byref(sn), None)
            if lib.LZ4F_isError(r):
                raise ValueError("malformed LZ4 frame (liblz4)")
            out += chunk.raw[:dn.value]
            pos += sn.value
            if r == 0:
                break
            if sn.value == 0 and dn.value == 0:
                raise ValueError("truncated LZ4 frame")
            if len(out) > max_size:
                raise ValueError("LZ4 frame larger than max_size")
    finally:
        lib.LZ4F_freeDecompressionContext(ctx)
    return bytes(out)


def _xxh32(b):
    import xxhash
    return xxhash.xxh32(b, seed=0).intdigest()


def _decode_block(src, out, hist_start):
    """One LZ4 block appended to ``out`` (matches may reach back to hist_start)."""
    i = 0
    n = len(src)
    while True:
        tok = src[i]
        i += 1
        L = tok >> 4
        if L == 15:
            while True:
                x = src[i]
                i += 1
                L += x
                if x != 255:
                    break
        out += src[i:i + L]
        i += L
        if i == n:
            return
        off = src[i] | (src[i + 1] << 8)
        i += 2
        M = tok & 15
        if M == 15:
            while True:
                x = src[i]
                i += 1
                M += x
                if x != 255:
                    break
        M += 4
        p = len(out) - off
        if off == 0 or p < hist_start:
            raise ValueError("match offset out of range")
        for t in range(M):
            out.append(out[p + t])


def decode_frame(frame):
    """Content of an LZ4 frame (pure Python restatement of the frame / block format)."""
    b = bytes(frame)
    if int.from_bytes(b[0:4], "little") != 0x184D2204:
        raise ValueError("bad magic")
    flg, bd = b[4], b[5]
    if flg >> 6 != 1:
        raise ValueError("bad version")
    pos = 6
    csize = None
    if flg & 0x08:
        csize = int.from_bytes(b[pos:pos + 8], "little")
        pos += 8
    if flg & 0x01:
        pos += 4
    if (_xxh32(b[4:pos]) >> 8) & 0xFF != b[pos]:
        raise ValueError("bad header checksum")
    pos += 1
    linked = not (flg & 0x20)
    out = bytearray()
    while True:
        sz = int.from_bytes(b[pos:pos + 4], "little")
        pos += 4
        if sz == 0:
            break
        data = b[pos:pos + (sz & 0x7FFFFFFF)]
        pos += (sz & 0x7FFFFFFF) + (4 if flg & 0x10 else 0)
        start = 0 if linked else len(out)
        if sz >> 31:
            out += data
        else:
            _decode_block(data, out, start)
    if csize is not None and csize != len(out):
        raise ValueError("content size mismatch")
    return bytes(out)


def wrapper_compress(arr):
    """Lz4Wrapper.compress (compress_metadata): sort in place, int32 gaps, frame."""
    arr.sort()
    return ref_compress(np.diff(arr, prepend=0).astype(np.int32).tobytes("C"))


def wrapper_decompress(frame):
    """Lz4Wrapper.decompress: int64 running sum of the int32 gaps."""
    return np.cumsum(np.frombuffer(decode_frame(frame), dtype=np.int32))
