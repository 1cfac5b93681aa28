"""Oracle: block-floating fp32 value coding — TEST INFRASTRUCTURE ONLY.

The reference codes payload values with fpzip (``compression/EliasFpzip.py:19-51``, precision 0,
lossless; ``compression/EliasFpzipLossy.py:14-58``, precision p = 16 by default).  fpzip is not
in this image, so the build uses its own byte format (``csrc/dpz_fpz.hip``) and this module is
the numpy statement of that format — parity with fpzip's bytes is UNPINNED; what is pinned is
fpzip's contract: precision 0 round-trips every fp32 bit pattern, precision p keeps the p most
significant bits of each bit pattern (the rest truncated; from p = 10 on a NaN stays a NaN).

Format (little-endian uint32 words): header ``[MAGIC, n, precision (32 = lossless), nblk]``;
``nblk + 1`` block offsets (words from the start of the block area); per block of 256 values a
meta word ``emin | w << 8 | mb << 16`` and three LSB-first bit planes — sign (1 bit), exponent
minus ``emin`` (w = bit length of the block's exponent range), mantissa (mb bits) — each padded
to whole words.
"""
import numpy as np

MAGIC = 0x5A465044
BLOCK = 256


def mantissa_bits(precision):
    """(stored precision, mantissa bits) for a requested precision (0 or >= 32: lossless)."""
    precision = int(precision)
    if precision < 0:
        raise ValueError("precision must be >= 0")
    if precision == 0 or precision >= 32:
        return 32, 23
    return precision, max(precision - 9, 0)


def _pack(fields, bits):
    """LSB-first bit stream of ``bits``-bit fields, padded to whole uint32 words."""
    if bits == 0:
        return np.zeros(0, dtype=np.uint32)
    f = np.asarray(fields, dtype=np.uint64)
    stream = ((f[:, None] >> np.arange(bits, dtype=np.uint64)) & 1).astype(np.uint8).ravel()
    nw = (len(f) * bits + 31) // 32
    stream = np.concatenate([stream, np.zeros(nw * 32 - stream.size, dtype=np.uint8)])
    return (stream.reshape(nw, 32).astype(np.uint64) << np.arange(32, dtype=np.uint64)).sum(
        axis=1).astype(np.uint32)


def _unpack(words, cnt, bits):
    if bits == 0:
        return np.zeros(cnt, dtype=np.uint32)
    w = np.asarray(words, dtype=np.uint32).astype(np.uint64)
    stream = ((w[:, None] >> np.arange(32, dtype=np.uint64)) & 1).ravel()[:cnt * bits]
    return (stream.reshape(cnt, bits) << np.arange(bits, dtype=np.uint64)).sum(axis=1).astype(
        np.uint32)


def truncate_bits(u, precision):
    """The top ``precision`` bits of every fp32 bit pattern (uint32); from 10 bits on a NaN whose
    kept mantissa is zero gets the quiet bit, so it stays a NaN."""
    prec, _ = mantissa_bits(precision)
    u = np.asarray(u, dtype=np.uint32)
    if prec >= 32:
        return u.copy()
    t = u & np.uint32((0xFFFFFFFF << (32 - prec)) & 0xFFFFFFFF)
    nan = ((u & 0x7F800000) == 0x7F800000) & ((u & 0x7FFFFF) != 0) & ((t & 0x7FFFFF) == 0)
    if prec >= 10:
        t = np.where(nan, t | np.uint32(0x400000), t)
    return t.astype(np.uint32)


def truncate(x, precision):
    """What a lossy round trip returns."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32)
    return truncate_bits(u, precision).view(np.float32)


def encode(x, precision=0):
    prec, mb = mantissa_bits(precision)
    u = truncate_bits(np.ascontiguousarray(x, dtype=np.float32).ravel().view(np.uint32), prec)
    n = u.size
    nblk = (n + BLOCK - 1) // BLOCK
    blocks, table = [], [0]
    for b in range(nblk):
        ub = u[b * BLOCK:(b + 1) * BLOCK]
        e = (ub >> 23) & 0xFF
        emin = int(e.min())
        w = int(int(e.max()) - emin).bit_length()
        f = (ub & 0x7FFFFF) >> (23 - mb)
        words = np.concatenate([np.array([emin | (w << 8) | (mb << 16)], dtype=np.uint32),
                                _pack(ub >> 31, 1), _pack(e - emin, w), _pack(f, mb)])
        blocks.append(words)
        table.append(table[-1] + words.size)
    head = np.array([MAGIC, n, prec, nblk], dtype=np.uint32)
    parts = [head, np.array(table, dtype=np.uint32)] + blocks
    return np.concatenate(parts).astype("<u4").view(np.uint8)


def parse_header(buf):
    """(n, precision, nblk) of a stream; ValueError when it is not one."""
    b = np.frombuffer(memoryview(buf), dtype=np.uint8)
    if b.size < 16 or b.size % 4:
        raise ValueError("float stream: truncated header")
    magic, n, prec, nblk = (int(v) for v in b[:16].view("<u4"))
    if magic != MAGIC or nblk != (n + BLOCK - 1) // BLOCK or b.size < 4 * (4 + nblk + 1 + nblk):
        raise ValueError("float stream: bad header")
    mantissa_bits(prec)
    return n, prec, nblk


def decode(buf):
    n, prec, nblk = parse_header(buf)
    _, mb = mantissa_bits(prec)
    w32 = np.frombuffer(memoryview(buf), dtype="<u4").astype(np.uint32)
    table = w32[4:4 + nblk + 1]
    area = w32[4 + nblk + 1:]
    out = np.empty(n, dtype=np.uint32)
    for b in range(nblk):
        cnt = min(BLOCK, n - b * BLOCK)
        blk = area[table[b]:table[b + 1]]
        meta = int(blk[0])
        emin, w = meta & 0xFF, (meta >> 8) & 0xFF
        if w > 8 or (meta >> 16) & 0xFF != mb:
            raise ValueError("float stream: bad block")
        ns, ne = (cnt + 31) // 32, (cnt * w + 31) // 32
        s = _unpack(blk[1:1 + ns], cnt, 1)
        e = _unpack(blk[1 + ns:1 + ns + ne], cnt, w)
        f = _unpack(blk[1 + ns + ne:], cnt, mb)
        out[b * BLOCK:b * BLOCK + cnt] = (s << 31) | (((emin + e) & 0xFF) << 23) | (f << (23 - mb))
    return out.view(np.float32)
