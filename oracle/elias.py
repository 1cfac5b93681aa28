"""Oracle: Elias-gamma coding of sorted index gaps — TEST INFRASTRUCTURE ONLY.

Restates ``compression/Elias.py`` of the reference:

* ``Elias.compress``   reference ``compression/Elias.py:20-52``: sort (in place) -> ``first = a[0]``;
  gaps ``g = diff(a)`` (uint32); ``l = floor(log2 g)``; each gap coded as ``l`` zero bits followed
  by ``g`` in ``l+1`` bits MSB-first; codes concatenated; 128 zero bits appended; ``np.packbits``
  (MSB-first per byte); bytes ``[-16:-8]`` = int64-LE ``first``; bytes ``[-8:]`` = int64-LE total
  bit count (payload bits + 128).
* ``Elias.decompress`` reference ``compression/Elias.py:54-97``: walk the codes, cumulative sum from
  ``first``; returns int64.

Known-answer vector (reproduced from the reference here):
``compress(int32[10,3,6,5])`` -> ``520003000000000000008900000000000000`` (18 bytes).
"""
import numpy as np


def encode(idx):
    a = np.sort(np.asarray(idx).astype(np.int64))
    first = a[0]                                   # IndexError on empty input, as the reference
    g = np.diff(a).astype(np.int32).view(np.uint32).astype(np.uint64)
    if g.shape[0] == 0:
        raise IndexError("index -1 is out of bounds for axis 0 with size 0")
    l = np.floor(np.log2(g.astype(np.float64))).astype(np.int64)
    lens = 2 * l + 1
    ends = np.cumsum(lens)
    nbits = int(ends[-1]) + 128
    bits = np.zeros(nbits, dtype=np.uint8)
    for b in range(int(l.max()) + 1):
        m = l >= b
        bits[ends[m] - 1 - b] = ((g[m] >> np.uint64(b)) & np.uint64(1)).astype(np.uint8)
    packed = np.packbits(bits)
    packed[-8:] = np.frombuffer(np.int64(nbits).tobytes(), dtype=np.uint8)
    packed[-16:-8] = np.frombuffer(np.int64(first).tobytes(), dtype=np.uint8)
    return packed


def decode(data):
    data = np.frombuffer(bytes(data), dtype=np.uint8)
    nbits = int(np.frombuffer(data[-8:].tobytes(), dtype=np.int64)[0])
    first = int(np.frombuffer(data[-16:-8].tobytes(), dtype=np.int64)[0])
    bits = np.unpackbits(data[:-16])
    payload = nbits - 128
    out = [first]
    pos = 0
    while pos < payload:
        l = 0
        while bits[pos + l] == 0:
            l += 1
        g = 0
        for t in range(l + 1):
            g = (g << 1) | int(bits[pos + l + t])
        out.append(g)
        pos += 2 * l + 1
    return np.cumsum(np.asarray(out, dtype=np.int64))
