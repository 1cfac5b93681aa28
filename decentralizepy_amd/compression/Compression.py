"""Identity compressor: the reference's base API (compression/Compression.py:1-78).

Loaded by ``Sharing.__init__`` as ``cls(float_precision=...)``; ``compress``/``decompress`` act
on index arrays, ``compress_float``/``decompress_float`` on value arrays, and the base class
returns its input unchanged.
"""


class Compression:
    """Compression API"""

    def __init__(self, *args, **kwargs):
        pass

    def compress(self, arr):
        return arr

    def decompress(self, bytes):
        return bytes

    def compress_float(self, arr):
        return arr

    def decompress_float(self, bytes):
        return bytes
