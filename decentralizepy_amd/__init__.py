"""decentralizepy_amd — MI355X-native model-update codec for decentralizepy's Sharing plugins.

Drop-in plugin classes live in ``decentralizepy_amd.sharing`` (Sharing, PartialModel,
JWINS.Wavelet, JWINS.JWINS) and ``decentralizepy_amd.compression``; the hand-written HIP
kernels behind them are reached through ``decentralizepy_amd.codec`` (ctypes over the C ABI in
``include/dpz_codec.h``).
"""
__version__ = "0.1.0"
