"""CPU oracle for the decentralizepy model-update codec — TEST INFRASTRUCTURE ONLY.

This package restates, in plain numpy, the reference algorithms on the hot path so
that the HIP kernels can be checked against them:

  * ``topk``    — PartialModel/Wavelet top-k magnitude selection
                  (reference ``sharing/PartialModel.py:164-255``, ``sharing/JWINS/Wavelet.py:142-231``)
  * ``fold``    — replace-then-Metro-Hastings fold
                  (reference ``sharing/Sharing.py:156-229``, ``sharing/PartialModel.py:257-303``,
                  ``sharing/JWINS/Wavelet.py:269-385``)
  * ``wavelet`` — pywt-exact fp32 sym2 wavedec / waverec
                  (reference ``sharing/JWINS/Wavelet.py:12-32, 311-316``)
  * ``elias``   — Elias-gamma index codec (reference ``compression/Elias.py:20-97``)
  * ``ref_ops`` — the reference's own torch-CPU op sequence, used as the timed CPU baseline.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this package, and only as the checker / the baseline being timed.  The product
path (``decentralizepy_amd``) never imports it and fails loudly when the HIP library is
missing.

Parity pinning: the restatement is checked against golden vectors produced by the
unmodified reference classes (``tests/golden/make_golden.py``) and, for the wavelet,
against PyWavelets 1.1.1 (the version the reference was exercised with in this image).
"""
