"""Oracle: pywt-exact fp32 sym2 and haar multilevel DWT / IDWT — TEST INFRASTRUCTURE ONLY.

The reference calls PyWavelets (third-party, not vendored):

* ``change_transformer_wavelet``  reference ``sharing/JWINS/Wavelet.py:12-32``:
  ``pywt.wavedec(x, "sym2", level=4)`` (mode "symmetric") then ``pywt.coeffs_to_array`` ->
  the 1-D concatenation ``[cA_L, cD_L, ..., cD_1]``.
* ``Wavelet._averaging``          reference ``sharing/JWINS/Wavelet.py:311-316``:
  ``pywt.array_to_coeffs`` + ``pywt.waverec``; the caller keeps the first N outputs.

Dependency: PyWavelets 1.1.1 (the build present in this image's /opt/conda python3.9; the
reference's setup.cfg pins no version).  Its published C algorithm
(``downsampling_convolution`` / ``upsampling_convolution_valid_sf``) is restated below with the
exact fp32 summation order, verified bit-for-bit against pywt 1.1.1 by
``tests/golden/make_golden.py`` (fixtures ``tests/golden/wavelet_*.npz``):

forward, output o (input position i = 2o+1), half-sample symmetric extension
``x~[-1-m] = x[m]``, ``x~[n+m] = x[n-1-m]``::

    out[o] = ((f0*x~[i] + f1*x~[i-1]) + f2*x~[i-2]) + f3*x~[i-3]

except the last output when n is odd (i = n+2), where pywt's right-overhang loop visits the
extension first::

    out[last] = ((f2*x~[n] + f1*x~[n+1]) + f0*x~[n+2]) + f3*x~[n-1]

inverse (valid part, F/2 = 2 taps per phase), for m in [0, n-1)::

    y[2m+p] = (r[p]*a[m+1] + r[p+2]*a[m]) + (h[p]*d[m+1] + h[p+2]*d[m])

(approximation branch summed first into the zeroed output, detail branch added after).

haar (the reference Wavelet's default, ``Wavelet.py:56``), F = 2: no left overhang, so::

    out[o] = f0*x~[2o+1] + f1*x~[2o]          x~[n] = x[n-1] for odd n
    y[2m+p] = r[p]*a[m] + h[p]*d[m]            (output length 2 len(a))

verified bit-for-bit against pywt 1.1.1 (fixtures ``tests/golden/wavelet_haar_pywt.npz``).

Any other pywt discrete wavelet (filter length F even, <= 64; banks from
``decentralizepy_amd/wavelet_filters.json``, generated from pywt 1.1.1 by
``tools/gen_wavelet_filters.py``) follows the same C loops with F taps (``_dwt1_generic`` /
``_idwt1_generic``, needing every level's input length >= F: one reflection per side), every sum
started from 0 as pywt's ``TYPE sum = 0``:

    i = 2o+1 < n:   out[o] = sum_{j=0..F-1} f[j]*x~[i-j]                       (j ascending)
    i >= n:         e = i-n+1; j = e-1, e-2, ..., 0 (the extension terms, filter index
                    descending), then j = e, ..., F-1
    y[2m+p] = (0 + sum_{j<F/2} r[2j+p]*a[m+F/2-1-j]) + sum_{j<F/2} h[2j+p]*d[m+F/2-1-j]

verified bit-for-bit against pywt 1.1.1 (fixtures ``tests/golden/wavelet_generic_pywt.npz``,
``tests/golden/make_golden_wavelets.py``).
"""
import json
import os

import numpy as np

# sym2 filter bank (pywt 1.1.1 ``Wavelet('sym2')``), as the fp32 casts pywt uses for fp32 data.
DEC_LO = np.array([-0.12940952255092145, 0.22414386804185735,
                   0.836516303737469, 0.48296291314469025], dtype=np.float32)
DEC_HI = np.array([-0.48296291314469025, 0.836516303737469,
                   -0.22414386804185735, -0.12940952255092145], dtype=np.float32)
REC_LO = DEC_LO[::-1].copy()
REC_HI = DEC_HI[::-1].copy()

F = 4

# haar filter bank (pywt 1.1.1 ``Wavelet('haar')``), fp32 casts
H = np.float32(0.7071067811865476)
HAAR_DEC_LO = np.array([H, H], dtype=np.float32)
HAAR_DEC_HI = np.array([-H, H], dtype=np.float32)
HAAR_REC_LO = np.array([H, H], dtype=np.float32)
HAAR_REC_HI = np.array([H, -H], dtype=np.float32)
FILTER_LEN = {"sym2": 4, "haar": 2}
_BANKS = None


def filter_bank(wavelet):
    """(dec_lo, dec_hi, rec_lo, rec_hi) as float32 arrays, from the pywt-generated table."""
    global _BANKS
    if _BANKS is None:
        path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "decentralizepy_amd", "wavelet_filters.json")
        with open(path) as f:
            _BANKS = json.load(f)["wavelets"]
    if wavelet not in _BANKS:
        raise ValueError(f"unknown wavelet {wavelet!r}")
    return tuple(np.array(b, dtype=np.uint32).view(np.float32) for b in _BANKS[wavelet])


def filter_len(wavelet):
    return FILTER_LEN[wavelet] if wavelet in FILTER_LEN else filter_bank(wavelet)[0].shape[0]


def level_lengths(n, level, wavelet="sym2"):
    """[n_0=n, n_1, ..., n_L] with n_l = floor((n_{l-1} + F - 1) / 2)."""
    f = filter_len(wavelet)
    lens = [int(n)]
    for _ in range(level):
        lens.append((lens[-1] + f - 1) // 2)
    return lens


def coeff_len(n, level, wavelet="sym2"):
    """Length M of ``coeffs_to_array(wavedec(x))`` for a length-n input."""
    lens = level_lengths(n, level, wavelet)
    return lens[level] + sum(lens[1:])


def _dwt1_haar(x, flt):
    x = np.asarray(x, dtype=np.float32)
    n = x.shape[0]
    xe = np.concatenate([x, x[-1:]]) if n % 2 else x
    f0, f1 = np.float32(flt[0]), np.float32(flt[1])
    return (f0 * xe[1::2] + f1 * xe[0::2]).astype(np.float32)


def _idwt1_haar(a, d):
    n = d.shape[0]
    if a.shape[0] == n + 1:
        a = a[:n]
    y = np.empty(2 * n, dtype=np.float32)
    y[0::2] = HAAR_REC_LO[0] * a + HAAR_REC_HI[0] * d
    y[1::2] = HAAR_REC_LO[1] * a + HAAR_REC_HI[1] * d
    return y


def _dwt1(x, flt):
    x = np.asarray(x, dtype=np.float32)
    n = x.shape[0]
    if n < F:
        raise ValueError("oracle dwt needs n >= 4 at every level")
    nout = (n + F - 1) // 2
    xe = np.empty(n + 6, dtype=np.float32)       # x~[-3 .. n+2] at offset 3
    xe[3:n + 3] = x
    xe[0:3] = x[2::-1]
    xe[n + 3:n + 6] = x[n - 1:n - 4:-1]
    f0, f1, f2, f3 = (np.float32(v) for v in flt)
    i = 2 * np.arange(nout) + 1 + 3               # offset into xe
    out = ((f0 * xe[i] + f1 * xe[i - 1]) + f2 * xe[i - 2]) + f3 * xe[i - 3]
    if n % 2 == 1:
        out[-1] = ((f2 * xe[n + 3] + f1 * xe[n + 4]) + f0 * xe[n + 5]) + f3 * xe[n + 2]
    return out.astype(np.float32)


def _dwt1_generic(x, flt):
    """pywt ``downsampling_convolution`` (mode symmetric, step 2) with F = len(flt) taps."""
    x = np.asarray(x, dtype=np.float32)
    f = [np.float32(v) for v in flt]
    F, n = len(f), x.shape[0]
    if n < F:
        raise ValueError("oracle generic dwt needs n >= F at every level")
    nout = (n + F - 1) // 2
    xe = np.empty(n + 2 * (F - 1), dtype=np.float32)  # x~[-(F-1) .. n+F-2] at offset F-1
    xe[F - 1:F - 1 + n] = x
    xe[0:F - 1] = x[F - 2::-1]
    xe[F - 1 + n:] = x[n - 1:n - F:-1] if n > F else x[n - 1::-1][:F - 1]
    i = 2 * np.arange(nout) + 1
    main = i < n
    im = i[main] + (F - 1)
    s = np.zeros(im.shape[0], dtype=np.float32)
    for j in range(F):
        s = s + f[j] * xe[im - j]
    out = np.empty(nout, dtype=np.float32)
    out[main] = s
    for o in np.flatnonzero(~main):
        io = int(i[o])
        e = io - n + 1
        acc = np.float32(0.0)
        for j in list(range(e - 1, -1, -1)) + list(range(e, F)):
            acc = np.float32(acc + np.float32(f[j] * xe[io - j + F - 1]))
        out[o] = acc
    return out


def _idwt1_generic(a, d, rec_lo, rec_hi):
    """pywt ``idwt``: ``upsampling_convolution_valid_sf`` of a with rec_lo into a zeroed
    output, then of d with rec_hi added (F/2 taps per phase)."""
    n = d.shape[0]
    if a.shape[0] == n + 1:
        a = a[:n]
    assert a.shape[0] == n
    F2 = len(rec_lo) // 2
    r = [np.float32(v) for v in rec_lo]
    h = [np.float32(v) for v in rec_hi]
    m = np.arange(n - F2 + 1)
    y = np.empty(2 * (n - F2 + 1), dtype=np.float32)
    for p in (0, 1):
        sa = np.zeros(m.shape[0], dtype=np.float32)
        sd = np.zeros(m.shape[0], dtype=np.float32)
        for j in range(F2):
            sa = sa + r[2 * j + p] * a[m + F2 - 1 - j]
            sd = sd + h[2 * j + p] * d[m + F2 - 1 - j]
        y[p::2] = (np.float32(0.0) + sa) + sd
    return y


def wavedec_array(x, level=4, wavelet="sym2"):
    """``coeffs_to_array(wavedec(x, wavelet, level=level))`` as one fp32 vector."""
    a = np.asarray(x, dtype=np.float32)
    details = []
    for _ in range(level):
        if wavelet not in FILTER_LEN:
            dec_lo, dec_hi, _, _ = filter_bank(wavelet)
            d, a = _dwt1_generic(a, dec_hi), _dwt1_generic(a, dec_lo)
        elif wavelet == "haar":
            d, a = _dwt1_haar(a, HAAR_DEC_HI), _dwt1_haar(a, HAAR_DEC_LO)
        else:
            d = _dwt1(a, DEC_HI)
            a = _dwt1(a, DEC_LO)
        details.append(d)
    return np.concatenate([a] + details[::-1]).astype(np.float32)


def _idwt1(a, d):
    n = d.shape[0]
    if a.shape[0] == n + 1:
        a = a[:n]
    assert a.shape[0] == n
    r0, r1, r2, r3 = (np.float32(v) for v in REC_LO)
    h0, h1, h2, h3 = (np.float32(v) for v in REC_HI)
    y = np.empty(2 * n - 2, dtype=np.float32)
    a1, a0, d1, d0 = a[1:], a[:-1], d[1:], d[:-1]
    y[0::2] = (r0 * a1 + r2 * a0) + (h0 * d1 + h2 * d0)
    y[1::2] = (r1 * a1 + r3 * a0) + (h1 * d1 + h3 * d0)
    return y


def waverec_array(coeffs, n, level=4, wavelet="sym2"):
    """``waverec(array_to_coeffs(coeffs))`` truncated to the original length n."""
    lens = level_lengths(n, level, wavelet)
    c = np.asarray(coeffs, dtype=np.float32)
    pos = lens[level]
    a = c[:pos]
    for lvl in range(level, 0, -1):
        d = c[pos:pos + lens[lvl]]
        pos += lens[lvl]
        if wavelet not in FILTER_LEN:
            _, _, rec_lo, rec_hi = filter_bank(wavelet)
            a = _idwt1_generic(a, d, rec_lo, rec_hi)
        else:
            a = _idwt1_haar(a, d) if wavelet == "haar" else _idwt1(a, d)
    return a[:n].copy()
