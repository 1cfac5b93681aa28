"""CPU: the generic-filter wavelet path's oracle and host side — the oracle restatement of
pywt's downsampling / upsampling convolutions against PyWavelets 1.1.1's own outputs
(tests/golden/wavelet_generic_pywt.npz, make_golden_wavelets.py), the filter table, and the
library's level-length / workspace entry points (host code, no GPU)."""
import json
import os

import numpy as np
import pytest

from oracle import wavelet as owav

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cases():
    z = np.load(os.path.join(GOLDEN, "wavelet_generic_pywt.npz"))
    return z, [k[:-2] for k in z.files if k.endswith("/x")]


def test_oracle_generic_matches_pywt():
    z, cases = _cases()
    assert len(cases) >= 20
    for key in cases:
        name, n, level = key.split("/")
        n, level = int(n), int(level)
        c = owav.wavedec_array(z[key + "/x"], level, name)
        np.testing.assert_array_equal(c.view(np.uint32), z[key + "/coeffs"].view(np.uint32),
                                      err_msg=key)
        r = owav.waverec_array(z[key + "/c"], n, level, name)
        np.testing.assert_array_equal(r.view(np.uint32), z[key + "/rec"][:n].view(np.uint32),
                                      err_msg=key)


@pytest.mark.parametrize("name", ["sym2", "haar"])
def test_generic_restatement_equals_the_fused_forms(name):
    """sym2 / haar through the generic F-tap loops agree with their specialised restatements
    (and so with pywt) — the generic order contains pywt's sym2 odd-tail exception."""
    z, _ = _cases()
    key = f"{name}/1001/4"
    dec_lo, dec_hi, rec_lo, rec_hi = owav.filter_bank(name)
    a = z[key + "/x"]
    det = []
    for _ in range(4):
        det.append(owav._dwt1_generic(a, dec_hi))
        a = owav._dwt1_generic(a, dec_lo)
    c = np.concatenate([a] + det[::-1])
    np.testing.assert_array_equal(c.view(np.uint32), z[key + "/coeffs"].view(np.uint32))


def test_filter_table():
    with open(os.path.join(ROOT, "decentralizepy_amd", "wavelet_filters.json")) as f:
        d = json.load(f)
    w = d["wavelets"]
    assert d["pywavelets"] == "1.1.1" and len(w) == 93
    for name, banks in w.items():
        assert len(banks) == 4 and len({len(b) for b in banks}) == 1, name
        assert len(banks[0]) % 2 == 0 and len(banks[0]) <= 64, name
    # the coiflet float banks are pywt's float-arithmetic products, not casts (1 ulp apart)
    assert d["float_bank_differs_from_cast"] == [f"coif{i}" for i in range(1, 11)]


def test_library_generic_lengths_and_workspace():
    from decentralizepy_amd import _lib
    L = _lib.lib()
    for name, n, level in [("db4", 4099, 4), ("dmey", 20011, 2), ("coif3", 6000, 3),
                           ("sym2", 4099, 6)]:
        f = owav.filter_len(name)
        assert L.dpz_wavedec_len_generic(n, level, f) == owav.coeff_len(n, level, name)
        lens = owav.level_lengths(n, level, name)
        assert L.dpz_wavelet_generic_workspace_bytes(n, level, f) == 16 * lens[1]
    assert L.dpz_wavedec_len_generic(60, 1, 64) == -1      # a 60-value input, 64 taps
    assert L.dpz_wavedec_len_generic(64, 2, 64) == -1      # level 2 input: 63 values
    assert L.dpz_wavedec_len_generic(1000, 2, 5) == -1     # odd filter length
    assert L.dpz_wavedec_len_generic(1000, 9, 4) == -1     # level past 8
    assert L.dpz_wavelet_generic_workspace_bytes(1000, 1, 8) == 0
    from decentralizepy_amd import codec
    with pytest.raises(NotImplementedError):  # the Wavelet plugin's documented error
        codec.wavedec_len(62, 2, "dmey")
