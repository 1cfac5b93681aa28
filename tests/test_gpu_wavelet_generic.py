"""GPU parity of the generic-filter wavelet kernels (dpz_dwt_generic / dpz_idwt_generic) — every
pywt discrete wavelet other than the fused sym2 / haar: against PyWavelets 1.1.1's own outputs
(tests/golden/wavelet_generic_pywt.npz) and, for the forms the plugins use (the W(x), W(x - x0)
pair, the accumulating post-step with and without the sliced encode's rewind mask), against the
oracle (oracle/wavelet.py, pinned to the same fixtures).  Bit-exact throughout.  The reference's
Wavelet plugin with these wavelets is replayed by test_gpu_plugins.py (wg_* scenarios)."""
import os

import numpy as np
import pytest
import torch

from oracle import wavelet as owav

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _bits(a):
    return np.asarray(a, dtype=np.float32).view(np.uint32)


def test_generic_matches_pywt(dev):
    from decentralizepy_amd import codec
    z = np.load(os.path.join(GOLDEN, "wavelet_generic_pywt.npz"))
    keys = [k[:-2] for k in z.files if k.endswith("/x")]
    for key in keys:
        name, n, level = key.split("/")
        n, level = int(n), int(level)
        if codec._fused(name, level):
            continue  # sym2 / haar: the fused kernels (their own pywt tests)
        x = torch.from_numpy(z[key + "/x"]).to(dev)
        cx, _ = codec.wavedec(x, level, wavelet=name)
        np.testing.assert_array_equal(_bits(cx.cpu().numpy()), _bits(z[key + "/coeffs"]),
                                      err_msg=key)
        c = torch.from_numpy(z[key + "/c"]).to(dev)
        r = codec.waverec(c, n, level, wavelet=name)
        np.testing.assert_array_equal(_bits(r.cpu().numpy()), _bits(z[key + "/rec"][:n]),
                                      err_msg=key)


def _mask_of(idx, m):
    words = np.zeros((m + 31) // 32, dtype=np.uint32)
    np.bitwise_or.at(words, idx >> 5, (np.uint32(1) << (idx & 31).astype(np.uint32)))
    return words


@pytest.mark.parametrize("name,n,level", [("db4", 100_003, 4), ("coif3", 65_536, 3),
                                          ("dmey", 50_001, 2), ("sym2", 100_003, 6),
                                          ("bior3.5", 77_777, 4), ("db32", 40_000, 2),
                                          ("haar", 70_001, 9)])
def test_generic_pair_and_accumulate_match_oracle(dev, name, n, level):
    from decentralizepy_amd import codec
    if name == "haar":  # past the fused haar kernel's 8 levels: the table has no level 9 path
        with pytest.raises(Exception):
            codec.wavedec_len(n, level, name)
        return
    rng = np.random.default_rng(n + level)
    x = rng.standard_normal(n).astype(np.float32)
    x0 = (x - 0.01 * rng.standard_normal(n)).astype(np.float32)
    m = codec.wavedec_len(n, level, name)
    assert m == owav.coeff_len(n, level, name)
    tx, tx0 = torch.from_numpy(x).to(dev), torch.from_numpy(x0).to(dev)
    cx, cd = codec.wavedec(tx, level, x0=tx0, wavelet=name)
    want_x = owav.wavedec_array(x, level, name)
    want_d = owav.wavedec_array((x - x0).astype(np.float32), level, name)
    np.testing.assert_array_equal(_bits(cx.cpu().numpy()), _bits(want_x))
    np.testing.assert_array_equal(_bits(cd.cpu().numpy()), _bits(want_d))
    # accumulate: acc += W(x - x0); with the rewind mask: acc = (sel ? +0 : acc) + W(x - x0)
    acc = (0.01 * rng.standard_normal(m)).astype(np.float32)
    sel = np.sort(rng.choice(m, size=m // 10, replace=False)).astype(np.int64)
    acc[sel[:5]] = -0.0
    a1 = torch.from_numpy(acc).to(dev)
    codec.wavedec(tx, level, x0=tx0, want_x=False, coeffs_diff=a1, accumulate=True, wavelet=name)
    np.testing.assert_array_equal(_bits(a1.cpu().numpy()), _bits((acc + want_d).astype(np.float32)))
    a2 = torch.from_numpy(acc).to(dev)
    mask = torch.from_numpy(_mask_of(sel, m).view(np.int32)).to(dev)
    codec.wavedec(tx, level, x0=tx0, want_x=False, coeffs_diff=a2, accumulate=True, wavelet=name,
                  rewind_mask=mask)
    want = acc.copy()
    want[sel] = 0.0
    np.testing.assert_array_equal(_bits(a2.cpu().numpy()), _bits((want + want_d).astype(np.float32)))
    # inverse of the pair's W(x): the oracle's waverec of the same coefficients
    r = codec.waverec(cx, n, level, wavelet=name)
    np.testing.assert_array_equal(_bits(r.cpu().numpy()),
                                  _bits(owav.waverec_array(want_x, n, level, name)))


def test_generic_rejects_short_levels(dev, tmp_path):
    """A level whose input is shorter than the filter raises NotImplementedError, from the codec
    and from the Wavelet plugin's constructor (its documented error)."""
    from decentralizepy_amd import codec
    from decentralizepy_amd.sharing.JWINS.Wavelet import Wavelet
    from tests import scenario
    with pytest.raises(NotImplementedError):
        codec.wavedec_len(62, 2, "dmey")  # level-2 input of 61 values < 62 taps
    model = scenario.make_model([4, 4, 2])  # 30 parameters: dmey's 62 taps at level 1 already
    with pytest.raises(NotImplementedError):
        Wavelet(0, 0, None, scenario._Mapping(), scenario._Graph([1]), model, None,
                str(tmp_path), wavelet="dmey", level=2)
    with pytest.raises(NotImplementedError):
        codec.wavedec_len(100_000, 2, "db40")
