"""GPU: the FFT plugin (decentralizepy_amd/sharing/JWINS/FFT.py: the native real FFTs + the HIP
complex-key / gather / pair-index kernels + the shared top-k and fold kernels) replays the
reference FFT plugin's recorded rounds: exact indices and counters, complex values, accumulators
and averaged models within scenario.fft_tol (an fp32 FFT vs torch's CPU pocketfft)."""
from collections import deque

import numpy as np
import pytest
import torch

from tests import scenario

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", scenario.fft_names())
def test_fft_plugin_replays_reference(name, dev, tmp_path):
    scenario.replay_fft_plugin(name, tmp_path)


def test_fft_full_payload_raises_keyerror_like_reference(dev, tmp_path):
    """reference FFT.deserialized_model reads m["indices"] for a full payload as well."""
    from decentralizepy_amd.sharing.JWINS.FFT import FFT
    meta, arrays = scenario.load_fft("fft_plain")
    model = scenario.make_model(meta["shape"])
    scenario.set_flat(model, arrays["x0"])
    plugin = FFT(0, 0, None, scenario._Mapping(), scenario._Graph([1]), model, None,
                 str(tmp_path), **meta["kwargs"])
    plugin.get_data_to_send(degree=1)
    full = {"params": np.zeros(meta["m"], np.complex64), "degree": 1, "iteration": 0,
            "CHANNEL": "DPSGD"}
    with pytest.raises(KeyError):
        plugin._averaging({1: deque([full])})
    with pytest.raises(KeyError):
        plugin.deserialized_model({"params": np.zeros(meta["m"], np.complex64)})


@pytest.mark.parametrize("cls,ok", [("Elias", True), ("EliasFpzip", False),
                                    ("Lz4Wrapper", False), ("EliasFp16", False)])
def test_fft_complex_values_only_through_pass_through_float_leg(dev, tmp_path, cls, ok):
    """Complex64 values may not go through an fp32 float codec (it would drop the imaginary
    part): Elias (indices only) works, the float codecs raise."""
    from decentralizepy_amd.sharing.JWINS.FFT import FFT
    meta, arrays = scenario.load_fft("fft_plain")
    model = scenario.make_model(meta["shape"])
    scenario.set_flat(model, arrays["x0"])
    kw = dict(meta["kwargs"], compress=True, compression_class=cls,
              compression_package=f"decentralizepy_amd.compression.{cls}")
    plugin = FFT(0, 0, None, scenario._Mapping(), scenario._Graph([1]), model, None,
                 str(tmp_path), **kw)
    scenario.set_flat(model, arrays["r0_x"])
    if ok:
        data = plugin.get_data_to_send(degree=1)
        assert np.iscomplexobj(data["params"])
    else:
        with pytest.raises(NotImplementedError):
            plugin.get_data_to_send(degree=1)


# native kernel sizes: even n (M = n / 2 complex) and odd n (a complex DFT of n), radices 2..13,
# other primes (one output per thread), a prime pass of its own (683, the reference fixture's M),
# n = 2 (no pass), and two fallbacks to hipFFT (a prime factor above 4096)
FFT_SIZES = [(4098, True), (1 << 20, True), (11_000_000, True), (25_000_000, True),
             (2, True), (3, True), (30030, True), (4097, True), (2 * 17 * 19 * 23, True),
             (16_777_216, True), (100_003, False), (2 * 9839, False)]


@pytest.mark.parametrize("n,native", FFT_SIZES)
def test_rfft_irfft_against_numpy(dev, n, native):
    """dpz_rfft / dpz_irfft against a float64 numpy FFT (error bound as scenario.fft_tol) and the
    round trip; sizes include a power of two and the C2 model size (2^6 5^6 11).  dpz_fft_native
    says which sizes the hand-written kernels take (the rest: hipFFT)."""
    from decentralizepy_amd import _lib, codec
    assert _lib.lib().dpz_fft_native(n) == int(native)
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(n, device=dev, generator=g)
    f = codec.rfft(x)
    xh = x.cpu().numpy()
    ref = np.fft.rfft(xh.astype(np.float64))
    scale = float(np.abs(xh).max())
    err = np.abs(f.cpu().numpy() - ref).max()
    assert err <= scenario.fft_tol("params", n, scale), err
    # the inverse ignores Im X[0] (and Im X[n/2] for even n), as torch / pocketfft's c2r does
    fin = f.clone()
    fin[0] += 0.25j
    if n % 2 == 0:
        fin[-1] -= 0.5j
    back = codec.irfft(fin, n)
    err2 = np.abs(back.cpu().numpy() - xh).max()
    assert err2 <= scenario.fft_tol("model", n, scale), err2
    # an arbitrary spectrum (not the transform of a real vector) against numpy's c2r
    spec = (torch.randn(n // 2 + 1, device=dev, generator=g)
            + 1j * torch.randn(n // 2 + 1, device=dev, generator=g)).to(torch.complex64)
    sh = spec.cpu().numpy().astype(np.complex128)
    got = codec.irfft(spec.clone(), n).cpu().numpy()
    want = np.fft.irfft(sh, n)
    err3 = np.abs(got - want).max()
    assert err3 <= scenario.fft_tol("model", n, float(np.abs(want).max())), err3


def test_cplx_kernels_exact(dev):
    """dpz_cplx_key (all accumulation modes), dpz_cplx_gather with the rewind and
    dpz_cplx_pair_indices against fp32 numpy restatements (bit-exact)."""
    from decentralizepy_amd import codec
    from oracle import fft as offt
    rng = np.random.default_rng(3)
    m = 100_003
    c = (rng.standard_normal(m) + 1j * rng.standard_normal(m)).astype(np.complex64)
    a = (0.1 * (rng.standard_normal(m) + 1j * rng.standard_normal(m))).astype(np.complex64)
    cd = torch.from_numpy(c).to(dev)
    for mode in (codec.DPZ_ACC_NONE, codec.DPZ_ACC_ACCUMULATE, codec.DPZ_ACC_ADD):
        ad = torch.from_numpy(a.copy()).to(dev)
        key = codec.cplx_key(cd, ad if mode else None, mode).cpu().numpy()
        if mode == codec.DPZ_ACC_ACCUMULATE:
            acc_ref = (a.view(np.float32) + c.view(np.float32)).view(np.complex64)
            np.testing.assert_array_equal(ad.cpu().numpy().view(np.uint32), acc_ref.view(np.uint32))
            src = acc_ref
        elif mode == codec.DPZ_ACC_ADD:
            src = (c.view(np.float32) + a.view(np.float32)).view(np.complex64)
        else:
            src = c
        np.testing.assert_array_equal(key.view(np.uint32), offt.cabs(src).view(np.uint32))
    idx = np.sort(rng.choice(m, 5000, replace=False)).astype(np.int32)
    idd = torch.from_numpy(idx).to(dev)
    ad = torch.from_numpy(a.copy()).to(dev)
    out = codec.cplx_gather(cd, idd, acc=ad).cpu().numpy()
    np.testing.assert_array_equal(out.view(np.uint64), c[idx].view(np.uint64))
    a2 = a.copy()
    a2[idx] = 0
    np.testing.assert_array_equal(ad.cpu().numpy().view(np.uint64), a2.view(np.uint64))
    pair = codec.cplx_pair_indices(idd).cpu().numpy()
    np.testing.assert_array_equal(pair, offt.pair_indices(idx).astype(np.int32))


@pytest.mark.parametrize("n", [4098, 30030, 11_000_000, 2 * 17 * 19 * 23])
def test_fft_inplace_passes_forced(dev, diag_lib, monkeypatch, n):
    """The in-place pass variant (one LDS buffer, sub-passes staged in registers; passes whose
    radices are all in {2, 3, 4, 5, 7, 8}) forced on through the diagnostic build
    (DPZ_FFT_INPLACE=1): the same tolerances against numpy as the default passes, and bit-equal
    to them where both run the same arithmetic (the butterflies and twiddles are the same)."""
    from decentralizepy_amd import codec
    g = torch.Generator(device=dev).manual_seed(11)
    x = torch.randn(n, device=dev, generator=g)
    monkeypatch.setenv("DPZ_FFT_INPLACE", "0")
    f0 = codec.rfft(x).cpu().numpy()
    monkeypatch.setenv("DPZ_FFT_INPLACE", "1")
    f1 = codec.rfft(x)
    xh = x.cpu().numpy()
    scale = float(np.abs(xh).max())
    ref = np.fft.rfft(xh.astype(np.float64))
    assert np.abs(f1.cpu().numpy() - ref).max() <= scenario.fft_tol("params", n, scale)
    np.testing.assert_array_equal(f1.cpu().numpy().view(np.uint64), f0.view(np.uint64))
    back = codec.irfft(f1.clone(), n).cpu().numpy()
    assert np.abs(back - xh).max() <= scenario.fft_tol("model", n, scale)


@pytest.mark.parametrize("n", [2, 4098, 30030, 11_000_000, 2 * 17 * 19 * 23, 1 << 20])
def test_fft_pairing_fused_matches_separate_pass(dev, diag_lib, monkeypatch, n):
    """The even-n rfft pairing X[k] / X[M - k] done in the last pass's stores (the block holding
    columns j and S - j) against the separate pairing pass (DPZ_FFT_POST_FUSED=0, diagnostic
    build): bit-identical (the same arithmetic), and within tolerance of numpy."""
    from decentralizepy_amd import codec
    g = torch.Generator(device=dev).manual_seed(13)
    x = torch.randn(n, device=dev, generator=g)
    monkeypatch.setenv("DPZ_FFT_POST_FUSED", "0")
    f0 = codec.rfft(x).cpu().numpy()
    monkeypatch.setenv("DPZ_FFT_POST_FUSED", "1")
    f1 = codec.rfft(x).cpu().numpy()
    np.testing.assert_array_equal(f1.view(np.uint64), f0.view(np.uint64))
    xh = x.cpu().numpy()
    ref = np.fft.rfft(xh.astype(np.float64))
    assert np.abs(f1 - ref).max() <= scenario.fft_tol("params", n, float(np.abs(xh).max()))
