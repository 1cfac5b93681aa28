"""GPU tests of the block-floating float codec (csrc/dpz_fpz.hip) through the C-ABI: the device
stream is byte-identical to the oracle's (oracle/fpz.py), decodes back to the top-p truncation
(every bit pattern at precision 0), rejects malformed streams without writing, and the
EliasFpzip / EliasFpzipLossy compressors carry it (reference compression/EliasFpzip.py:19-51,
EliasFpzipLossy.py:14-58; parity with fpzip's bytes unpinned)."""
import numpy as np
import pytest
import torch

from oracle import fpz as ofpz
from tests.test_oracle_fpz import SPECIALS

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [1, 63, 256, 257, 4099, 110_000, 1_000_003])
@pytest.mark.parametrize("precision", [0, 16, 10, 8])
def test_device_stream_matches_oracle(dev, n, precision):
    from decentralizepy_amd import codec
    x = (0.02 * np.random.default_rng(n).standard_normal(n)).astype(np.float32)
    x[:: max(1, n // 7)] = 0.0  # wide exponent ranges in some blocks
    enc = codec.fpz_encode(torch.from_numpy(x).to(dev), precision)
    ref = ofpz.encode(x, precision)
    np.testing.assert_array_equal(enc.cpu().numpy(), ref)
    n_, prec = int(ref[4:8].view("<u4")[0]), int(ref[8:12].view("<u4")[0])
    back = codec.fpz_decode(enc.clone(), n_, prec)
    np.testing.assert_array_equal(back.cpu().numpy().view(np.uint32),
                                  ofpz.truncate(x, precision).view(np.uint32))


def test_every_bit_pattern_round_trips(dev):
    from decentralizepy_amd import codec
    u = np.random.default_rng(5).integers(0, 2**32, size=300_000, dtype=np.uint64).astype(np.uint32)
    x = np.concatenate([u.view(np.float32), SPECIALS])
    enc = codec.fpz_encode(torch.from_numpy(x).to(dev), 0)
    np.testing.assert_array_equal(enc.cpu().numpy(), ofpz.encode(x, 0))
    back = codec.fpz_decode(enc, x.size, 32)
    np.testing.assert_array_equal(back.cpu().numpy().view(np.uint32), x.view(np.uint32))
    y = codec.fpz_decode(codec.fpz_encode(torch.from_numpy(SPECIALS).to(dev), 12), SPECIALS.size, 12)
    assert np.array_equal(np.isnan(y.cpu().numpy()), np.isnan(SPECIALS))


def test_empty_and_unaligned_input(dev):
    from decentralizepy_amd import codec
    enc = codec.fpz_encode(torch.empty(0, device=dev), 0)
    np.testing.assert_array_equal(enc.cpu().numpy(), ofpz.encode(np.zeros(0, np.float32), 0))
    base = torch.from_numpy(np.arange(1001, dtype=np.float32)).to(dev)
    x = base[1:]  # 4-byte aligned, not 16: the scalar load path
    enc = codec.fpz_encode(x, 0)
    np.testing.assert_array_equal(enc.cpu().numpy(), ofpz.encode(x.cpu().numpy(), 0))


def test_malformed_stream_is_rejected(dev):
    from decentralizepy_amd import codec
    x = np.random.default_rng(7).standard_normal(5000).astype(np.float32)
    good = ofpz.encode(x, 0)
    nblk = (x.size + 255) // 256
    cases = []
    b = good.copy().view("<u4")
    b[4 + 3] = b[4 + 4] + 5  # a table entry out of order
    cases.append(b.view(np.uint8))
    b = good.copy().view("<u4")
    b[4 + nblk] = 0xFFFFFF  # block area longer than the buffer
    cases.append(b.view(np.uint8))
    b = good.copy().view("<u4")
    b[4 + nblk + 1] |= 0x0F00  # exponent width 15
    cases.append(b.view(np.uint8))
    b = good.copy().view("<u4")
    b[1] += 1  # header n disagrees with the caller's n
    cases.append(b.view(np.uint8))
    for bad in cases:
        out = torch.full((x.size,), 7.0, device=dev)
        with pytest.raises(ValueError):
            codec.fpz_decode(torch.from_numpy(bad.copy()).to(dev), x.size, 32, out=out)
    with pytest.raises(ValueError):  # shorter than header + table + one word a block
        codec.fpz_decode(torch.from_numpy(good[:64].copy()).to(dev), x.size, 32)


@pytest.mark.parametrize("cls_name,precision", [("EliasFpzip", 0), ("EliasFpzipLossy", 16),
                                                ("EliasFpzipLossy", 8)])
def test_compressors(dev, cls_name, precision):
    import importlib
    mod = importlib.import_module(f"decentralizepy_amd.compression.{cls_name}")
    c = getattr(mod, cls_name)(float_precision=precision if cls_name != "EliasFpzip" else None)
    x = (0.05 * np.random.default_rng(11).standard_normal(25_001)).astype(np.float32)
    enc = c.compress_float(x)
    assert enc.dtype == np.uint8
    np.testing.assert_array_equal(enc, ofpz.encode(x, precision))
    np.testing.assert_array_equal(c.decompress_float(enc).view(np.uint32),
                                  ofpz.truncate(x, precision).view(np.uint32))
    d = c.decompress_float_device(enc)
    assert d.is_cuda and d.dtype == torch.float32
    assert enc.size < (0.92 if precision == 0 else 0.5) * 4 * x.size
