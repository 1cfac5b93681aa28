"""CPU checks of the block-floating float-coding oracle (oracle/fpz.py) — the format statement
the device codec (csrc/dpz_fpz.hip) is compared with byte for byte in tests/test_gpu_fpz.py.
Parity with fpzip's own bytes is unpinned (fpzip is absent); the contract pinned is fpzip's:
precision 0 is lossless for every fp32 bit pattern, precision p keeps the top p bits."""
import numpy as np
import pytest

from oracle import fpz

SPECIALS = np.concatenate([
    np.array([np.nan, np.inf, -np.inf, 0.0, -0.0, 1e-45, -1e-45, 3.4e38, -1e-40, 1.0],
             dtype=np.float32),
    np.array([0x7F800001, 0xFF800003, 0x7FC00000, 0x7FFFFFFF, 0x00000001, 0x807FFFFF],
             dtype=np.uint32).view(np.float32)])


@pytest.mark.parametrize("n", [0, 1, 31, 255, 256, 257, 1000, 20_011])
@pytest.mark.parametrize("precision", [0, 32, 16, 10, 9, 8, 1, 31])
def test_round_trip_is_top_bit_truncation(n, precision):
    x = (0.05 * np.random.default_rng(n).standard_normal(n)).astype(np.float32)
    y = fpz.decode(fpz.encode(x, precision))
    np.testing.assert_array_equal(y.view(np.uint32), fpz.truncate(x, precision).view(np.uint32))
    if precision in (0, 32):
        np.testing.assert_array_equal(y.view(np.uint32), x.view(np.uint32))


def test_all_bit_patterns_lossless():
    u = np.random.default_rng(1).integers(0, 2**32, size=50_000, dtype=np.uint64).astype(np.uint32)
    x = np.concatenate([u.view(np.float32), SPECIALS])
    y = fpz.decode(fpz.encode(x, 0))
    np.testing.assert_array_equal(y.view(np.uint32), x.view(np.uint32))


@pytest.mark.parametrize("precision", [10, 12, 16, 24])
def test_lossy_keeps_nan_and_bounds_error(precision):
    y = fpz.decode(fpz.encode(SPECIALS, precision))
    assert np.array_equal(np.isnan(y), np.isnan(SPECIALS))
    x = np.random.default_rng(2).standard_normal(10_000).astype(np.float32)
    z = fpz.decode(fpz.encode(x, precision))
    rel = np.abs(z - x) / np.abs(x)
    assert rel.max() < 2.0 ** -(precision - 9)
    assert np.all(np.abs(z) <= np.abs(x))  # truncation toward zero


def test_sizes():
    x = (0.01 * np.random.default_rng(3).standard_normal(100_000)).astype(np.float32)
    raw = 4 * x.size
    assert len(fpz.encode(x, 0)) < 0.92 * raw
    assert len(fpz.encode(x, 16)) < 0.42 * raw
    b = fpz.encode(x, 0)
    assert len(b) % 4 == 0
    assert fpz.parse_header(b) == (x.size, 32, (x.size + 255) // 256)


def test_bad_streams_raise():
    b = fpz.encode(np.ones(300, np.float32), 0)
    with pytest.raises(ValueError):
        fpz.parse_header(b[:12])
    bad = b.copy()
    bad[0] ^= 1
    with pytest.raises(ValueError):
        fpz.decode(bad)
