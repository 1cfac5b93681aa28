"""CPU: the LZ4 frame oracle (oracle/lz4.py) against liblz4 1.9.3 with python-lz4's default
preferences (the reference Lz4Wrapper's lz4.frame), and the C-ABI frame walk / header checksum
(dpz_lz4_frame_info, host code) on liblz4-produced frames."""
import numpy as np
import pytest

from oracle import lz4 as olz4

pytestmark = pytest.mark.skipif(not olz4.available(), reason="liblz4 not in this image")


def _cases():
    rng = np.random.default_rng(7)
    idx = np.sort(rng.choice(11_000_000, 110_000, replace=False)).astype(np.int32)
    return {
        "empty": b"",
        "tiny": b"abc",
        "zeros_1M": bytes(1 << 20),
        "random_300k": rng.integers(0, 256, 300_000, dtype=np.uint8).tobytes(),
        "idx_gaps_c2": np.diff(idx, prepend=0).astype(np.int32).tobytes(),
        "fp32_values": (0.01 * rng.standard_normal(50_000)).astype(np.float32).tobytes(),
        "text_repeat": b"decentralizepy " * 9000,
    }


@pytest.mark.parametrize("name", list(_cases()))
def test_oracle_decoder_reads_liblz4_frames(name):
    data = _cases()[name]
    for linked in (True, False):
        frame = olz4.ref_compress(data, block_linked=linked)
        assert olz4.ref_decompress(frame) == data
        assert olz4.decode_frame(frame) == data


def test_wrapper_index_leg_round_trip():
    rng = np.random.default_rng(3)
    a = rng.choice(1_000_000, 10_000, replace=False).astype(np.int32)
    a_sorted = np.sort(a)
    frame = olz4.wrapper_compress(a)
    np.testing.assert_array_equal(a, a_sorted)  # sorted in place, as the reference does
    out = olz4.wrapper_decompress(frame)
    assert out.dtype == np.int64
    np.testing.assert_array_equal(out, a_sorted)
    assert len(frame) < a.nbytes  # the gaps compress


@pytest.mark.parametrize("name", ["zeros_1M", "idx_gaps_c2", "text_repeat", "empty"])
def test_c_abi_frame_walk_of_liblz4_frames(name):
    from decentralizepy_amd import codec
    data = _cases()[name]
    frame = olz4.ref_compress(data)
    cs, nb, linked, bmax = codec.lz4_frame_info(frame)
    # liblz4 leaves an empty content size unset and writes one-block frames as independent
    assert cs == (len(data) if data else -1) and bmax == 65536
    assert linked == (len(data) > 65536)
    assert nb == (len(data) + 65535) // 65536
    ind = olz4.ref_compress(data, block_linked=False)
    assert codec.lz4_frame_info(ind)[2] is False
    bad = bytearray(frame)
    bad[6 + (8 if data else 0)] ^= 0xFF  # header checksum byte
    with pytest.raises(ValueError):
        codec.lz4_frame_info(bytes(bad))
    with pytest.raises(ValueError):
        codec.lz4_frame_info(frame[:-3])
