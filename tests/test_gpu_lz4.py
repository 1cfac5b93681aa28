"""GPU: the device LZ4 frame codec (csrc/dpz_lz4.hip) and the Lz4Wrapper drop-in
(reference compression/Lz4Wrapper.py:20-98) — device frames decoded by liblz4 1.9.3 (what
python-lz4 wraps) and by the oracle's frame restatement, liblz4 frames (linked and independent)
decoded on the device, malformed frames rejected, and the PartialModel scenarios replayed with
Lz4Wrapper on the wire."""
import numpy as np
import pytest
import torch

from oracle import lz4 as olz4
from tests import scenario
from tests.test_oracle_lz4 import _cases

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not olz4.available(), reason="liblz4 not in this image")]


def _dev_bytes(b, dev):
    return torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev) if b else \
        torch.empty(0, dtype=torch.uint8, device=dev)


@pytest.mark.parametrize("par", ["1", "0"])
@pytest.mark.parametrize("name", list(_cases()))
def test_device_frames_decode_with_liblz4(dev, name, par, monkeypatch, diag_lib):
    """par 1: independent blocks that decode to <= 4 KB take the parallel decoder (parse, then
    pointer jumping); par 0: the sequential decoder for every block (DPZ_LZ4_PAR=0)."""
    monkeypatch.setenv("DPZ_LZ4_PAR", par)
    from decentralizepy_amd import codec
    data = _cases()[name]
    frame = bytes(codec.lz4_compress(_dev_bytes(data, dev)).cpu().numpy().tobytes())
    assert olz4.ref_decompress(frame) == data
    assert olz4.decode_frame(frame) == data
    back = codec.lz4_decompress(frame, dev)
    assert bytes(back.cpu().numpy().tobytes()) == data
    if name in ("zeros_1M", "idx_gaps_c2", "text_repeat"):
        assert len(frame) < 0.9 * len(data), (len(frame), len(data))
    from decentralizepy_amd import _lib
    assert len(frame) <= int(_lib.lib().dpz_lz4_max_bytes(len(data)))  # raw blocks at worst


@pytest.mark.parametrize("name", list(_cases()))
@pytest.mark.parametrize("linked", [True, False])
def test_device_decodes_liblz4_frames(dev, name, linked):
    """liblz4's frames: linked 64 KB blocks (sequential decoder), independent blocks (the
    parallel decoder for those that decode to <= 4 KB, the rest handed to the sequential one)."""
    from decentralizepy_amd import codec
    data = _cases()[name]
    frame = olz4.ref_compress(data, block_linked=linked)
    assert bytes(codec.lz4_decompress(frame, dev).cpu().numpy().tobytes()) == data


def test_malformed_frames_are_rejected(dev):
    from decentralizepy_amd import codec
    data = _cases()["idx_gaps_c2"]
    frame = bytearray(olz4.ref_compress(data))
    # a block whose first match offset points before the start of the output
    body = 6 + 8 + 1 + 4
    bad = bytearray(frame)
    tok = bad[body]
    i = body + 1
    L = tok >> 4
    if L == 15:
        while bad[i] == 255:
            L += 255
            i += 1
        L += bad[i]
        i += 1
    i += L
    bad[i], bad[i + 1] = 0xFF, 0xFF
    with pytest.raises(ValueError):
        codec.lz4_decompress(bytes(bad), dev)
    with pytest.raises(ValueError):
        codec.lz4_decompress(bytes(frame[:-10]), dev)
    # this codec's independent frame (the parallel decoder): the same corruption of the first
    # match offset, and a literal run reaching past its block
    own = bytearray(codec.lz4_compress(_dev_bytes(data, dev)).cpu().numpy().tobytes())
    bad = bytearray(own)
    tok = bad[body]
    i = body + 1
    L = tok >> 4
    if L == 15:
        while bad[i] == 255:
            L += 255
            i += 1
        L += bad[i]
        i += 1
    i += L
    bad[i], bad[i + 1] = 0xFF, 0xFF
    with pytest.raises(ValueError):
        codec.lz4_decompress(bytes(bad), dev)
    bad = bytearray(own)
    bad[body] = 0xF0  # literal length 15 + extension bytes read from the block's data
    bad[body + 1] = 0xFF
    with pytest.raises(ValueError):
        codec.lz4_decompress(bytes(bad), dev)


def test_untrusted_content_size_is_bounded_before_allocation(dev):
    """A peer frame whose header claims 2^40 content bytes (header checksum recomputed, so the
    header itself is well-formed) is rejected from the block bound, before any allocation."""
    import struct

    import xxhash

    from decentralizepy_amd import codec
    frame = bytearray(olz4.ref_compress(_cases()["idx_gaps_c2"]))
    assert frame[4] & 0x08  # content size present (python-lz4's default store_size=True)
    frame[6:14] = struct.pack("<Q", 1 << 40)
    frame[14] = (xxhash.xxh32(bytes(frame[4:14])).intdigest() >> 8) & 0xFF
    cs, nb, _, bmax = codec.lz4_frame_info(bytes(frame))
    assert cs == 1 << 40 and cs > nb * bmax
    with pytest.raises(ValueError):
        codec.lz4_decompress(bytes(frame), dev)
    good = olz4.ref_compress(_cases()["idx_gaps_c2"])
    with pytest.raises(ValueError):  # a caller's max_size below the stored size
        codec.lz4_decompress(good, dev, max_size=16)


def test_lz4wrapper_index_and_value_legs(dev):
    from decentralizepy_amd.compression.Lz4Wrapper import Lz4Wrapper
    rng = np.random.default_rng(11)
    a = rng.choice(11_000_000, 110_000, replace=False).astype(np.int32)
    ref = np.sort(a)
    c = Lz4Wrapper(float_precision=None)
    frame = c.compress(a)
    np.testing.assert_array_equal(a, ref)  # sorted in place
    np.testing.assert_array_equal(olz4.wrapper_decompress(frame), ref)
    out = c.decompress(frame)
    assert out.dtype == np.int64
    np.testing.assert_array_equal(out, ref)
    # a reference node's frame (liblz4, linked 64 KB blocks)
    np.testing.assert_array_equal(c.decompress(olz4.wrapper_compress(ref.copy())), ref)
    vals = (0.01 * rng.standard_normal(110_000)).astype(np.float32)
    assert c.compress_float(vals) is vals  # compress_data defaults to False
    cv = Lz4Wrapper(compress_data=True)
    fv = cv.compress_float(vals)
    np.testing.assert_array_equal(np.frombuffer(olz4.ref_decompress(fv), np.float32), vals)
    np.testing.assert_array_equal(cv.decompress_float(fv), vals)
    cm = Lz4Wrapper(compress_metadata=False)
    assert cm.compress(a) is a and cm.decompress(a) is a


@pytest.mark.parametrize("name", ["pm_a01_plain", "pm_a01_acc", "wv_acc"])
def test_plugin_replays_with_lz4wrapper_on_the_wire(name, dev, tmp_path):
    scenario.replay_plugin(name, tmp_path, compression_class="Lz4Wrapper")


def test_running_sum_and_delta_kernels(dev):
    from decentralizepy_amd import codec
    rng = np.random.default_rng(2)
    for k in (1, 4095, 4096, 4097, 1_000_003):
        d = rng.integers(-1000, 100_000, k, dtype=np.int32)
        t = torch.from_numpy(d).to(dev)
        np.testing.assert_array_equal(codec.running_sum_i32(t).cpu().numpy(), np.cumsum(d))
        np.testing.assert_array_equal(codec.running_sum_i32(t, dtype=torch.int32).cpu().numpy(),
                                      np.cumsum(d).astype(np.int32))
        np.testing.assert_array_equal(codec.delta_i32(t).cpu().numpy(),
                                      np.diff(d, prepend=0).astype(np.int32))


def test_c2_index_frame_within_15_percent_of_liblz4(dev):
    """the device encoder's linked frames (2 KB blocks whose matches reach 14 KB
    back, 5-byte hash) on a C2 payload's index gaps stay within 15 % of liblz4's linked 64 KB
    frame (python-lz4's default), and both decoders read them."""
    from decentralizepy_amd import codec
    rng = np.random.default_rng(13)
    idx = np.sort(rng.choice(11_000_000, 110_000, replace=False)).astype(np.int32)
    gaps = np.diff(idx, prepend=0).astype(np.int32).tobytes()
    frame = bytes(codec.lz4_compress(_dev_bytes(gaps, dev)).cpu().numpy().tobytes())
    ref = olz4.ref_compress(gaps)
    assert len(frame) <= 1.15 * len(ref), (len(frame), len(ref))
    assert not (frame[4] & 0x20)  # linked blocks (B.Indep clear), python-lz4's default mode
    assert olz4.ref_decompress(frame) == gaps
    assert bytes(codec.lz4_decompress(frame, dev).cpu().numpy().tobytes()) == gaps
