"""GPU parity of the Elias-gamma codec (dpz_elias_encode / dpz_elias_decode) and the compression
classes against the reference's own bytes (tests/golden/elias.npz, made by the unmodified
reference Elias) and the reference-pinned oracle (oracle/elias.py) at full sizes."""
import os

import numpy as np
import pytest
import torch

from oracle import elias as oelias
from tests import scenario

pytestmark = pytest.mark.gpu

GOLDEN = scenario.GOLDEN


def _golden():
    return dict(np.load(os.path.join(GOLDEN, "elias.npz"))), scenario.load_meta()["elias_cases"]


def test_elias_known_answer_device(dev):
    from decentralizepy_amd import codec
    idx = torch.tensor([3, 5, 6, 10], dtype=torch.int32, device=dev)
    enc = codec.elias_encode(idx)
    assert enc.cpu().numpy().tobytes().hex() == "520003000000000000008900000000000000"


def test_elias_reference_bytes_encode_decode(dev):
    from decentralizepy_amd.compression.Elias import Elias
    a, cases = _golden()
    c = Elias()
    for case in cases:
        inp = a[f"{case}_input"].copy()
        enc = c.compress(inp)
        np.testing.assert_array_equal(inp, a[f"{case}_sorted"], err_msg=case)  # sorted in place
        np.testing.assert_array_equal(enc, a[f"{case}_bytes"], err_msg=case)
        dec = c.decompress(a[f"{case}_bytes"])
        assert dec.dtype == np.int64
        np.testing.assert_array_equal(dec, a[f"{case}_decoded"], err_msg=case)


@pytest.mark.parametrize("n,k,seed", [(11_000_000, 110_000, 1), (25_000_009, 250_000, 2),
                                      (67_108_864, 67_109, 3), (16_777_216, 167_772, 4),
                                      (5000, 4000, 5), (2**31 - 1, 1000, 6)])
def test_elias_full_size_vs_oracle(dev, n, k, seed):
    from decentralizepy_amd import codec
    rng = np.random.default_rng(seed)
    idx = np.sort(rng.choice(n, size=k, replace=False)).astype(np.int32)
    ref = oelias.encode(idx)
    d = torch.from_numpy(idx).to(dev)
    enc = codec.elias_encode(d).cpu().numpy()
    np.testing.assert_array_equal(enc, ref)
    nbytes = ref.size
    buf = torch.zeros(((nbytes + 3) // 4) * 4 + 16, dtype=torch.uint8)
    buf[:nbytes] = torch.from_numpy(ref)
    nbits = int(ref[-8:].view("<i8")[0])
    first = int(ref[-16:-8].view("<i8")[0])
    for dt in (torch.int64, torch.int32):
        out = codec.elias_decode(buf.to(dev), nbytes, nbits, first, nbits - 127, dtype=dt)
        np.testing.assert_array_equal(out.cpu().numpy(), idx.astype(out.cpu().numpy().dtype))


def test_elias_extreme_gaps(dev):
    from decentralizepy_amd.compression.Elias import Elias
    c = Elias()
    cases = [np.array([0, 2**31 - 1], np.int32),                     # one 61-bit code
             np.arange(0, 70_000, dtype=np.int32),                   # all 1-bit codes
             np.array([0] + [2**j for j in range(31)], np.int64).cumsum().clip(max=2**31 - 1)
             .astype(np.int32)[:31],
             np.concatenate([np.arange(0, 3000, dtype=np.int32),    # codes straddling chunks
                             np.arange(3000, 2**31 - 1, 2**22, dtype=np.int32)])]
    rng = np.random.default_rng(7)
    for _ in range(4):  # mixed lengths: random gaps with log-uniform magnitude
        g = (2 ** rng.uniform(0, 16, size=20_000)).astype(np.int64) + 1
        cases.append(np.cumsum(g).astype(np.int32))
    for a in cases:
        a = np.unique(a)
        enc = c.compress(a.copy())
        np.testing.assert_array_equal(enc, oelias.encode(a))
        np.testing.assert_array_equal(c.decompress(enc), a.astype(np.int64))


def test_elias_errors(dev):
    from decentralizepy_amd import codec
    from decentralizepy_amd.compression.Elias import Elias
    c = Elias()
    with pytest.raises(IndexError):
        c.compress(np.array([5], np.int32))
    with pytest.raises(IndexError):
        c.compress(np.array([], np.int32))
    with pytest.raises(ValueError):  # duplicate index -> zero gap, invalid in the reference too
        codec.elias_encode(torch.tensor([1, 4, 4, 9], dtype=torch.int32, device=dev))


def test_elias_device_entry_points(dev):
    from decentralizepy_amd.compression.Elias import Elias
    c = Elias()
    idx = torch.arange(7, 7 + 3 * 50_000, 3, dtype=torch.int32, device=dev)
    enc = c.compress_device(idx)
    np.testing.assert_array_equal(enc, oelias.encode(idx.cpu().numpy()))
    back = c.decompress_device(enc)
    assert back.dtype == torch.int32 and back.is_cuda
    assert torch.equal(back, idx)


@pytest.mark.parametrize("name", ["pm_a01_plain", "pm_a02_accavg", "wv_acc", "jwins_tutorial"])
@pytest.mark.parametrize("cls", ["Elias", "EliasFpzip"])
def test_plugin_with_compression(name, cls, dev, tmp_path):
    scenario.replay_plugin(name, tmp_path, compression_class=cls)


def test_fp16_compressor_roundtrip(dev):
    from decentralizepy_amd.compression.EliasFp16 import EliasFp16
    c = EliasFp16()
    x = np.random.default_rng(3).standard_normal(100_001).astype(np.float32)
    enc = c.compress_float(x)
    assert enc.dtype == np.uint8 and enc.size == 2 * x.size
    np.testing.assert_array_equal(c.decompress_float(enc), x.astype(np.float16).astype(np.float32))
