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


def _padded(enc):
    nbytes = enc.size
    buf = torch.zeros(((nbytes + 3) // 4) * 4 + 16, dtype=torch.uint8)
    buf[:nbytes] = torch.from_numpy(enc)
    return buf, nbytes, int(enc[-8:].view("<i8")[0]), int(enc[-16:-8].view("<i8")[0])


@pytest.mark.parametrize("dt", [torch.int32, torch.int64])
def test_elias_async_decode(dev, dt):
    """dpz_elias_decode_async: the values of dpz_elias_decode with no host synchronisation; the
    status word stays 0 for a well-formed stream of the expected count and is OR-ed nonzero for a
    count mismatch or a malformed stream (all-zero code bits: no code ever terminates)."""
    from decentralizepy_amd import codec
    rng = np.random.default_rng(9)
    for idx in (np.sort(rng.choice(25_000_009, 250_000, replace=False)).astype(np.int32),
                np.array([0, 2**31 - 1], np.int32), np.arange(3, 70_003, dtype=np.int32)):
        buf, nbytes, nbits, first = _padded(oelias.encode(idx))
        status = torch.zeros(1, dtype=torch.int32, device=dev)
        out = codec.elias_decode_async(buf.to(dev), nbytes, nbits, first, idx.size, status,
                                       dtype=dt)
        np.testing.assert_array_equal(out.cpu().numpy(), idx.astype(out.cpu().numpy().dtype))
        assert int(status.item()) == 0
        for wrong in (idx.size - 1, idx.size + 1):
            s2 = torch.zeros(1, dtype=torch.int32, device=dev)
            codec.elias_decode_async(buf.to(dev), nbytes, nbits, first, wrong, s2, dtype=dt)
            assert int(s2.item()) != 0
    # one value (L = 0): the trailer alone
    one = np.zeros(16, np.uint8)
    one[:8] = np.frombuffer(np.int64(41).tobytes(), np.uint8)
    one[8:] = np.frombuffer(np.int64(128).tobytes(), np.uint8)
    buf, nbytes, nbits, first = _padded(one)
    for count, bad in ((1, False), (2, True)):
        s = torch.zeros(1, dtype=torch.int32, device=dev)
        out = codec.elias_decode_async(buf.to(dev), nbytes, nbits, first, count, s, dtype=dt)
        assert int(out[0].item()) == 41 and (int(s.item()) != 0) == bad
    # malformed: 4096 zero code bits
    zeros = np.zeros(512 + 16, np.uint8)
    zeros[-16:-8] = np.frombuffer(np.int64(5).tobytes(), np.uint8)
    zeros[-8:] = np.frombuffer(np.int64(128 + 4096).tobytes(), np.uint8)
    buf, nbytes, nbits, first = _padded(zeros)
    s = torch.zeros(1, dtype=torch.int32, device=dev)
    codec.elias_decode_async(buf.to(dev), nbytes, nbits, first, 100, s, dtype=dt)
    assert int(s.item()) != 0
    with pytest.raises(ValueError):
        codec.elias_decode(buf.to(dev), nbytes, nbits, first, 4096, dtype=dt)


@pytest.mark.parametrize("cls", ["Elias", "EliasFpzip"])
def test_plugin_async_receive_rejects_a_malformed_payload(cls, dev, tmp_path):
    """The plugin's receive decodes without host synchronisation; a neighbour payload whose
    index stream holds fewer values than its value leg (or a malformed float stream) raises
    ValueError at the round's one status check, before the model is loaded, and the next round
    with good payloads runs normally."""
    from collections import deque

    from decentralizepy_amd.sharing.PartialModel import PartialModel
    meta, arrays = scenario.load("pm_a01_plain")
    model = scenario.make_model(meta["shape"])
    scenario.set_flat(model, arrays["x0"])
    kwargs = dict(meta["kwargs"], compress=True, compression_class=cls,
                  compression_package=f"decentralizepy_amd.compression.{cls}")
    plugin = PartialModel(0, 0, None, scenario._Mapping(), scenario._Graph([1, 2, 3]), model,
                          None, str(tmp_path), **kwargs)
    mr = meta["rounds"][0]
    scenario.set_flat(model, arrays["r0_x"])
    plugin.get_data_to_send(degree=3)
    before = scenario.get_flat(model)
    msgs = scenario._elias_wire(scenario.neighbour_msgs(mr, arrays, 0), cls)
    j = next(i for i, m in enumerate(msgs) if "indices" in m)  # a partial share
    bad = dict(msgs[j])
    idx = oelias.decode(np.asarray(bad["indices"]))
    bad["indices"] = oelias.encode(idx[:-1].astype(np.int32))  # one index short
    msgs[j] = bad
    peer = {uid: deque([m]) for uid, m in zip([1, 2, 3], msgs)}
    with pytest.raises(ValueError):
        plugin._averaging(peer)
    np.testing.assert_array_equal(scenario.get_flat(model), before)  # nothing loaded
    # a good round after the failed one: the status word was cleared
    plugin.get_data_to_send(degree=3)
    msgs = scenario._elias_wire(scenario.neighbour_msgs(mr, arrays, 0), cls)
    plugin._averaging({uid: deque([m]) for uid, m in zip([1, 2, 3], msgs)})
