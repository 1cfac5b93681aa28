"""CPU: pin the oracle against the reference's own outputs (golden fixtures generated from the
unmodified reference by tests/golden/make_golden.py)."""
import os

import numpy as np
import pytest

from oracle import elias as oelias
from oracle import fold as ofold
from oracle import wavelet as owav
from tests import scenario

GOLDEN = scenario.GOLDEN


@pytest.mark.parametrize("name", scenario.scenario_names())
def test_oracle_replays_reference_scenario(name):
    scenario.replay_oracle(name)


@pytest.mark.parametrize("name", ["sharing_full", "server_sharing"])
def test_oracle_full_model_sharing_fold(name):
    meta = next(s for s in scenario.load_meta()["scenarios"] if s["name"] == name)
    a = dict(np.load(os.path.join(GOLDEN, f"{name}.npz")))
    pays = [(None, a[f"r0_nbr{i}_params"]) for i in range(3)]
    if meta.get("averaging") == "_averaging_server":  # reference Sharing.py:200-229
        out = ofold.fold(a["x0"], pays, [1 / 3] * 3, None)
    else:
        w = [ofold.mh_weight(3, nb["degree"]) for nb in meta["neighbours"]]
        wt = 0
        for v in w:
            wt += v
        out = ofold.fold(a["x0"], pays, w, 1 - wt)
    np.testing.assert_array_equal(out.view(np.uint32), a["r0_model_after"].view(np.uint32))
    np.testing.assert_array_equal(a["sent_params"], a["x0"])


def test_oracle_elias_matches_reference_bytes():
    a = dict(np.load(os.path.join(GOLDEN, "elias.npz")))
    for case in scenario.load_meta()["elias_cases"]:
        enc = oelias.encode(a[f"{case}_input"])
        np.testing.assert_array_equal(enc, a[f"{case}_bytes"], err_msg=case)
        np.testing.assert_array_equal(oelias.decode(a[f"{case}_bytes"]), a[f"{case}_decoded"])
        np.testing.assert_array_equal(a[f"{case}_decoded"], a[f"{case}_sorted"])


def test_elias_known_answer_vector():
    # Elias().compress(int32[10,3,6,5]) -> 18 bytes
    assert oelias.encode(np.array([10, 3, 6, 5], np.int32)).tobytes().hex() == \
        "520003000000000000008900000000000000"


def test_oracle_haar_matches_pywt():
    """haar (the reference Wavelet's default) wavedec / waverec of PyWavelets 1.1.1, levels 1-8,
    odd and even sizes (tests/golden/make_golden.py --haar)."""
    import json
    a = dict(np.load(os.path.join(GOLDEN, "wavelet_haar_pywt.npz")))
    with open(os.path.join(GOLDEN, "haar_scenarios.json")) as f:
        cases = json.load(f)["pywt_cases"]
    for n, level in cases:
        key = f"n{n}_l{level}"
        c = owav.wavedec_array(a[f"{key}_x"], level, "haar")
        np.testing.assert_array_equal(c.view(np.uint32), a[f"{key}_coeffs"].view(np.uint32))
        assert c.shape[0] == owav.coeff_len(n, level, "haar")
        rec = owav.waverec_array(a[f"{key}_coeffs"], n, level, "haar")
        np.testing.assert_array_equal(rec.view(np.uint32), a[f"{key}_rec"][:n].view(np.uint32))


def test_oracle_wavelet_matches_pywt():
    a = dict(np.load(os.path.join(GOLDEN, "wavelet_pywt.npz")))
    for n in scenario.load_meta()["wavelet_sizes"]:
        x = a[f"n{n}_x"]
        c = owav.wavedec_array(x, 4)
        np.testing.assert_array_equal(c.view(np.uint32), a[f"n{n}_coeffs"].view(np.uint32))
        rec = owav.waverec_array(a[f"n{n}_coeffs"], n, 4)
        np.testing.assert_array_equal(rec.view(np.uint32), a[f"n{n}_rec"][:n].view(np.uint32))
