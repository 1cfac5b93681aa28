"""CPU: the Choco oracle (oracle/choco.py) replays the reference's own Choco runs
(tests/golden/choco.npz from the unmodified reference sharing/Choco.py, see
make_golden_choco.py) bit-exactly: threshold sparsification with every tie kept, the nonzero
filter, the k = 0 branch, and the x_hat / s / x updates of _averaging over three rounds."""
import json
import os

import numpy as np
import pytest

from oracle import choco as ochoco

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


@pytest.mark.parametrize("tag", ["a", "z"])
def test_choco_oracle_matches_reference_fixture(tag):
    meta = json.load(open(os.path.join(GOLD, "choco.json")))[tag]
    g = np.load(os.path.join(GOLD, "choco.npz"))
    n = meta["n"]
    k = round(meta["alpha"] * n)
    x_hat = np.zeros(n, np.float32)
    s = np.zeros(n, np.float32)
    for r, rm in enumerate(meta["rounds"]):
        x = g[f"{tag}_r{r}_x"]
        q = ochoco.sparsify(x - x_hat, k)
        idx, vals = ochoco.serialize(q)
        np.testing.assert_array_equal(idx, g[f"{tag}_r{r}_idx"])
        np.testing.assert_array_equal(_bits(vals), _bits(g[f"{tag}_r{r}_vals"]))
        pays = [(g[f"{tag}_r{r}_nbr{j}_idx"], g[f"{tag}_r{r}_nbr{j}_vals"]) for j in range(3)]
        x, x_hat, s = ochoco.averaging(x, x_hat, s, q, pays, rm["degrees"], meta["step_size"])
        np.testing.assert_array_equal(_bits(x_hat), _bits(g[f"{tag}_r{r}_x_hat"]))
        np.testing.assert_array_equal(_bits(s), _bits(g[f"{tag}_r{r}_s"]))
        np.testing.assert_array_equal(_bits(x), _bits(g[f"{tag}_r{r}_x_after"]))
