import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built HIP library")


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


_DIAG = None


@pytest.fixture
def diag_lib(monkeypatch):
    """Route codec calls through the diagnostic build (libdpzcodec_diag.so, csrc/dpz_knobs.h)
    for one test, so DPZ_* environment switches set with monkeypatch force kernel paths.  The
    product library reads no environment variable."""
    global _DIAG
    from decentralizepy_amd import _lib
    if _DIAG is None and not os.path.exists(_lib.DIAG_PATH):
        pytest.skip("libdpzcodec_diag.so not built (make -C decentralizepy_amd/csrc diag-lib)")
    if _DIAG is None:
        _DIAG = _lib.diag_lib()
    monkeypatch.setattr(_lib, "_lib", _DIAG)
    return _DIAG
