"""CPU: the FFT-plugin oracle (oracle/fft.py) replays the reference FFT plugin's recorded rounds
(tests/golden/make_golden_fft.py): exact indices and counters, complex values / accumulators /
averaged models within scenario.fft_tol (float64 numpy FFT vs torch's float32 pocketfft)."""
import pytest

from tests import scenario


@pytest.mark.parametrize("name", scenario.fft_names())
def test_fft_oracle_replays_reference(name):
    scenario.replay_fft_oracle(name)
