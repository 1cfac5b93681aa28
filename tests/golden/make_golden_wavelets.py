#!/usr/bin/env python3
"""Golden vectors for the generic-filter wavelet path: PyWavelets 1.1.1 (the only pywt in this
image, /opt/conda/bin/python3.9) on seeded fp32 inputs, mode "symmetric" as the reference's
Wavelet plugin calls it (sharing/JWINS/Wavelet.py:12-32 wavedec + coeffs_to_array,
:311-316 array_to_coeffs + waverec).  Run in the build container:

    python tests/golden/make_golden_wavelets.py

Writes tests/golden/wavelet_generic_pywt.npz (allow_pickle=False): per case ``<name>/<n>/<level>``
the input x, ``coeffs_to_array(wavedec(x))``, a second coefficient vector c and
``waverec(array_to_coeffs(c))``.
"""
import os
import subprocess

PY39 = "/opt/conda/bin/python3.9"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "wavelet_generic_pywt.npz")
CASES = [("db1", 1001, 4), ("db2", 1001, 4), ("db3", 4098, 4), ("db4", 4099, 4),
         ("db8", 10007, 3), ("db20", 20000, 2), ("sym3", 2049, 4), ("sym5", 5001, 4),
         ("sym8", 7777, 3), ("coif1", 999, 4), ("coif3", 6000, 3), ("bior2.6", 3001, 3),
         ("bior3.5", 4000, 4), ("rbio1.3", 1500, 4), ("rbio3.7", 3333, 3), ("dmey", 20011, 2),
         ("haar", 1001, 4), ("sym2", 1001, 4), ("db4", 64, 1), ("db4", 15, 1)]

_GEN = r"""
import sys, warnings
import numpy as np
warnings.filterwarnings("ignore")
import pywt
cases, out = eval(sys.argv[1]), sys.argv[2]
arrs = {"pywavelets": np.array(pywt.__version__)}
for name, n, level in cases:
    rng = np.random.default_rng(n * 31 + level)
    x = rng.standard_normal(n).astype(np.float32)
    c, _ = pywt.coeffs_to_array(pywt.wavedec(x, name, mode="symmetric", level=level))
    shapes = pywt.wavedec(np.zeros(n, np.float32), name, mode="symmetric", level=level)
    _, slices = pywt.coeffs_to_array(shapes)
    cr = rng.standard_normal(c.shape[0]).astype(np.float32)
    rec = pywt.waverec(pywt.array_to_coeffs(cr, slices, output_format="wavedec"), name,
                       mode="symmetric")
    key = "%s/%d/%d" % (name, n, level)
    arrs[key + "/x"] = x
    arrs[key + "/coeffs"] = np.asarray(c, dtype=np.float32)
    arrs[key + "/c"] = cr
    arrs[key + "/rec"] = np.asarray(rec, dtype=np.float32)
np.savez(out, **arrs)
"""


def main():
    subprocess.run([PY39, "-c", _GEN, repr(CASES), OUT], check=True)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
