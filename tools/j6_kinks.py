"""CPU scan of J = 6 windows for ReLU units within fp32 noise of their kink
(tests/test_gpu_parity_s256.py::_relu_kinks on the oracle's own fp64 features): the windows the
J = 6 end-to-end test can hold an fp32 step to the fp64 oracle on.
Usage: python tools/j6_kinks.py FIRST LAST"""
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "vae-teb_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402
from test_gpu_parity_s256 import _oracle_features, _relu_kinks  # noqa: E402
from vaeteb import synthetic  # noqa: E402
from vaeteb.frontend import load_stats  # noqa: E402

torch.set_num_threads(8)
st = load_stats(6, 1, 16, 4096)
fe = types.SimpleNamespace(plan=types.SimpleNamespace(J=6, Q=1, T=16, N=4096))
eps = np.random.default_rng(6).standard_normal((2, 256, 32)).astype(np.float32)
for w in range(int(sys.argv[1]), int(sys.argv[2]) + 1):
    x = synthetic.batch(w, 2, 4096)
    f64 = _oracle_features(fe, x, st, np.float64, "numpy")
    widths = (f64["fhr_st"].shape[2], f64["fhr_ph"].shape[2], f64["fhr_up_ph"].shape[2])
    n, worst = _relu_kinks(f64, eps, widths)
    print(f"window {w}: {n} ReLU inputs within 10x fp32 noise of the kink (smallest ratio {worst:.2f})", flush=True)
