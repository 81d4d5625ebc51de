import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "vae-teb_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: long-running CPU case")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    return load


@pytest.fixture(autouse=True)
def _h16_format_reset():
    """Every test starts and ends with the library's 16-bit operand format at bf16 (the default):
    the format is library-wide state (vt_set_h16_format) that the model ops select per call, but a
    test calling the C ABI directly would otherwise inherit the fp16 format a previous test left."""
    def reset():
        try:
            from vaeteb import _lib
            if _lib._lib is not None:
                _lib.set_h16(False)
        except Exception:
            pass
    reset()
    yield
    reset()
