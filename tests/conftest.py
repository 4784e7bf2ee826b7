import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the in-tree artefacts once if they are missing (make is incremental)."""
    from vampomi_amd import _lib
    from oracle import pyoracle

    if not (os.path.exists(_lib.LIB_PATH) and os.path.exists(pyoracle.LIB_PATH) and os.path.exists(_lib.CLI_PATH)):
        from vampomi_amd import build

        build.build(oracle=True)
    yield


def relerr(a, b):
    import numpy as np

    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    nb = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / nb) if nb > 0 else float(np.linalg.norm(a))
