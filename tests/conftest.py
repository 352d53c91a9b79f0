import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "nlp-filter_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through libmhe.so)")


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    return {name: np.load(os.path.join(GOLDEN, name + ".npz"))
            for name in ("collocation", "plugins", "ekf_gnss_stationary", "least_squares")}
