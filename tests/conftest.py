import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden", "r9_golden.npz")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through liblpa_hip.so)")
    config.addinivalue_line("markers", "slow: full-size configuration")


@pytest.fixture(scope="session")
def golden():
    return dict(np.load(GOLDEN, allow_pickle=False))


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as o

    o.build()
    return o
