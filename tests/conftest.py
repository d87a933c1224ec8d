import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.join(ROOT, "tests")
for _p in (ROOT, TESTS):
    if _p not in sys.path:
        sys.path.insert(0, _p)
os.environ["PYTHONPATH"] = os.pathsep.join([ROOT, TESTS] + [x for x in os.environ.get("PYTHONPATH", "").split(os.pathsep) if x])
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: longer CPU test")


def load_golden(name):
    return np.load(os.path.join(GOLDEN, f"{name}.npz"))


@pytest.fixture(scope="session")
def golden():
    return load_golden
