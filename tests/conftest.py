import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def load_golden(name):
    """Open a committed fixture; returns (npz, meta-dict)."""
    npz = np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    meta = json.loads(bytes(npz["__meta__"]).decode())
    return npz, meta


@pytest.fixture(scope="session")
def golden():
    return load_golden
