import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
if GOLDEN not in sys.path:
    sys.path.insert(0, GOLDEN)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")


@pytest.fixture(scope="session")
def golden():
    return np.load(os.path.join(GOLDEN, "golden.npz"))


@pytest.fixture(scope="session")
def golden_index():
    with open(os.path.join(GOLDEN, "golden_index.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    from omnifed_amd.build import build

    build()
    return torch.device("cuda", 0)
