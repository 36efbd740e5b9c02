import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); runs on the GPU box")
    config.addinivalue_line("markers", "slow: full-size (BASELINE) shapes")


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import geeps_amd
    geeps_amd.lib()  # the HIP library must load: no fallback
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def golden_rowops():
    import numpy as np
    return np.load(os.path.join(GOLDEN, "rowops.npz"))


@pytest.fixture(scope="session")
def golden_bucket():
    import numpy as np
    return np.load(os.path.join(GOLDEN, "bucket.npz"))


@pytest.fixture(scope="session")
def manifest():
    import json
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)
