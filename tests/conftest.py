import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


@pytest.fixture(scope="session")
def stif():
    import stif_pkg
    return stif_pkg.load()


@pytest.fixture(scope="session")
def sd(stif):
    return stif.weights.make_state_dict(seed=0)


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    d = os.path.join(REPO, "tests", "golden")
    return {n: np.load(os.path.join(d, n + ".npz")) for n in ("model_16x20", "window_7x16x16", "ops", "decoders_16x20")}
