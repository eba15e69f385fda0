import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
os.environ.setdefault("ZP_QUIET", "1")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through libzp.so)")


def has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        # materialised: an NpzFile re-reads (and re-inflates) the member on every item access
        with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
            return {k: z[k] for k in z.files}
    return load


@pytest.fixture
def gpu():
    if not has_gpu():
        pytest.skip("no GPU")
    import torch
    return torch.device("cuda:0")
