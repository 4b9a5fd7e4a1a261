import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "red-diffeq_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

collect_ignore_glob = ["golden/*.py"]   # fixture generators: run the reference, never on the box


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels)")


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def ctx_of(z):
    return {k[4:]: (z[k].item() if z[k].ndim == 0 else z[k]) for k in z.files if k.startswith("ctx_")}


def vnorm(v):
    return ((v - 1500) / 3000 * 2 - 1).astype(np.float32)


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
