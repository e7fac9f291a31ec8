import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HERE = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

import wst_amd  # noqa: E402,F401  (registers the package under its importable name)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built HIP library")
    config.addinivalue_line("markers", "slow: longer CPU test")


GOLDEN = os.path.join(HERE, "golden")


def load_golden(name):
    import numpy as np
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}
