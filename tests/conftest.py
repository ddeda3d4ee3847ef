import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device) -- run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


GOLDEN = os.path.join(ROOT, "tests", "golden")
REFERENCE = os.environ.get("PUCFEM_REFERENCE", "/root/reference")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    cache = {}

    def load(name):
        if name not in cache:
            cache[name] = dict(np.load(os.path.join(GOLDEN, f"golden_{name}.npz")))
        return cache[name]

    return load


def load_pkg():
    """The product package (its directory name has hyphens, so import it by name)."""
    import importlib

    return importlib.import_module("puc-fluidsimulation-project_amd")


@pytest.fixture(scope="session")
def pf():
    return load_pkg()


def has_gpu():
    try:
        return load_pkg().device_count() > 0
    except Exception:
        return False
