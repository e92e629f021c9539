import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP library)")
    # build the in-tree libraries only when absent (they normally come prebuilt)
    from foundationdb_amd import build as B
    if not all(os.path.exists(p) for p in (B.LIB, B.WL_LIB, B.ORACLE_LIB)):
        B.build_all()


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    if not gpu_available():
        pytest.skip("no GPU")
    return True
