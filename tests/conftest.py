import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


@pytest.fixture(scope="session")
def built():
    from openge_amd.build import build
    build()
    import oracle
    oracle.build()
    return True


@pytest.fixture(scope="session")
def ctx(built):
    from openge_amd import lib as L
    c = L.Context(0)
    yield c
    c.close()
