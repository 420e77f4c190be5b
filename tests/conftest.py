import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "opensim-moco_amd")
if PKG not in sys.path:
    sys.path.insert(0, PKG)
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Make sure the oracle and a libmocohip.so built from this tree exist."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    import __graft_entry__
    __graft_entry__.ensure_built()   # rebuilds a stale library here, refuses one on a GPU box
    yield
