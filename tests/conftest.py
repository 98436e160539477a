import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) device")


def _ensure_built():
    lib = os.path.join(ROOT, "bioseqdb_amd", "libbsq.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "bioseqdb_amd", "csrc")], check=True)
    orc = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(orc):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def gpu_available():
    from bioseqdb_amd._native import lib
    return lib().bsq_device_count() > 0
