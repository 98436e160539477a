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


@pytest.fixture(autouse=True)
def _introsort_guard_stays_zero(request):
    """every GPU test ends with bsq_sort_guard_total() == 0 -- no introsort partition scan in
    k_chain / k_chain_s / k_extend was stopped by the `i < t` bound instead of klib's sentinel (the round-2
    hang's would-be runaway).  A non-zero count fails the test that produced it."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    from bioseqdb_amd._native import lib
    g = lib().bsq_sort_guard_total()
    assert g == 0, f"{g} introsort scans stopped by the bound, not the sentinel"


@pytest.fixture(scope="session")
def gpu_available():
    from bioseqdb_amd._native import lib
    return lib().bsq_device_count() > 0


def pytest_sessionstart(session):
    # Two HIP runtimes share this process: torch's bundled one and the system one libbsq links.  Both
    # work when torch is loaded and has initialised the GPU before libbsq does (torch's HSA runtime is
    # then the process-wide one); the other order leaves torch with "No HIP GPUs are available".  The
    # multi-GPU driver orders them the same way (bench.py, bioseqdb_amd/dist.py).
    try:
        import torch
        if torch.cuda.device_count() > 0:   # counting does not initialise the GPU; init() does
            torch.cuda.init()
    except Exception:
        pass
