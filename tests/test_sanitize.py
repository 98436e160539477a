"""ASan/UBSan run of the host code of the path and of the CPU oracle: the nuclseq codec,
libbsq's host index build, the bwa_result renderer and the FASTA reader, compiled with
-fsanitize=address,undefined beside the oracle and checked against it (tools/sanitize/host_check.cpp)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_code_clean_under_asan_ubsan():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools", "sanitize"), "run"], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0 and "host_check: ok" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
