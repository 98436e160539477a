"""bench.py --gpus N without a launcher: N devices driven from one process (bsq_group), the way the Postgres
backend drives them and the way an 8-GPU node runs the BASELINE metric's 1/2/4/8 curve.

The one-GPU box holds the N = 3 group as three replicas of the index on device 0 (device-to-device copies
instead of the RCCL broadcast, which cannot hold one device twice).  The line must report n_gpus = 3 and
3x the reads of one member; member k's rows (checksummed in the oracle's format with member-local read
indices) must equal a one-GPU run of the same reads (--seed-offset k: reads of seed READ_SEED + k, lrand48
position k * reads), and the bench's own oracle sample of the first and last member must match.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--reads", "40000", "--ref-bp", "2000000", "--steps", "2", "--warmup", "1", "--no-codec", "--checksums"]


def _bench(*args):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *SMALL, *args], capture_output=True,
                       text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_group_bench_three_members_equal_one_gpu_runs():
    g = _bench("--gpus", "3", "--group-devices", "0,0,0")
    assert g["n_gpus"] == 3
    assert g["config"]["distinct_devices"] == 1
    assert g["value"] > 0 and g["ms_per_step"] > 0
    assert len(g["checksums"]) == 3
    assert all(p["checksum_match"] for p in g["parity_sample"]), g["parity_sample"]
    assert g["roofline"]["frac"] > 0
    for k in range(3):
        one = _bench("--seed-offset", str(k), "--timed-only")
        assert one["n_gpus"] == 1
        assert one["checksums"][0] == g["checksums"][k], k


def test_group_bench_fails_loudly_without_enough_devices():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *SMALL, "--gpus", "64"], capture_output=True,
                       text=True, timeout=300, cwd=ROOT)
    assert r.returncode != 0
    assert "HIP device(s) visible" in r.stderr
