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


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_group_bench_gather_via_first_member():
    """--exchange via-first: member 1's records reach the host through member 0's HBM (peer DMA, then member 0's
    link) under the stream-of-rounds schedule; the rows are the same as one-GPU runs'."""
    g = _bench("--gpus", "2", "--group-devices", "0,0", "--exchange", "via-first", "--no-isolated")
    assert g["exchange"]["mode"] == "via-first" and "xGMI" in g["exchange"]["path"]
    assert "stream of rounds" in g["config"]["step_schedule"]
    assert all(p["checksum_match"] for p in g["parity_sample"]), g["parity_sample"]
    for k in range(2):
        one = _bench("--seed-offset", str(k), "--timed-only")
        assert one["checksums"][0] == g["checksums"][k], k


def test_native_exchange_world1_stream_of_rounds():
    """The torchrun path with a one-rank RCCL group (--exchange-world1): the exchange lanes (bsq_xchg) run beside
    the stream of rounds and the records are those of the launcher-free run."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *SMALL, "--exchange-world1", "--timed-only"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    x = json.loads(r.stdout.strip().splitlines()[-1])
    assert "bsq_xchg" in x["exchange"]["path"] and x["exchange"]["lanes"] == 4
    assert "stream of batch runs" in x["config"]["step_schedule"]
    one = _bench("--timed-only")
    assert x["checksums"] == one["checksums"]


def test_native_exchange_failure_stops_cleanly():
    """A batch failure inside the exchanged stream of rounds (injected on lane 2, round 1 by BSQ_XCHG_TEST_FAIL) is
    carried by the header all-gather's status word: the run stops at that (round, lane), the RCCL communicator is
    aborted, and bench.py exits non-zero naming it -- instead of the other lanes (and, with more ranks, the other
    ranks) waiting forever in their collectives."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0", BSQ_XCHG_TEST_FAIL="2:1", BSQ_XCHG_TIMEOUT_S="60")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *SMALL, "--exchange-world1", "--timed-only"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode != 0
    assert "rank 0 lane 2 round 1 failed" in r.stderr and "injected failure" in r.stderr, r.stderr[-3000:]
