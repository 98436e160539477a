"""The driver's torchrun bench with the NATIVE RCCL record exchange between processes (the rows of
every rank reach the caller's tuplestore, bioseqdb/extension.cpp:362-370), on the one-GPU box.

RCCL refuses two ranks on one device ("Duplicate GPU detected", judged by host id + bus id), so bench.py's
BSQ_REHEARSE_SHARED_GPU=1 gives every rank a host id of its own (NCCL_HOSTID) and RCCL connects them over its socket
transport on the loopback device.  The exchange then runs for real: ncclCommInitRank at world 2, the header
all-gathers, ncclSend/ncclRecv of the 32-B wire records and the per-read counts, rank 0's host expansion.  Rank 0's copy
of every rank's records (checksummed in the oracle's format) must equal a one-GPU run of that rank's reads
(--seed-offset r).  The 8-GPU node runs the same code over xGMI."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--reads", "40000", "--ref-bp", "2000000", "--steps", "2", "--warmup", "1", "--checksums", "--no-cpu-baseline",
         "--no-codec"]


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_native_exchange_two_processes_equal_one_gpu_runs():
    env = dict(os.environ, BSQ_REHEARSE_SHARED_GPU="1", BSQ_XCHG_TIMEOUT_S="120")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                        os.path.join(ROOT, "bench.py"), "--gpus", "2", *SMALL],
                       capture_output=True, text=True, timeout=540, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and len(line["checksums"]) == 2
    x = line["exchange"]
    assert "bsq_xchg" in x["path"] and x["lanes"] == 4 and x["bytes_per_step"] > 0
    for k in range(2):
        one = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *SMALL, "--timed-only", "--seed-offset",
                              str(k)], capture_output=True, text=True, timeout=300, cwd=ROOT)
        assert one.returncode == 0, one.stderr[-3000:]
        assert json.loads(one.stdout.strip().splitlines()[-1])["checksums"] == [line["checksums"][k]], k
