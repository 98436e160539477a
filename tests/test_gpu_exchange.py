"""The exchange step of a read-sharded job on the device (bench.py --gpus N):
bsq_batch_copy_records puts a batch's records (hits, then CIGAR words) into device memory exactly as the host
view holds them -- from the packed device arrays, or from the pinned host view when a read needed the retry
pass or the batch ran in chunks -- and RecordExchange over an RCCL process group of one rank delivers them to
the caller's host across pipelined steps."""
import ctypes
import os
import socket

import numpy as np
import pytest

from bioseqdb_amd import _native as N
from bioseqdb_amd import synth
from parity_util import build_pair

pytestmark = pytest.mark.gpu


def _host_bytes(L, b):
    H = L.bsq_batch_hits(b).contents
    nb, nc = H.n_hits * ctypes.sizeof(N.Hit), H.n_cigar * 4
    hb = ctypes.string_at(ctypes.cast(H.hits, ctypes.c_void_p), nb) if nb else b""
    cb = ctypes.string_at(ctypes.cast(H.cigar, ctypes.c_void_p), nc) if nc else b""
    return hb + cb


def _run(pi, reads, keep):
    L = N.lib()
    b = ctypes.c_void_p()
    N.check(L.bsq_batch_create(pi.handle, reads.n, int(reads.offsets[-1]), ctypes.byref(b)))
    codes, offs = np.ascontiguousarray(reads.codes), np.ascontiguousarray(reads.offsets)
    keep += [codes, offs]
    N.check(L.bsq_batch_set_reads(b, codes.ctypes.data, offs.ctypes.data, reads.n))
    N.check(L.bsq_batch_run(b, ctypes.byref(pi.options), 0))
    return b


def _device_bytes(L, b, torch):
    n = ctypes.c_int64()
    N.check(L.bsq_batch_copy_records(b, None, 0, ctypes.byref(n)))
    buf = torch.zeros(n.value + 64, dtype=torch.uint8, device="cuda")
    got = ctypes.c_int64()
    assert L.bsq_batch_copy_records(b, ctypes.c_void_p(buf.data_ptr()), n.value - 1, ctypes.byref(got)) != 0 or n.value == 0
    N.check(L.bsq_batch_copy_records(b, ctypes.c_void_p(buf.data_ptr()), n.value, ctypes.byref(got)))
    assert got.value == n.value and int(buf[n.value:].sum()) == 0   # nothing written past the records
    return bytes(buf[:n.value].cpu().numpy())


@pytest.mark.parametrize("mode", ["device", "retry", "chunks"])
def test_copy_records_equals_host_view(monkeypatch, mode):
    import torch
    if mode == "retry":
        monkeypatch.setenv("BSQ_TEST_TINY_CAPS", "1")   # every read through the retry pass: host view
    if mode == "chunks":
        monkeypatch.setenv("BSQ_CHUNK", "700")
    ref = synth.make_reference(500_000, n_rows=2, n_run_every=200_000, n_run_len=200)
    pi, _ = build_pair([t.decode() for t in ref.texts()])
    pi.upload()
    reads = synth.make_reads(ref, 3000, seed=7)
    keep = []
    L = N.lib()
    b = _run(pi, reads, keep)
    try:
        host = _host_bytes(L, b)
        assert len(host) > 3000 * 72
        if mode != "device":
            assert mode == "chunks" or L.bsq_batch_retried(b) > 0
        assert _device_bytes(L, b, torch) == host
    finally:
        L.bsq_batch_free(b)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_record_exchange_rccl_world1():
    """Three pipelined steps of the RCCL exchange with a one-rank process group: after each finish the caller's
    pinned host buffer holds exactly the step's device records."""
    import torch
    import torch.distributed as dist
    from bioseqdb_amd import dist as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        ref = synth.make_reference(400_000, n_rows=1)
        pi, _ = build_pair([t.decode() for t in ref.texts()])
        pi.upload()
        L = N.lib()
        x = D.RecordExchange(device=torch.device("cuda", 0))
        keep = []
        for step in range(3):
            reads = synth.make_reads(ref, 1500 + 500 * step, seed=11 + step)
            b = _run(pi, reads, keep)
            try:
                want = _host_bytes(L, b)
                n = ctypes.c_int64()
                N.check(L.bsq_batch_copy_records(b, None, 0, ctypes.byref(n)))

                def fill(send):
                    got = ctypes.c_int64()
                    N.check(L.bsq_batch_copy_records(b, ctypes.c_void_p(send.data_ptr()), n.value, ctypes.byref(got)))
                x.post_fill(n.value, fill)
                x.finish()
                res = x.result()
                assert len(res) == 1 and res[0].tobytes() == want
            finally:
                L.bsq_batch_free(b)
    finally:
        dist.destroy_process_group()
