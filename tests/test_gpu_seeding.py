"""Seeding only (BASELINE.json configs[1], "C2"): the GPU's mem_collect_intv intervals per read equal the
oracle's, interval for interval (x[0], x[2], qbeg, qend; x[1] is outside the contract, include/bsq.h)."""
import ctypes

import numpy as np
import pytest

import oracle_py as O
from bioseqdb_amd import synth
from bioseqdb_amd import _native as N
from parity_util import build_pair

pytestmark = pytest.mark.gpu


def _seed(pi, reads, opts):
    L = N.lib()
    pi.upload()
    b = ctypes.c_void_p()
    N.check(L.bsq_batch_create(pi.handle, reads.n, int(reads.offsets[-1]), ctypes.byref(b)))
    try:
        codes = np.ascontiguousarray(reads.codes)
        offs = np.ascontiguousarray(reads.offsets)
        N.check(L.bsq_batch_set_reads(b, codes.ctypes.data, offs.ctypes.data, reads.n))
        N.check(L.bsq_batch_seed(b, ctypes.byref(opts)))
        ro = ctypes.POINTER(ctypes.c_int64)()
        iv = ctypes.POINTER(ctypes.c_uint64)()
        nt = ctypes.c_int64()
        N.check(L.bsq_batch_intervals(b, ctypes.byref(ro), ctypes.byref(iv), ctypes.byref(nt)))
        off = np.ctypeslib.as_array(ro, shape=(reads.n + 1,)).copy()
        arr = np.ctypeslib.as_array(iv, shape=(max(int(nt.value), 1) * 4,)).copy()[: int(nt.value) * 4]
        return off, arr.reshape(-1, 4), int(L.bsq_batch_retried(b))
    finally:
        L.bsq_batch_free(b)


def _check(pi, oi, reads):
    off, iv, retried = _seed(pi, reads, pi.options)
    oo = O.opts_from(pi.options)
    bad = []
    total = 0
    for r in range(reads.n):
        codes = bytes(reads.codes[reads.offsets[r]:reads.offsets[r + 1]])
        exp = [(x0, x2, info) for x0, _x1, x2, info in oi.collect_intv(oo, codes)]
        got = [tuple(int(v) for v in (row[0], row[2], row[3])) for row in iv[off[r]:off[r + 1]]]
        total += len(exp)
        if got != exp:
            bad.append((r, got[:4], exp[:4]))
    return total, bad, retried


def test_seeding_parity_c2_shape():
    ref = synth.make_reference(1_000_000, n_run_every=400_000, n_run_len=500)
    reads = synth.make_reads(ref, 4000, seed=41)
    pi, oi = build_pair([t.decode() for t in ref.texts()])
    total, bad, _ = _check(pi, oi, reads)
    assert total > 4000
    assert not bad, bad[:5]


def test_seeding_parity_retry_path(monkeypatch):
    """Tiny main-pass slots: every read's intervals come from the large-capacity retry kernel."""
    monkeypatch.setenv("BSQ_TEST_TINY_CAPS", "1")
    ref = synth.make_reference(300_000, n_run_every=100_000, n_run_len=200, dup_frac=0.02)
    reads = synth.make_reads(ref, 600, seed=43)
    pi, oi = build_pair([t.decode() for t in ref.texts()])
    total, bad, retried = _check(pi, oi, reads)
    assert retried > 300
    assert not bad, bad[:5]


def test_seeding_parity_chunked(monkeypatch):
    monkeypatch.setenv("BSQ_CHUNK", "900")
    ref = synth.make_reference(400_000, n_run_every=150_000, n_run_len=200)
    reads = synth.make_reads(ref, 2500, seed=47)
    pi, oi = build_pair([t.decode() for t in ref.texts()])
    total, bad, _ = _check(pi, oi, reads)
    assert total > 2500
    assert not bad, bad[:5]
