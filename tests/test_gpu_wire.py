"""The exchange's wire form (bsq_xchg; the rows that reach the caller's tuplestore,
bioseqdb/extension.cpp:362-370) checked on one GPU: a batch's records through the same device pack the send path
launches (k_wire_pack) and back through rank 0's host expansion must equal the batch's own view byte for byte --
records on the device (one chunk, no retry) and the staged host view (reads through the retry pass), several
reference rows (ref_id / ref_match_* from the anns), both strands, reads without hits.  And the bytes it saves."""
import ctypes

import numpy as np
import pytest

from bioseqdb_amd import _native as N
from bioseqdb_amd import synth
from parity_util import build_pair

pytestmark = pytest.mark.gpu


def _wire_check(pi, reads, first_call=0):
    L = N.lib()
    b = ctypes.c_void_p()
    codes = np.ascontiguousarray(reads.codes)
    offs = np.ascontiguousarray(reads.offsets)
    N.check(L.bsq_batch_create(pi.handle, reads.n, int(offs[-1]), ctypes.byref(b)))
    try:
        N.check(L.bsq_batch_set_reads(b, codes.ctypes.data, offs.ctypes.data, reads.n))
        N.check(L.bsq_batch_run(b, ctypes.byref(pi.options), first_call))
        h = L.bsq_batch_hits(b).contents
        wb, rb, bad = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        N.check(L.bsq_xchg_wire_check(b, pi.handle, ctypes.byref(wb), ctypes.byref(rb), ctypes.byref(bad)))
        return int(h.n_hits), wb.value, rb.value, bad.value
    finally:
        L.bsq_batch_free(b)


def _ref():
    return synth.make_reference(600_000, n_rows=5, n_run_every=150_000, n_run_len=200)


def test_wire_roundtrip_device_records():
    ref = _ref()
    pi, _ = build_pair([t.decode() for t in ref.texts()], ids=[11, -3, 7, 1 << 40, 5])
    pi.upload()
    reads = synth.make_reads(ref, 20_000, seed=41)
    n_hits, wire, raw, bad = _wire_check(pi, reads, first_call=9)
    assert n_hits > 18_000 and bad == 0
    assert wire <= 0.6 * raw, (wire, raw)   # >= 40 % fewer bytes per (round, lane) on the link


def test_wire_roundtrip_staged_host_view(monkeypatch):
    monkeypatch.setenv("BSQ_TEST_TINY_CAPS", "1")   # reads through the retry pass: the records are a host view
    ref = _ref()
    pi, _ = build_pair([t.decode() for t in ref.texts()])
    pi.upload()
    reads = synth.make_reads(ref, 800, seed=43)
    n_hits, wire, raw, bad = _wire_check(pi, reads)
    assert n_hits > 700 and bad == 0
