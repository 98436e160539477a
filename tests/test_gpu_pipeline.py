"""Pipelined cursor fetches (bsq_pipeline) and the pipelined one-shot call.

The reference aligns a cursor row by row, fetch after fetch (extension.cpp:156-195, 362-370).  The pipeline
keeps up to n_slots fetches on the device while the caller stages the next one and consumes the last: every
fetch's rows must equal aligning that fetch alone (read order, lrand48 positions, CIGAR offsets), results
must come back in submission order, a submission's reads may be released as soon as submit returns, and the
nuclseq columns rendered in the pipeline must equal bsq_batch_render_nuclseqs.  bsq_align_batch splits a
large call over its index's pipeline: the rows must not depend on the split.
"""
import ctypes
import gc

import pytest

from bioseqdb_amd import NucleotideSequence, synth
from bioseqdb_amd import _native as N
from parity_util import build_pair

pytestmark = pytest.mark.gpu


def _records(H, n):
    hits = ctypes.string_at(H.hits, H.n_hits * ctypes.sizeof(N.Hit)) if H.n_hits else b""
    cig = ctypes.string_at(H.cigar, H.n_cigar * 4) if H.n_cigar else b""
    off = ctypes.string_at(H.read_off, (n + 1) * 8)
    return hits, cig, off


def _one_shot(L, h, opts, seqs, first_call):
    n = len(seqs)
    ptrs = (ctypes.c_void_p * max(n, 1))(*[s.ptr for s in seqs])
    out = ctypes.POINTER(N.Hits)()
    N.check(L.bsq_align_batch(h, ctypes.byref(opts), ptrs, n, first_call, ctypes.byref(out)))
    try:
        return _records(out.contents, n)
    finally:
        L.bsq_hits_free(out)


def _columns(L, h, opts, seqs, first_call):
    """build_tuple_bwa's columns of one fetch through a plain batch (the reference for the pipeline's)."""
    n = len(seqs)
    ptrs = (ctypes.c_void_p * n)(*[s.ptr for s in seqs])
    b = ctypes.c_void_p()
    N.check(L.bsq_batch_create(h, n, sum(len(s) for s in seqs) + 1, ctypes.byref(b)))
    try:
        N.check(L.bsq_batch_set_nuclseqs(b, ptrs, n))
        N.check(L.bsq_batch_run(b, ctypes.byref(opts), first_call))
        nh = L.bsq_batch_hits(b).contents.n_hits
        if nh == 0:
            return b""
        out, oo = ctypes.c_void_p(), ctypes.c_void_p()
        N.check(L.bsq_batch_render_nuclseqs(b, ptrs, ctypes.byref(out), ctypes.byref(oo)))
        off = ctypes.cast(oo, ctypes.POINTER(ctypes.c_int64))
        data = ctypes.string_at(out, off[2 * nh])
        L.bsq_free(out)
        L.bsq_free(oo)
        return data
    finally:
        L.bsq_batch_free(b)


@pytest.fixture(scope="module")
def setup():
    ref = synth.make_reference(1_500_000, n_rows=2, n_run_every=400_000, n_run_len=300, dup_frac=0.02)
    reads = synth.make_reads(ref, 24_000, seed=91)
    pi, oi = build_pair([t.decode() for t in ref.texts()])
    pi.upload()
    seqs = [NucleotideSequence.from_text(reads.text(i)) for i in range(reads.n)]
    return pi, seqs


@pytest.mark.parametrize("slots", [1, 3])
def test_pipeline_fetches_equal_single_calls(setup, slots):
    pi, seqs = setup
    L = N.lib()
    sizes = [5000, 0, 1, 777, 12000, 3, 2219]
    fetches, lo = [], 0
    for s in sizes:
        fetches.append((lo, seqs[lo:lo + s]))
        lo += s
    p = ctypes.c_void_p()
    N.check(L.bsq_pipeline_create(pi.handle, slots, ctypes.byref(p)))
    try:
        pending, got = [], []

        def take():
            v = ctypes.POINTER(N.Hits)()
            c = ctypes.c_void_p()
            o = ctypes.POINTER(ctypes.c_int64)()
            N.check(L.bsq_pipeline_next(p, ctypes.byref(v), ctypes.byref(c), ctypes.byref(o)))
            first, n = pending.pop(0)
            rec = _records(v.contents, n)
            nh = v.contents.n_hits
            cols = ctypes.string_at(c, o[2 * nh]) if nh else b""
            got.append((first, n, rec, cols))
            N.check(L.bsq_pipeline_release(p))

        for first, fs in fetches:
            if len(pending) == slots:
                take()
            # the fetch's varlenas live only until submit returns (the SPI tuple table is freed after it)
            copies = [NucleotideSequence(s.raw) for s in fs]
            ptrs = (ctypes.c_void_p * max(len(fs), 1))(*[s.ptr for s in copies])
            N.check(L.bsq_pipeline_submit(p, ctypes.byref(pi.options), ptrs, len(fs), 500 + first, 1))
            del copies, ptrs
            gc.collect()
            pending.append((first, len(fs)))
        while pending:
            take()
    finally:
        L.bsq_pipeline_free(p)
    assert [g[0] for g in got] == [f[0] for f in fetches]   # submission order
    for (first, fs), (_, n, rec, cols) in zip(fetches, got):
        assert rec == _one_shot(L, pi.handle, pi.options, fs, 500 + first), first
        if fs:
            assert cols == _columns(L, pi.handle, pi.options, fs, 500 + first), first


@pytest.mark.parametrize("slots,run_cap", [(2, None), (4, None), (8, "2"), (6, "1")])
def test_deferred_staging_fetches_equal_single_calls(setup, monkeypatch, slots, run_cap):
    """bsq_pipeline_submit_deferred (the drop-in's cursor loop since round 5, extension_bsq.cpp for_each_fetch_held):
    fetch k is staged by a pipeline worker; the caller frees its varlenas (here: overwrites them with other reads)
    only after submitting fetch k+1 and bsq_pipeline_wait_staged past k's ticket.  Every fetch's rows and columns
    equal aligning it alone, tickets count submissions, and a fetch freed after its wait cannot change its rows.
    With fewer concurrent alignments than slots (BSQ_PIPE_RUN) the slots share run_cap device workspace sets, lent
    per alignment turn to fetches of different sizes (a set sized for 1 read grows for 6,000)."""
    if run_cap:
        monkeypatch.setenv("BSQ_PIPE_RUN", run_cap)
    pi, seqs = setup
    L = N.lib()
    sizes = [4000, 1, 0, 6000, 333, 5000, 2]
    fetches, lo = [], 0
    for s in sizes:
        fetches.append((lo, seqs[lo:lo + s]))
        lo += s
    junk = seqs[-1].raw
    p = ctypes.c_void_p()
    N.check(L.bsq_pipeline_create(pi.handle, slots, ctypes.byref(p)))
    try:
        pending, got, held = [], [], None

        def take():
            v = ctypes.POINTER(N.Hits)()
            c = ctypes.c_void_p()
            o = ctypes.POINTER(ctypes.c_int64)()
            N.check(L.bsq_pipeline_next(p, ctypes.byref(v), ctypes.byref(c), ctypes.byref(o)))
            first, n = pending.pop(0)
            nh = v.contents.n_hits
            got.append((first, n, _records(v.contents, n), ctypes.string_at(c, o[2 * nh]) if nh else b""))
            N.check(L.bsq_pipeline_release(p))

        def free(h):   # "SPI_freetuptable": the buffers now hold another read's bytes
            ticket, bufs, _ptrs = h
            N.check(L.bsq_pipeline_wait_staged(p, ticket + 1))
            for b in bufs:
                ctypes.memmove(b, junk, min(len(junk), ctypes.sizeof(b)))

        for k, (first, fs) in enumerate(fetches):
            if len(pending) == slots:
                take()
            bufs = [ctypes.create_string_buffer(s.raw, len(s.raw)) for s in fs]
            ptrs = (ctypes.c_void_p * max(len(fs), 1))(*[ctypes.addressof(b) for b in bufs])
            tk = ctypes.c_int64(-7)
            N.check(L.bsq_pipeline_submit_deferred(p, ctypes.byref(pi.options), ptrs, len(fs), 900 + first, 1,
                                                   ctypes.byref(tk)))
            assert tk.value == k   # tickets number the submissions
            if held is not None:
                free(held)
            held = (tk.value, bufs, ptrs)   # the pointer array is read by the worker too
            pending.append((first, len(fs)))
        free(held)
        while pending:
            take()
    finally:
        L.bsq_pipeline_free(p)
    assert [g[0] for g in got] == [f[0] for f in fetches]
    for (first, fs), (_, n, rec, cols) in zip(fetches, got):
        assert rec == _one_shot(L, pi.handle, pi.options, fs, 900 + first), first
        if fs:
            assert cols == _columns(L, pi.handle, pi.options, fs, 900 + first), first


def test_pipeline_full_and_empty(setup):
    pi, seqs = setup
    L = N.lib()
    p = ctypes.c_void_p()
    N.check(L.bsq_pipeline_create(pi.handle, 2, ctypes.byref(p)))
    try:
        v = ctypes.POINTER(N.Hits)()
        assert L.bsq_pipeline_next(p, ctypes.byref(v), None, None) == N.BSQ_E_INVALID   # nothing submitted
        ptrs = (ctypes.c_void_p * 10)(*[s.ptr for s in seqs[:10]])
        for k in range(2):
            N.check(L.bsq_pipeline_submit(p, ctypes.byref(pi.options), ptrs, 10, 10 * k, 0))
        assert L.bsq_pipeline_submit(p, ctypes.byref(pi.options), ptrs, 10, 20, 0) == N.BSQ_E_INVALID   # full
        assert b"slot" in L.bsq_last_error()
        N.check(L.bsq_pipeline_next(p, ctypes.byref(v), None, None))
        assert v.contents.n_reads == 10
        # the taken slot is still held: submitting needs its release
        assert L.bsq_pipeline_submit(p, ctypes.byref(pi.options), ptrs, 10, 20, 0) == N.BSQ_E_INVALID
        N.check(L.bsq_pipeline_release(p))
        N.check(L.bsq_pipeline_submit(p, ctypes.byref(pi.options), ptrs, 10, 20, 0))
        bad = N.Opts.from_buffer_copy(pi.options)
        bad.e_del = 0
        N.check(L.bsq_pipeline_next(p, ctypes.byref(v), None, None))
        N.check(L.bsq_pipeline_release(p))
        assert L.bsq_pipeline_submit(p, ctypes.byref(bad), ptrs, 10, 30, 0) == N.BSQ_E_INVALID
    finally:
        L.bsq_pipeline_free(p)   # one submission still on the device: free waits for it



def test_failed_take_behind_a_held_view(setup, monkeypatch):
    """A fetch that fails while an older taken fetch is still held must not free the held slot: the next
    submission would land on it and overwrite the rows the caller is reading.  The failure is
    injected at job 1's staging (BSQ_PIPE_FAILPOINT); a 2-slot pipeline puts job 2 on job 0's slot."""
    pi, seqs = setup
    L = N.lib()
    monkeypatch.setenv("BSQ_PIPE_FAILPOINT", "1")
    ptrs = (ctypes.c_void_p * 50)(*[s.ptr for s in seqs[:50]])
    p = ctypes.c_void_p()
    N.check(L.bsq_pipeline_create(pi.handle, 2, ctypes.byref(p)))
    try:
        N.check(L.bsq_pipeline_submit(p, ctypes.byref(pi.options), ptrs, 50, 0, 0))    # job 0, slot 0
        N.check(L.bsq_pipeline_submit(p, ctypes.byref(pi.options), ptrs, 50, 50, 0))   # job 1, slot 1: fails
        v0 = ctypes.POINTER(N.Hits)()
        N.check(L.bsq_pipeline_next(p, ctypes.byref(v0), None, None))
        before = _records(v0.contents, 50)
        v1 = ctypes.POINTER(N.Hits)()
        assert L.bsq_pipeline_next(p, ctypes.byref(v1), None, None) == N.BSQ_E_INVALID
        assert b"injected" in L.bsq_last_error()
        # slot 0 is still the caller's: job 2 (slot 0 again) is refused and the held rows stay as they were
        other = (ctypes.c_void_p * 25)(*[x.ptr for x in seqs[100:125]])
        assert L.bsq_pipeline_submit(p, ctypes.byref(pi.options), other, 25, 100, 0) == N.BSQ_E_INVALID
        assert _records(v0.contents, 50) == before
        N.check(L.bsq_pipeline_release(p))   # frees slot 0 and, behind it, the failed slot 1
        assert L.bsq_pipeline_release(p) == N.BSQ_E_INVALID
        monkeypatch.delenv("BSQ_PIPE_FAILPOINT")
        N.check(L.bsq_pipeline_submit(p, ctypes.byref(pi.options), ptrs, 50, 0, 0))
        N.check(L.bsq_pipeline_next(p, ctypes.byref(v0), None, None))
        assert _records(v0.contents, 50) == before   # the same fetch aligned again: the same rows
        N.check(L.bsq_pipeline_release(p))
    finally:
        L.bsq_pipeline_free(p)

def test_one_shot_split_does_not_change_rows(setup, monkeypatch):
    """bsq_align_batch over 1 slot vs 4 concurrent slots (24k reads -> shares of >= 32768 reads: one share;
    force small shares through BSQ_PIPE_SLOTS with a larger call): identical records."""
    pi, seqs = setup
    L = N.lib()
    big = seqs * 3   # 72k reads: 3 shares of 24k on a 4-slot pipeline
    monkeypatch.setenv("BSQ_PIPE_SLOTS", "1")
    a = _one_shot(L, pi.handle, pi.options, big, 42)
    # a fresh index object is not needed: the pooled pipeline grows to the requested slots
    monkeypatch.setenv("BSQ_PIPE_SLOTS", "4")
    b = _one_shot(L, pi.handle, pi.options, big, 42)
    assert a == b


def test_large_fetch_threaded_staging(setup):
    """A fetch of >= 65536 reads is staged on several host threads (stage_nuclseqs); its rows and columns must
    equal the same reads aligned as three one-shot shares (each staged on one thread)."""
    pi, seqs = setup
    L = N.lib()
    big = (seqs * 3)[:70001]
    holed = sum(1 for s in big if s.holes_num)
    assert holed > 10   # reads with N exercise the holed-read list of the staging
    p = ctypes.c_void_p()
    N.check(L.bsq_pipeline_create(pi.handle, 1, ctypes.byref(p)))
    try:
        ptrs = (ctypes.c_void_p * len(big))(*[s.ptr for s in big])
        N.check(L.bsq_pipeline_submit(p, ctypes.byref(pi.options), ptrs, len(big), 7, 1))
        v = ctypes.POINTER(N.Hits)()
        c = ctypes.c_void_p()
        o = ctypes.POINTER(ctypes.c_int64)()
        N.check(L.bsq_pipeline_next(p, ctypes.byref(v), ctypes.byref(c), ctypes.byref(o)))
        got = _records(v.contents, len(big))
        nh = v.contents.n_hits
        cols = ctypes.string_at(c, o[2 * nh])
        N.check(L.bsq_pipeline_release(p))
    finally:
        L.bsq_pipeline_free(p)
    assert got == _one_shot(L, pi.handle, pi.options, big, 7)
    assert cols == _columns(L, pi.handle, pi.options, big, 7)
