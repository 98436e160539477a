"""bsq_batch_run_many (bench.py's default: 3 batches per GPU): S batches over contiguous read ranges, run
concurrently on their own streams and host threads, give exactly the records of one batch over all the
reads, with each batch's lrand48 position continuing where the previous range ends (Q10)."""
import ctypes

import numpy as np
import pytest

from bioseqdb_amd import _native as N
from bioseqdb_amd import synth
from parity_util import build_pair

pytestmark = pytest.mark.gpu


def _rows(L, b, base):
    H = L.bsq_batch_hits(b).contents
    out = []
    for k in range(H.n_hits):
        x = H.hits[k]
        cig = tuple(H.cigar[x.cigar_off + c] for c in range(x.n_cigar))
        out.append((x.read_index + base, x.ref_id, x.rb, x.re, x.qb, x.qe, x.score, x.is_primary, x.is_secondary,
                    x.is_reverse, cig))
    return out


def _batch(L, pi, reads, keep):
    b = ctypes.c_void_p()
    N.check(L.bsq_batch_create(pi.handle, reads.n, int(reads.offsets[-1]), ctypes.byref(b)))
    codes = np.ascontiguousarray(reads.codes)
    offs = np.ascontiguousarray(reads.offsets)
    keep += [codes, offs]
    N.check(L.bsq_batch_set_reads(b, codes.ctypes.data, offs.ctypes.data, reads.n))
    return b


@pytest.mark.parametrize("S", [2, 3, 5])
def test_run_many_equals_one_batch(S):
    ref = synth.make_reference(1_000_000, n_rows=2, n_run_every=250_000, n_run_len=300, dup_frac=0.02)
    reads = synth.make_reads(ref, 6000, seed=41)
    pi, _ = build_pair([t.decode() for t in ref.texts()])
    pi.upload()
    L = N.lib()
    keep = []
    first = 17
    whole = _batch(L, pi, reads, keep)
    lo = [reads.n * k // S for k in range(S + 1)]
    subs = [_batch(L, pi, reads.subset(lo[k], lo[k + 1]), keep) for k in range(S)]
    try:
        N.check(L.bsq_batch_run(whole, ctypes.byref(pi.options), first))
        exp = _rows(L, whole, 0)
        arr = (ctypes.c_void_p * S)(*[b.value for b in subs])
        fc = (ctypes.c_uint64 * S)(*[first + lo[k] for k in range(S)])
        for _ in range(2):   # a second round on the same batches (buffers reused) gives the same rows
            N.check(L.bsq_batch_run_many(arr, S, ctypes.byref(pi.options), fc))
            got = [r for k in range(S) for r in _rows(L, subs[k], lo[k])]
            assert len(got) == len(exp) and len(exp) > 5000
            assert got == exp
        # bench.py's timed steps: three rounds with no barrier between them end with the same rows
        N.check(L.bsq_batch_run_rounds(arr, S, ctypes.byref(pi.options), fc, 3))
        assert [r for k in range(S) for r in _rows(L, subs[k], lo[k])] == exp
    finally:
        L.bsq_batch_free(whole)
        for b in subs:
            L.bsq_batch_free(b)


def test_one_shot_calls_concurrent_and_repeated():
    """bsq_align_batch from several host threads on one index (one takes the index's pooled batch, the
    others batches of their own) and repeated calls of different sizes give the same rows."""
    import threading
    from bioseqdb_amd import NucleotideSequence
    ref = synth.make_reference(500_000, n_rows=1, n_run_every=200_000, n_run_len=300)
    reads = synth.make_reads(ref, 3000, seed=43)
    pi, _ = build_pair([t.decode() for t in ref.texts()])
    seqs = [NucleotideSequence.from_text(reads.text(i)) for i in range(reads.n)]
    exp = pi.align_sequences(seqs, pi.options, first_call=0)
    assert pi.align_sequences(seqs[:10], pi.options, first_call=0) == exp[:10]   # smaller call, pooled batch
    assert pi.align_sequences(seqs, pi.options, first_call=0) == exp             # and back to the full size
    got = [None] * 4

    def run(k):
        got[k] = pi.align_sequences(seqs, pi.options, first_call=0)

    th = [threading.Thread(target=run, args=(k,)) for k in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert all(g == exp for g in got)
