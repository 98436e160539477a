"""Long reads: reads long enough that mem_flt_chained_seeds is active
(5.5 ln l <= 0.05 l, l >~ 700) -- short seeds re-scored by ksw_align2 (mem_seed_sw) and filtered, chains
ordered by those scores -- align identically to the oracle, alone and mixed with 150 bp reads."""
import pytest

from bioseqdb_amd import synth
from parity_util import build_pair, compare

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pair():
    ref = synth.make_reference(1_000_000, n_rows=2, n_run_every=300_000, n_run_len=500)
    pi, oi = build_pair([t.decode() for t in ref.texts()])
    return ref, pi, oi


@pytest.mark.parametrize("length", [700, 1000, 2000])
def test_long_reads_match_oracle(pair, length):
    ref, pi, oi = pair
    reads = synth.make_reads(ref, 120, length=length, seed=length)
    rows, bad = compare(pi, oi, [reads.text(i) for i in range(reads.n)], first_call=3)
    assert not bad, bad[:5]
    assert rows >= 100


def test_mixed_lengths(pair):
    ref, pi, oi = pair
    a = synth.make_reads(ref, 150, length=150, seed=1)
    b = synth.make_reads(ref, 60, length=1500, seed=2)
    texts = [a.text(i) for i in range(a.n)] + [b.text(i) for i in range(b.n)]
    rows, bad = compare(pi, oi, texts, first_call=11)
    assert not bad, bad[:5]
    assert rows >= 200


def test_seed_filter_runs(pair):
    # the filter's SW cells show up in the chain stage's work counter (zero for 150 bp batches)
    import ctypes
    import numpy as np
    from bioseqdb_amd import _native as N
    ref, pi, _ = pair
    L = N.lib()
    pi.upload()

    def chain_cells(length):
        reads = synth.make_reads(ref, 64, length=length, seed=9)
        b = ctypes.c_void_p()
        N.check(L.bsq_batch_create(pi.handle, reads.n, int(reads.offsets[-1]), ctypes.byref(b)))
        try:
            codes = np.ascontiguousarray(reads.codes)
            offs = np.ascontiguousarray(reads.offsets)
            N.check(L.bsq_batch_set_reads(b, codes.ctypes.data, offs.ctypes.data, reads.n))
            N.check(L.bsq_batch_run(b, ctypes.byref(pi.options), 0))
            w = (ctypes.c_double * 6)()
            L.bsq_batch_stage_work(b, w, 6)
            return w[1]
        finally:
            L.bsq_batch_free(b)

    assert chain_cells(150) == 0
    assert chain_cells(1500) > 0
