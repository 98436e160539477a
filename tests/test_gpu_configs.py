"""GPU parity at BASELINE.json's config sizes and over the bwa_options surface.

* C3 (configs[2]): 100 Mbp synthetic reference, 20k x 150 bp reads, all 14 bwa_result columns of the
  GPU path (bsq_align_batch + bsq_render_tsv) against the CPU oracle, row by row (ref_subseq skipped on
  reverse rows, Q7).  The oracle's FM tables (BWT, occ, L2, sampled SA) are derived on the host from the
  GPU-built suffix array, after the SA has passed two certificates that each prove it is the unique SA of T$:
  the device one (bsq_index_certify_sa) and the oracle's own host check (range, one primary row, adjacent
  suffixes strictly increasing; orc_index_build_from_sa).  The oracle's own suffix sort is too slow at 2e8
  suffixes; the certificates are what keeps a mis-sorted SA from reaching both sides (parity_util).
* C2 (configs[1]): seeding only on the same index, bsq_batch_seed intervals against orc_collect_intv.
* The option matrix: non-default bwa_opts() values, with the Q1 field swap and the Q2 scoring matrix
  that keeps a=1/b=4 while opt->a/opt->b change (bioseqdb/bwa.cpp:80, extension.cpp:220-231).
"""
import ctypes

import numpy as np
import pytest

import oracle_py as O
from bioseqdb_amd import BwaIndex, NucleotideSequence, bwa_opts, effective_opts, synth
from bioseqdb_amd import _native as N
from parity_util import build_pair, compare_batch, oracle_from_device_sa

pytestmark = pytest.mark.gpu


def _seqs(reads):
    return [NucleotideSequence.from_text(reads.text(i)) for i in range(reads.n)]


@pytest.fixture(scope="module")
def c3_pair():
    """The bench's C3 reference (100 Mbp, one row, N runs + segmental duplications) in both indexes."""
    ref = synth.make_reference(100_000_000)
    pi = BwaIndex()
    oi = O.OracleIndex()
    for i, t in enumerate(ref.texts()):
        s = t.decode()
        ns = NucleotideSequence.from_text(s)
        on = O.Nuclseq(s)
        assert ns.raw == on.raw
        pi.add_ref_sequence(i + 1, ns)
        oi.add_ref(i + 1, on.raw)
    pi.build_on_device()
    oracle_from_device_sa(pi, oi, "C3 100 Mbp")
    pi.options = effective_opts(None, len(ref.rows))
    return ref, pi, oi


def test_c3_100mbp_all_columns(c3_pair):
    ref, pi, oi = c3_pair
    reads = synth.make_reads(ref, 20_000, seed=synth.READ_SEED)
    rows, bad = compare_batch(pi, oi, _seqs(reads), first_call=0)
    assert rows > 19_000
    assert not bad, bad[:20]


def test_c3_100mbp_second_call_continues_lrand48(c3_pair):
    """A second cursor batch continues the backend's lrand48 stream (Q10): reads 20000.. of the bench."""
    ref, pi, oi = c3_pair
    reads = synth.make_reads(ref, 5_000, seed=synth.READ_SEED + 1)
    rows, bad = compare_batch(pi, oi, _seqs(reads), first_call=20_000)
    assert rows > 4_500
    assert not bad, bad[:20]


def test_c2_100mbp_seeding(c3_pair):
    ref, pi, oi = c3_pair
    reads = synth.make_reads(ref, 20_000, seed=synth.READ_SEED + 2)
    L = N.lib()
    b = ctypes.c_void_p()
    N.check(L.bsq_batch_create(pi.handle, reads.n, int(reads.offsets[-1]), ctypes.byref(b)))
    try:
        codes = np.ascontiguousarray(reads.codes)
        offs = np.ascontiguousarray(reads.offsets)
        N.check(L.bsq_batch_set_reads(b, codes.ctypes.data, offs.ctypes.data, reads.n))
        N.check(L.bsq_batch_seed(b, ctypes.byref(pi.options)))
        ro = ctypes.POINTER(ctypes.c_int64)()
        iv = ctypes.POINTER(ctypes.c_uint64)()
        nt = ctypes.c_int64()
        N.check(L.bsq_batch_intervals(b, ctypes.byref(ro), ctypes.byref(iv), ctypes.byref(nt)))
        off = np.ctypeslib.as_array(ro, shape=(reads.n + 1,)).copy()
        arr = np.ctypeslib.as_array(iv, shape=(max(int(nt.value), 1) * 4,)).copy()[: int(nt.value) * 4].reshape(-1, 4)
    finally:
        L.bsq_batch_free(b)
    oo = O.opts_from(pi.options)
    bad, total = [], 0
    for r in range(reads.n):
        q = bytes(reads.codes[reads.offsets[r]:reads.offsets[r + 1]])
        exp = [(x0, x2, info) for x0, _x1, x2, info in oi.collect_intv(oo, q)]
        got = [(int(a), int(c), int(d)) for a, _b, c, d in arr[off[r]:off[r + 1]]]
        total += len(exp)
        if got != exp:
            bad.append((r, got[:3], exp[:3]))
    assert total > 20_000
    assert not bad, bad[:5]


@pytest.mark.parametrize("exchange", [0, 1])
def test_c3_100mbp_replicated_group_8(c3_pair, exchange):
    """C5's sharding at the C3 index on the one-GPU box: an 8-member device group (device 0
    listed 8 times: replicas by device-to-device copies), 24,003 reads split into 8 ragged shares, the lrand48
    stream continuing from an earlier call (member k starts at first_call + k*n/8), records over every member's
    link (exchange 0) or gathered in member 0's HBM first (exchange 1), one barrier-free stream of 2 rounds.  Every
    column equals the oracle's rows; the segments come back in member order at the shares' first reads."""
    ref, pi, oi = c3_pair
    from parity_util import _oracle_batch_tsv, compare_tsv
    reads = synth.make_reads(ref, 24_003, seed=synth.READ_SEED + 11)
    seqs = _seqs(reads)
    n = len(seqs)
    G = 8
    ptrs = (ctypes.c_void_p * n)(*[s.ptr for s in seqs])
    L = N.lib()
    g = ctypes.c_void_p()
    N.check(L.bsq_group_create((ctypes.c_int * G)(*([0] * G)), G, ctypes.byref(g)))
    try:
        N.check(L.bsq_group_set_exchange(g, exchange))
        N.check(L.bsq_group_replicate(g, pi.handle, None))
        first_call = 40_000
        N.check(L.bsq_group_run(g, ctypes.byref(pi.options), ptrs, n, first_call))
        N.check(L.bsq_group_run_rounds(g, ctypes.byref(pi.options), n, first_call, 2))
        segs = (ctypes.POINTER(N.Hits) * 64)()
        slo = (ctypes.c_int32 * 64)()
        ns = L.bsq_group_segments(g, segs, slo, 64)
        lo = [k * n // G for k in range(G)]
        assert ns >= G and sorted(set(slo[:ns])) == list(slo[:ns]) and set(lo) <= set(slo[:ns]), list(slo[:ns])
        assert sum(segs[i].contents.n_reads for i in range(ns)) == n
        H = L.bsq_group_hits(g)
        p = L.bsq_render_tsv(pi.handle, H, ptrs)
        text = ctypes.string_at(p).decode("latin-1")
        L.bsq_free(p)
        counts = [H.contents.read_off[i + 1] - H.contents.read_off[i] for i in range(n)]
    finally:
        L.bsq_group_free(g)
    exp, ec = _oracle_batch_tsv(oi, O.opts_from(pi.options), [s.raw for s in seqs], first_call)
    rows, bad = compare_tsv(text, counts, exp, ec)
    assert rows > 22_000
    assert not bad, bad[:20]


# ---- the bwa_options surface (bwa_opts() arguments, Q1 applied by bwa_opts) -------------------------
OPTION_SETS = {
    "q2_match2_mismatch3": dict(match_score=2, mismatch_penalty=3),
    "band10_zdrop20": dict(bandwidth=10, zdrop=20),
    "band50": dict(bandwidth=50),
    "band0_zdrop0": dict(bandwidth=0, zdrop=0),
    "clip0": dict(pen_clip3=0, pen_clip5=0),
    "clip100": dict(pen_clip3=100, pen_clip5=100),
    "clip_asym": dict(pen_clip3=1, pen_clip5=40),
    "seed15": dict(min_seed_len=15),
    "seed31": dict(min_seed_len=31),
    "max_occ5": dict(max_occ=5),
    "max_occ37": dict(max_occ=37),
    "gaps_swapped": dict(o_ins=3, e_del=2),              # Q1: e_del <- 3, o_ins <- 2
    "gaps_cheap": dict(o_del=1, o_ins=1, e_del=1, e_ins=1),
    "gaps_dear": dict(o_del=20, o_ins=15, e_del=4, e_ins=7),
    "match0": dict(match_score=0),
    "mismatch0": dict(mismatch_penalty=0),
    "match200_global_rows": dict(match_score=200),       # beyond the u16 LDS row bound: k_extend<false>
    "seed_len0": dict(min_seed_len=0),
}


@pytest.fixture(scope="module")
def opt_pair():
    ref = synth.make_reference(2_000_000, n_rows=2, n_run_every=700_000, n_run_len=300, dup_frac=0.03)
    pi, oi = build_pair([t.decode() for t in ref.texts()])
    return ref, pi, oi


@pytest.mark.parametrize("name", sorted(OPTION_SETS))
def test_option_matrix(opt_pair, name):
    ref, pi, oi = opt_pair
    o = effective_opts(bwa_opts(**OPTION_SETS[name]), len(ref.rows))
    reads = synth.make_reads(ref, 2_000, seed=101 + sorted(OPTION_SETS).index(name))
    rows, bad = compare_batch(pi, oi, _seqs(reads), first_call=31, opts=o)
    assert rows > 1_000
    assert not bad, bad[:20]


def test_option_q1_swap_is_applied():
    o = effective_opts(bwa_opts(o_del=7, o_ins=3, e_del=2, e_ins=5), 1)
    assert (o.o_del, o.e_del, o.o_ins, o.e_ins) == (7, 3, 2, 5)
