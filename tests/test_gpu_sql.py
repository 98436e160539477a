"""The SQL-level functions end to end on the GPU (extension.cpp:311-378 through bioseqdb_amd.bwa):
nuclseq_multi_search_bwa and nuclseq_search_bwa rows against the oracle's, with query_id, NULL rows
skipped by the cursor (Q14), options through bwa_opts() (Q1/Q2), and the backend's lrand48 stream
continuing across calls (Q10) and across the cross-call index cache."""
import random

import pytest

import oracle_py as O
from bioseqdb_amd import NucleotideSequence, bwa_opts, synth
from bioseqdb_amd import bwa as B

pytestmark = pytest.mark.gpu

COLS = B.BWA_RESULT_COLUMNS


def _oracle_rows(oi, n_refs, opts, reads, first_call):
    """(query_id, nuclseq) rows -> expected bwa_result tuples; lrand48 call k for the k-th aligned read."""
    oo = O.opts_from(B.effective_opts(opts, n_refs))
    out = []
    k = first_call
    for qid, seq in reads:
        if qid is None or seq is None:
            continue
        for m in B.parse_tsv(oi.align_tsv(oo, seq.raw, O.lrand48_at(k))):
            out.append(B._rows(qid, [m])[0])
        k += 1
    return out, k


def _same(got, exp):
    bad = []
    if len(got) != len(exp):
        return [("n_rows", len(got), len(exp))]
    for r, (g, e) in enumerate(zip(got, exp)):
        for j, c in enumerate(COLS):
            if c == "ref_subseq" and e[12]:   # Q7: reverse rows
                continue
            if g[j] != e[j]:
                bad.append((r, c, g[j], e[j]))
    return bad


@pytest.fixture(scope="module")
def sql_world():
    rng = random.Random(77)
    ref = synth.make_reference(600_000, n_rows=3, n_run_every=200_000, n_run_len=150, dup_frac=0.02)
    texts = [t.decode() for t in ref.texts()]
    ref_rows = [(10, NucleotideSequence.from_text(texts[0])), (None, NucleotideSequence.from_text("ACGT" * 50)),
                (-7, NucleotideSequence.from_text(texts[1])), (3, None), (2 ** 35, NucleotideSequence.from_text(texts[2]))]
    oi = O.OracleIndex()
    n_refs = 0
    for rid, s in ref_rows:
        if rid is not None and s is not None:
            oi.add_ref(rid, s.raw)
            n_refs += 1
    oi.build()
    reads = synth.make_reads(ref, 900, seed=5)
    q = []
    for i in range(reads.n):
        s = NucleotideSequence.from_text(reads.text(i))
        q.append((1000 + i, s))
        if rng.random() < 0.03:
            q.append((None, s))          # NULL id: skipped, consumes no lrand48 value
        if rng.random() < 0.03:
            q.append((2000 + i, None))   # NULL sequence: skipped
    return ref_rows, oi, n_refs, q


def test_multi_search_rows_and_lrand48_across_calls(sql_world):
    ref_rows, oi, n_refs, q = sql_world
    B.INDEX_CACHE.clear()
    B.reset_lrand48(0)
    got1 = B.nuclseq_multi_search_bwa(q[:500], ref_rows)
    exp1, k = _oracle_rows(oi, n_refs, None, q[:500], 0)
    assert B.lrand48_calls() == k
    assert len(got1) > 400
    assert not _same(got1, exp1), _same(got1, exp1)[:10]
    got2 = B.nuclseq_multi_search_bwa(q[500:], ref_rows, batch_reads=97)   # several GPU batches
    exp2, k2 = _oracle_rows(oi, n_refs, None, q[500:], k)
    assert B.INDEX_CACHE.hits == 1 and B.INDEX_CACHE.builds == 1
    assert B.lrand48_calls() == k2
    assert not _same(got2, exp2), _same(got2, exp2)[:10]


def test_search_single_query_id_null(sql_world):
    ref_rows, oi, n_refs, q = sql_world
    B.reset_lrand48(12345)
    seqs = [s for qid, s in q[:40] if qid is not None and s is not None]
    k = 12345
    for s in seqs:
        got = B.nuclseq_search_bwa(s, ref_rows)
        exp, k = _oracle_rows(oi, n_refs, None, [(0, s)], k)
        exp = [e[:5] + (None,) + e[6:] for e in exp]   # build_tuple_bwa(std::nullopt, ...): query_id NULL
        assert all(g[5] is None for g in got)
        assert not _same(got, exp)
    assert B.lrand48_calls() == 12345 + len(seqs)


def test_multi_search_with_options(sql_world):
    ref_rows, oi, n_refs, q = sql_world
    opts = bwa_opts(match_score=2, mismatch_penalty=3, bandwidth=30, o_ins=4, e_del=2, max_occ=50, min_seed_len=17)
    B.reset_lrand48(777)
    got = B.nuclseq_multi_search_bwa(q[:400], ref_rows, opts)
    exp, k = _oracle_rows(oi, n_refs, opts, q[:400], 777)
    assert B.lrand48_calls() == k
    assert not _same(got, exp), _same(got, exp)[:10]


def test_empty_reference_consumes_nothing(sql_world):
    _ref_rows, _oi, _n, q = sql_world
    B.reset_lrand48(5)
    assert B.nuclseq_multi_search_bwa(q[:50], [(1, None), (None, NucleotideSequence.from_text("ACGT"))]) == []
    assert B.lrand48_calls() == 5   # bwa.cpp:142-143 returns before mem_align1
