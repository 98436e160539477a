"""The Postgres-side drop-in (bioseqdb_amd/pg/extension_bsq.cpp over bwa_bsq.cpp and libbsq) compiled against
the stub Postgres API in tests/pgstub and driven by its fake executor, the way the server calls
nuclseq_search_bwa / nuclseq_multi_search_bwa (extension.cpp:311-378).

CPU tests: the SQL-visible error behaviour (messages and SQLSTATEs of extension.cpp:173,177,206,240-262), the
option handling, NULL skipping, an empty reference, interrupts, and that no error longjmps over C++ objects
(no palloc'd memory or index left behind).  GPU tests: every bwa_result column of the rows against the CPU
oracle, through several SPI fetches, the index cache, the lrand48 stream across calls and non-default options."""
import ctypes
import os
import subprocess

import pytest

import oracle_py as O
from bioseqdb_amd import NucleotideSequence, bwa_opts, synth
from bioseqdb_amd import bwa as B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INT2, INT4, INT8, TEXT = 21, 23, 20, 25
OPT_FIELDS = ("min_seed_len", "max_occ", "match_score", "mismatch_penalty", "pen_clip3", "pen_clip5", "zdrop",
              "bandwidth", "o_del", "e_del", "o_ins", "e_ins")


class StubOpts(ctypes.Structure):
    _fields_ = [("values", ctypes.c_int32 * 12), ("nulls", ctypes.c_uint8 * 12)]


def _opts(o=None):
    o = o or bwa_opts()
    s = StubOpts()
    for i, f in enumerate(OPT_FIELDS):
        v = getattr(o, f)
        s.values[i] = 0 if v is None else v
        s.nulls[i] = v is None
    return s


@pytest.fixture(scope="module")
def stub(tmp_path_factory):
    out = tmp_path_factory.mktemp("pgstub") / "libpgstub_ext.so"
    libdir = os.path.join(ROOT, "bioseqdb_amd")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-shared", "-fPIC", "-Wall", "-Werror", "-Wno-unused-parameter",
                    f"-I{ROOT}/tests/pgstub/include", f"-I{ROOT}/include", f"-I{ROOT}/bioseqdb_amd/pg",
                    f"{ROOT}/bioseqdb_amd/pg/extension_bsq.cpp", f"{ROOT}/bioseqdb_amd/pg/bwa_bsq.cpp",
                    f"{ROOT}/tests/pgstub/pgstub.cpp", f"-L{libdir}", "-lbsq", f"-Wl,-rpath,{libdir}", "-o", str(out)],
                   check=True)
    L = ctypes.CDLL(str(out))
    L.pgstub_call.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_char_p,
                              ctypes.POINTER(StubOpts), ctypes.POINTER(ctypes.c_void_p), ctypes.c_char_p,
                              ctypes.POINTER(ctypes.c_void_p)]
    L.pgstub_add_table.argtypes = [ctypes.c_char_p, ctypes.c_uint, ctypes.c_uint]
    L.pgstub_add_row.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64,
                                 ctypes.c_int]
    L.pgstub_nuclseq_oid.restype = ctypes.c_uint
    L.pgstub_last_debug.restype = ctypes.c_char_p
    L.pgstub_live_allocs.restype = ctypes.c_long
    L.pgstub_index_cache_hits.restype = ctypes.c_long
    L.pgstub_index_cache_builds.restype = ctypes.c_long
    L.pgstub_set_lrand48_calls.argtypes = [ctypes.c_uint64]
    L.pgstub_lrand48_calls.restype = ctypes.c_uint64
    return L


class Db:
    """Tables of the fake executor plus a call wrapper."""

    def __init__(self, L):
        self.L = L
        L.pgstub_reset()
        L.pgstub_clear_index_cache()
        self.ns_oid = L.pgstub_nuclseq_oid()

    def table(self, sql, rows, id_type=INT8, seq_type=None):
        self.L.pgstub_add_table(sql.encode(), id_type, self.ns_oid if seq_type is None else seq_type)
        for rid, seq in rows:
            raw = seq.raw if seq is not None else b""
            self.L.pgstub_add_row(sql.encode(), rid or 0, rid is None, raw, len(raw), seq is None)

    def call(self, query, ref_sql, opts=None):
        """query: SQL text (multi search) or a NucleotideSequence (single search)."""
        rows = ctypes.c_void_p()
        msg = ctypes.c_void_p()
        state = ctypes.create_string_buffer(6)
        multi = isinstance(query, str)
        qbuf = None if multi else ctypes.create_string_buffer(query.raw, len(query.raw))
        rc = self.L.pgstub_call(int(multi), query.encode() if multi else None,
                                None if multi else ctypes.addressof(qbuf), ref_sql.encode(),
                                ctypes.byref(_opts(opts)), ctypes.byref(rows), state, ctypes.byref(msg))
        libc = ctypes.CDLL(None)
        libc.free.argtypes = [ctypes.c_void_p]
        if rc:
            m = ctypes.string_at(msg.value).decode()
            libc.free(msg)
            return None, (state.value.decode(), m)
        text = ctypes.string_at(rows.value).decode()
        libc.free(rows)
        return [ln.split("\t") for ln in text.splitlines()], None


def _ns(t):
    return NucleotideSequence.from_text(t)


# ---- CPU: errors and plumbing --------------------------------------------------------------------------

def test_set_returning_checks(stub):
    db = Db(stub)
    db.table("refs", [(1, _ns("ACGT" * 30))])
    db.table("reads", [(1, _ns("ACGT" * 10))])
    stub.pgstub_set_rsi_null(1)
    assert db.call("reads", "refs")[1] == ("0A000", "set-valued function called in context that cannot accept a set")
    stub.pgstub_set_rsi_null(0)
    stub.pgstub_set_allowed_modes(1)   # SFRM_ValuePerCall only
    assert db.call("reads", "refs")[1] == ("0A000", "materialize mode required, but it is not allowed in this context")
    stub.pgstub_set_allowed_modes(2)
    stub.pgstub_set_result_class(3)    # TYPEFUNC_RECORD
    assert db.call("reads", "refs")[1] == (
        "0A000", "function returning record called in context that cannot accept type record")
    stub.pgstub_set_result_class(0)    # TYPEFUNC_SCALAR
    assert db.call("reads", "refs")[1] == ("0A000", "return type must be a row type")
    assert stub.pgstub_live_allocs() == 0


def test_cursor_type_checks(stub):
    db = Db(stub)
    db.table("refs_text_ids", [(1, _ns("ACGT" * 30))], id_type=TEXT)
    db.table("refs_bad_seq", [(1, _ns("ACGT" * 30))], seq_type=TEXT)
    db.table("reads", [(1, _ns("ACGT" * 10))])
    assert db.call("reads", "refs_text_ids")[1] == ("42804", "expected column of integers")
    assert db.call("reads", "refs_bad_seq")[1] == ("42804", "expected column of nuclseqs")
    err = db.call("reads", "no such table")[1]
    assert err[0] == "42601" and "no such table" in err[1]   # a Postgres error passes through unchanged


def test_option_errors_in_reference_order(stub):
    db = Db(stub)
    db.table("refs", [(1, _ns("ACGT" * 30))])
    db.table("reads", [(1, _ns("ACGT" * 10))])
    assert db.call("reads", "refs", bwa_opts(zdrop=-1))[1] == ("22023", "bwa_opt zdrop must be nonnegative")
    # get_opt_or runs max_occ, min_seed_len, match_score, ... (extension.cpp:220-231): the first one wins
    assert db.call("reads", "refs", bwa_opts(e_ins=-2, min_seed_len=-1))[1] == (
        "22023", "bwa_opt min_seed_len must be nonnegative")
    # Q1: bwa_opts(o_ins=...) lands in e_del; e_del = 0 is a divisor of the reference (documented divergence)
    assert db.call("reads", "refs", bwa_opts(o_ins=0))[1] == ("22023", "bwa_opt e_del must be positive")
    assert db.call("reads", "refs", bwa_opts(max_occ=0))[1] == ("22023", "bwa_opt max_occ must be positive")
    assert stub.pgstub_live_allocs() == 0


def test_empty_reference_gives_no_rows(stub):
    db = Db(stub)
    db.table("no_refs", [(None, _ns("ACGT" * 8)), (4, None)])   # every row NULL: skipped
    db.table("reads", [(1, _ns("ACGT" * 10)), (2, _ns("GGCA" * 10))])
    stub.pgstub_set_lrand48_calls(9)
    assert db.call("reads", "no_refs") == ([], None)
    assert db.call(_ns("ACGT" * 10), "no_refs") == ([], None)
    assert stub.pgstub_lrand48_calls() == 9   # bwa.cpp:142-143: no mem_align1, no lrand48 draw
    assert b"0 reference rows" in stub.pgstub_last_debug()


def test_interrupt_and_no_device_release_everything(stub, gpu_available):
    db = Db(stub)
    db.table("refs", [(1, _ns("ACGTTGCA" * 400))])
    db.table("reads", [(i, _ns("ACGTTGCA" * 5)) for i in range(10)])
    stub.pgstub_cancel_after(1)   # the reference cursor's first fetch passes, the next check cancels
    assert db.call("reads", "refs")[1] == ("57014", "canceling statement due to user request")
    assert stub.pgstub_live_allocs() == 0
    stub.pgstub_cancel_after(-1)
    if not gpu_available:   # libbsq has no CPU fallback: a libbsq error, raised after cleanup
        state, msg = db.call("reads", "refs")[1]
        assert state == "38000" and msg.startswith("libbsq: ")
        assert stub.pgstub_live_allocs() == 0


# ---- GPU: rows against the oracle ---------------------------------------------------------------

def _expected(oi, n_refs, opts, reads, first_call, with_id=True):
    oo = O.opts_from(B.effective_opts(opts, n_refs))
    out, k = [], first_call
    for qid, seq in reads:
        if qid is None or seq is None:
            continue
        for m in B.parse_tsv(oi.align_tsv(oo, seq.raw, O.lrand48_at(k))):
            out.append((m, qid if with_id else None))
        k += 1
    return out, k


def _check_rows(got, exp):
    assert len(got) == len(exp), (len(got), len(exp))
    bad = []
    for g, (m, qid) in zip(got, exp):
        want = [str(m.ref_id), None if m.is_reverse else m.ref_subseq, str(m.ref_match_begin), str(m.ref_match_end),
                str(m.ref_match_len), "\\N" if qid is None else str(qid), m.query_subseq, str(m.query_match_begin),
                str(m.query_match_end), str(m.query_match_len), "tf"[not m.is_primary], "tf"[not m.is_secondary],
                "tf"[not m.is_reverse], m.cigar, str(m.score)]
        for j, w in enumerate(want):
            if w is not None and g[j] != w:
                bad.append((B.BWA_RESULT_COLUMNS[j], g[j][:40], w[:40]))
        # the nuclseq columns are nuclseq_from_text of their texts (build_tuple_bwa), byte for byte
        for j, fp in ((1, g[15]), (6, g[16])):
            raw = O.Nuclseq(g[j]).raw
            h = 0xcbf29ce484222325
            for byte in raw:
                h = ((h ^ byte) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
            if f"{h:016x}" != fp:
                bad.append((B.BWA_RESULT_COLUMNS[j], "varlena bytes", fp))
    assert not bad, bad[:10]


@pytest.fixture(scope="module")
def world():
    ref = synth.make_reference(400_000, n_rows=3, n_run_every=150_000, n_run_len=120, dup_frac=0.02)
    texts = [t.decode() for t in ref.texts()]
    ref_rows = [(7, _ns(texts[0])), (None, _ns("ACGT" * 40)), (-3, _ns(texts[1])), (5, None), (2 ** 33, _ns(texts[2]))]
    oi = O.OracleIndex()
    for rid, s in ref_rows:
        if rid is not None and s is not None:
            oi.add_ref(rid, s.raw)
    oi.build()
    reads = synth.make_reads(ref, 1200, seed=19)
    q = []
    for i in range(reads.n):
        s = _ns(reads.text(i))
        q.append((100 + i, s))
        if i % 37 == 0:
            q.append((None, s))
        if i % 41 == 0:
            q.append((900000 + i, None))
    return ref_rows, oi, q


@pytest.mark.gpu
def test_multi_search_rows_fetches_cache_and_lrand48(stub, world, monkeypatch):
    ref_rows, oi, q = world
    db = Db(stub)
    db.table("SELECT id, seq FROM refs", ref_rows)
    db.table("SELECT id, seq FROM reads", q[:700])
    db.table("SELECT id, seq FROM reads2", q[700:])
    monkeypatch.setenv("BSQ_FETCH_ROWS", "173")   # several SPI fetches per call
    stub.pgstub_set_lrand48_calls(0)
    got, err = db.call("SELECT id, seq FROM reads", "SELECT id, seq FROM refs")
    assert err is None, err
    exp, k = _expected(oi, 3, None, q[:700], 0)
    _check_rows(got, exp)
    assert stub.pgstub_lrand48_calls() == k
    got2, err = db.call("SELECT id, seq FROM reads2", "SELECT id, seq FROM refs")
    assert err is None, err
    exp2, k2 = _expected(oi, 3, None, q[700:], k)
    _check_rows(got2, exp2)
    assert stub.pgstub_index_cache_builds() == 1 and stub.pgstub_index_cache_hits() == 1
    assert stub.pgstub_lrand48_calls() == k2
    assert stub.pgstub_live_allocs() == 0


@pytest.mark.gpu
def test_multi_search_int2_ids_and_options(stub, world):
    ref_rows, oi, q = world
    db = Db(stub)
    small = [(i % 30000 if i is not None else None, s) for i, s in q[:500]]
    db.table("refs", ref_rows)
    db.table("reads", small, id_type=INT2)
    opts = bwa_opts(match_score=2, mismatch_penalty=3, bandwidth=20, zdrop=40, o_ins=3, e_del=2, pen_clip5=1,
                    min_seed_len=17, max_occ=80)
    stub.pgstub_set_lrand48_calls(4242)
    got, err = db.call("reads", "refs", opts)
    assert err is None, err
    exp, _ = _expected(oi, 3, opts, small, 4242)
    _check_rows(got, exp)


@pytest.mark.gpu
def test_single_search_query_id_null(stub, world):
    ref_rows, oi, q = world
    db = Db(stub)
    db.table("refs", ref_rows)
    stub.pgstub_set_lrand48_calls(77)
    k = 77
    for _qid, s in [x for x in q[:60] if x[0] is not None and x[1] is not None]:
        got, err = db.call(s, "refs")
        assert err is None, err
        exp, k = _expected(oi, 3, None, [(0, s)], k, with_id=False)
        _check_rows(got, exp)
    assert stub.pgstub_lrand48_calls() == k
    assert stub.pgstub_index_cache_builds() == 1


@pytest.mark.gpu
def test_multi_search_over_a_device_group(stub, world, monkeypatch):
    """BSQ_DEVICES lists several GPUs: each SPI fetch is aligned over a bsq_group (index broadcast once, reads
    sharded over the members, rows merged in read order).  The box has one GPU, so the group holds three
    replicas on it; rows, nuclseq columns and the lrand48 stream must not change."""
    ref_rows, oi, q = world
    db = Db(stub)
    db.table("refs", ref_rows)
    db.table("reads", q[:900])
    monkeypatch.setenv("BSQ_DEVICES", "0,0,0")
    monkeypatch.setenv("BSQ_FETCH_ROWS", "301")
    stub.pgstub_set_lrand48_calls(99)
    got, err = db.call("reads", "refs")
    assert err is None, err
    exp, k = _expected(oi, 3, None, q[:900], 99)
    _check_rows(got, exp)
    assert stub.pgstub_lrand48_calls() == k
    assert stub.pgstub_live_allocs() == 0
