"""One process driving a group of devices (bsq_group_*): the Postgres backend's multi-GPU
form of nuclseq_multi_search_bwa (extension.cpp:362-370 spread over the members).  The rows of a group run
must equal one device aligning all reads in order -- read order, lrand48 positions (Q10), CIGAR offsets --
and the oracle's rows.  The box has one GPU: a group listing device 0 once uses RCCL (ncclCommInitAll of
one rank), a group listing it several times holds replicas on that GPU (device-to-device copies), which
exercises the sharding, per-member runs and the merge."""
import ctypes

import pytest

import oracle_py as O
from bioseqdb_amd import NucleotideSequence, synth
from bioseqdb_amd import _native as N
from parity_util import _oracle_batch_tsv, build_pair, compare_tsv

pytestmark = pytest.mark.gpu


def _records(H, n):
    hits = ctypes.string_at(H.hits, H.n_hits * ctypes.sizeof(N.Hit)) if H.n_hits else b""
    cig = ctypes.string_at(H.cigar, H.n_cigar * 4) if H.n_cigar else b""
    off = ctypes.string_at(H.read_off, (n + 1) * 8)
    return hits, cig, off


def _one_device(L, h, opts, ptrs, n, first_call):
    out = ctypes.POINTER(N.Hits)()
    N.check(L.bsq_align_batch(h, ctypes.byref(opts), ptrs, n, first_call, ctypes.byref(out)))
    try:
        return _records(out.contents, n)
    finally:
        L.bsq_hits_free(out)


def _varlenas(buf, off, n):
    return [ctypes.string_at(buf.value + off[i], off[i + 1] - off[i])[:int.from_bytes(
        ctypes.string_at(buf.value + off[i], 4), "little") >> 2] for i in range(n)]


@pytest.fixture(scope="module")
def setup():
    ref = synth.make_reference(800_000, n_rows=3, n_run_every=250_000, n_run_len=400)
    reads = synth.make_reads(ref, 3001, seed=77)
    pi, oi = build_pair([t.decode() for t in ref.texts()])
    pi.upload()
    seqs = [NucleotideSequence.from_text(reads.text(i)) for i in range(reads.n)]
    return pi, oi, seqs


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_group_rows_equal_one_device(setup, devices):
    pi, oi, seqs = setup
    L = N.lib()
    n = len(seqs)
    ptrs = (ctypes.c_void_p * n)(*[s.ptr for s in seqs])
    first_call = 1234
    want = _one_device(L, pi.handle, pi.options, ptrs, n, first_call)
    g = ctypes.c_void_p()
    N.check(L.bsq_group_create((ctypes.c_int * len(devices))(*devices), len(devices), ctypes.byref(g)))
    try:
        assert L.bsq_group_size(g) == len(devices)
        ms = ctypes.c_double()
        N.check(L.bsq_group_replicate(g, pi.handle, ctypes.byref(ms)))
        N.check(L.bsq_group_run(g, ctypes.byref(pi.options), ptrs, n, first_call))
        got = _records(L.bsq_group_hits(g).contents, n)
        assert got[2] == want[2], "read offsets differ"
        assert got[1] == want[1], "CIGAR arenas differ"
        assert got[0] == want[0], "hit records differ"
        # the staged reads re-run (bench-style) give the same rows
        N.check(L.bsq_group_run(g, ctypes.byref(pi.options), None, n, first_call))
        assert _records(L.bsq_group_hits(g).contents, n) == want
        # and they are the oracle's rows
        p = L.bsq_render_tsv(pi.handle, L.bsq_group_hits(g), ptrs)
        text = ctypes.string_at(p).decode("latin-1")
        L.bsq_free(p)
        H = L.bsq_group_hits(g).contents
        counts = [H.read_off[i + 1] - H.read_off[i] for i in range(n)]
        exp, ec = _oracle_batch_tsv(oi, O.opts_from(pi.options), [s.raw for s in seqs], first_call)
        rows, bad = compare_tsv(text, counts, exp, ec)
        assert rows > 2500 and not bad, bad[:5]
    finally:
        L.bsq_group_free(g)



@pytest.mark.parametrize("devices,slots,exchange", [([0], 1, 0), ([0, 0], 1, 1), ([0, 0, 0], 4, 1), ([0, 0], 4, 0)])
def test_group_rounds_and_exchange_routes(setup, devices, slots, exchange):
    """bsq_group_run_rounds (the bench's barrier-free stream of rounds: one share per slot streams, fewer shares
    than slots run whole rounds) and the gather-to-member-0 exchange (BSQ_XCHG_VIA_FIRST: records by peer DMA into
    member 0's HBM, then its link) give the rows of one device aligning all reads."""
    pi, _, seqs = setup
    L = N.lib()
    n = len(seqs)
    ptrs = (ctypes.c_void_p * n)(*[s.ptr for s in seqs])
    want = _one_device(L, pi.handle, pi.options, ptrs, n, 99)
    g = ctypes.c_void_p()
    N.check(L.bsq_group_create((ctypes.c_int * len(devices))(*devices), len(devices), ctypes.byref(g)))
    try:
        N.check(L.bsq_group_set_slots(g, slots))
        N.check(L.bsq_group_set_exchange(g, exchange))
        N.check(L.bsq_group_replicate(g, pi.handle, None))
        N.check(L.bsq_group_run(g, ctypes.byref(pi.options), ptrs, n, 99))
        assert _records(L.bsq_group_hits(g).contents, n) == want
        for rounds in (1, 3):
            N.check(L.bsq_group_run_rounds(g, ctypes.byref(pi.options), n, 99, rounds))
            assert _records(L.bsq_group_hits(g).contents, n) == want, rounds
        N.check(L.bsq_group_set_exchange(g, 1 - exchange))   # switched between runs
        N.check(L.bsq_group_run_rounds(g, ctypes.byref(pi.options), n, 99, 2))
        assert _records(L.bsq_group_hits(g).contents, n) == want
        assert L.bsq_group_run_rounds(g, ctypes.byref(pi.options), n + 1, 99, 2) == N.BSQ_E_INVALID
        assert L.bsq_group_set_exchange(g, 7) == N.BSQ_E_INVALID
    finally:
        L.bsq_group_free(g)

def test_group_nuclseq_columns(setup):
    """build_tuple_bwa's two nuclseq columns rendered per member equal one batch's."""
    pi, _, seqs = setup
    L = N.lib()
    n = len(seqs)
    ptrs = (ctypes.c_void_p * n)(*[s.ptr for s in seqs])
    b = ctypes.c_void_p()
    N.check(L.bsq_batch_create(pi.handle, n, sum(len(s) for s in seqs), ctypes.byref(b)))
    g = ctypes.c_void_p()
    N.check(L.bsq_group_create((ctypes.c_int * 2)(0, 0), 2, ctypes.byref(g)))
    try:
        N.check(L.bsq_batch_set_nuclseqs(b, ptrs, n))
        N.check(L.bsq_batch_run(b, ctypes.byref(pi.options), 5))
        N.check(L.bsq_group_replicate(g, pi.handle, None))
        N.check(L.bsq_group_run(g, ctypes.byref(pi.options), ptrs, n, 5))
        nh = L.bsq_batch_hits(b).contents.n_hits
        assert L.bsq_group_hits(g).contents.n_hits == nh
        outs = []
        for fn, h in ((L.bsq_batch_render_nuclseqs, b), (L.bsq_group_render_nuclseqs, g)):
            buf, off = ctypes.c_void_p(), ctypes.c_void_p()
            N.check(fn(h, ptrs, ctypes.byref(buf), ctypes.byref(off)))
            o = ctypes.cast(off, ctypes.POINTER(ctypes.c_int64))
            outs.append(_varlenas(buf, o, 2 * nh))
            L.bsq_free(buf)
            L.bsq_free(off)
        assert outs[0] == outs[1]
    finally:
        L.bsq_group_free(g)
        L.bsq_batch_free(b)


def test_group_errors():
    L = N.lib()
    g = ctypes.c_void_p()
    assert L.bsq_group_create((ctypes.c_int * 1)(99), 1, ctypes.byref(g)) == N.BSQ_E_NODEV
    N.check(L.bsq_group_create((ctypes.c_int * 1)(0), 1, ctypes.byref(g)))
    try:
        rc = L.bsq_group_run(g, ctypes.byref(N.Opts(19, 500, 1, 4, 5, 5, 100, 100, 6, 6, 1, 1)), None, 0, 0)
        assert rc == N.BSQ_E_INVALID and b"replicate" in L.bsq_last_error()
    finally:
        L.bsq_group_free(g)


def test_group_two_distinct_devices_routes_agree(setup):
    """on a node with 2+ GPUs, a group over two distinct devices (RCCL broadcast of the tables, a member on
    each device) gives byte-identical records over both exchange routes -- every member's own link (LINKS) and peer
    DMA over xGMI into member 0 first (VIA_FIRST, the cross-device event wait and peer-access path of relay_records)
    -- and equal to one device.  Skipped on a one-GPU box."""
    L = N.lib()
    if L.bsq_device_count() < 2:
        pytest.skip("needs two HIP devices")
    pi, _, seqs = setup
    n = len(seqs)
    ptrs = (ctypes.c_void_p * n)(*[s.ptr for s in seqs])
    want = _one_device(L, pi.handle, pi.options, ptrs, n, 77)
    g = ctypes.c_void_p()
    N.check(L.bsq_group_create((ctypes.c_int * 2)(0, 1), 2, ctypes.byref(g)))
    try:
        N.check(L.bsq_group_replicate(g, pi.handle, None))
        got = []
        for mode in (0, 1, 0):
            N.check(L.bsq_group_set_exchange(g, mode))
            N.check(L.bsq_group_run(g, ctypes.byref(pi.options), ptrs, n, 77))
            got.append(_records(L.bsq_group_hits(g).contents, n))
            N.check(L.bsq_group_run_rounds(g, ctypes.byref(pi.options), n, 77, 2))
            got.append(_records(L.bsq_group_hits(g).contents, n))
        assert all(r == want for r in got)
    finally:
        L.bsq_group_free(g)
