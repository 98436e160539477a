"""C4 (BASELINE.json configs[3]) under GPU parity: the bench's 3 Gbp synthetic reference, 24 rows x 125 Mbp.

At 2 x 3e9 = 6e9 suffixes the index takes the 64-bit-row path for real (u64 suffix array, u64 SMEM lists,
k-mer table at K = 15, all 15 levels preloaded per SMEM call -- occ blocks of a 3 GB BWT outside the Infinity Cache).  The reference itself cannot
build this index at all (is_bwt takes an int length: bioseqdb/bwa.cpp:10,47; rows are capped at
INT32_MAX/4 bases: extension.cpp:50), so the oracle is the only check.  Its FM tables are derived on the host
from the GPU-built suffix array once that SA has passed two certificates, each a proof that it is the unique SA
of T$ over all 6e9 suffixes: the device one (bsq_index_certify_sa: range, every position once, adjacent suffixes
increasing) and the oracle's own host check (range, one primary row, adjacent suffixes strictly increasing;
orc_index_build_from_sa).  A mis-sorted SA therefore cannot reach both sides (parity_util.oracle_from_device_sa).

* all 14 bwa_result columns of 20k reads (bsq_align_batch + bsq_render_tsv, the path of
  BwaIndex::align_sequence, bwa.cpp:141-181) against the oracle's rows;
* a second cursor batch that continues the backend's lrand48 stream (Q10);
* bsq_batch_seed intervals (mem_collect_intv) of 20k reads on the same index;
* the index replicated to a 2-member device group (SURVEY.md 8(e), C5's code path on one GPU: a repeated device
  holds a replica imported from device-to-device copies of the 64-bit tables), 12k reads per member aligned with
  the lrand48 stream continuing from an earlier call, every column against the oracle.
The reference rows go through the GPU bulk codec (nuclseq_in, tested byte-for-byte in test_gpu_codec.py).
"""
import ctypes
import gc

import numpy as np
import pytest

import oracle_py as O
from bioseqdb_amd import BwaIndex, NucleotideSequence, effective_opts, loader, synth
from bioseqdb_amd import _native as N
from parity_util import _oracle_batch_tsv, compare_batch, compare_tsv, oracle_from_device_sa

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]


def _seqs(reads):
    return [NucleotideSequence.from_text(reads.text(i)) for i in range(reads.n)]


@pytest.fixture(scope="module")
def c4_pair():
    ref = synth.make_reference(3_000_000_000, n_rows=24)
    texts = ref.texts()
    offs = np.zeros(len(texts) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(t) for t in texts])
    raw, voff = loader.encode_concat(np.frombuffer(b"".join(texts), dtype=np.uint8), offs)
    del texts
    vals = loader._split(raw, voff)
    del raw
    pi = BwaIndex()
    oi = O.OracleIndex()
    for i, v in enumerate(vals):
        pi.add_ref_sequence(i + 1, v)
        oi.add_ref(i + 1, v.raw)
    del vals
    pi.build_on_device()
    L = N.lib()
    assert L.bsq_index_seq_len(pi.handle) == 6_000_000_000 > 2 ** 32
    cert = oracle_from_device_sa(pi, oi, "C4 3 Gbp")
    assert cert["sa_elem_bytes"] == 8   # 64-bit suffix array
    pi.options = effective_opts(None, 24)
    yield ref, pi, oi
    del pi, oi
    gc.collect()


def test_c4_3gbp_all_columns(c4_pair):
    ref, pi, oi = c4_pair
    reads = synth.make_reads(ref, 20_000, seed=synth.READ_SEED)
    rows, bad = compare_batch(pi, oi, _seqs(reads), first_call=0)
    assert rows > 19_000
    assert not bad, bad[:20]


def test_c4_3gbp_second_call_continues_lrand48(c4_pair):
    ref, pi, oi = c4_pair
    reads = synth.make_reads(ref, 5_000, seed=synth.READ_SEED + 1)
    rows, bad = compare_batch(pi, oi, _seqs(reads), first_call=20_000)
    assert rows > 4_500
    assert not bad, bad[:20]


def test_c4_3gbp_seeding(c4_pair):
    ref, pi, oi = c4_pair
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


def test_c4_3gbp_replicated_group(c4_pair):
    ref, pi, oi = c4_pair
    reads = synth.make_reads(ref, 24_000, seed=synth.READ_SEED + 3)
    seqs = _seqs(reads)
    n = len(seqs)
    ptrs = (ctypes.c_void_p * n)(*[s.ptr for s in seqs])
    L = N.lib()
    g = ctypes.c_void_p()
    N.check(L.bsq_group_create((ctypes.c_int * 2)(0, 0), 2, ctypes.byref(g)))
    try:
        N.check(L.bsq_group_set_exchange(g, 1))   # member 1's records through member 0's HBM
        N.check(L.bsq_group_replicate(g, pi.handle, None))
        first_call = 25_000   # continues the backend's lrand48 stream (Q10)
        N.check(L.bsq_group_run(g, ctypes.byref(pi.options), ptrs, n, first_call))
        N.check(L.bsq_group_run_rounds(g, ctypes.byref(pi.options), n, first_call, 2))
        H = L.bsq_group_hits(g)
        segs = (ctypes.POINTER(N.Hits) * 16)()
        slo = (ctypes.c_int32 * 16)()
        assert L.bsq_group_segments(g, segs, slo, 16) == 2 and list(slo[:2]) == [0, n // 2]
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
