"""GPU index construction: bsq_index_build_device yields the same suffix
array, primary row, L2 and occurrence counts as the host build (bsq_index_build), and aligns
byte-identically through it, on random, highly repetitive, tiny and multi-row (holes, padding) texts and
with 64-bit rows."""
import ctypes
import random

import numpy as np
import pytest

from bioseqdb_amd import BwaIndex, NucleotideSequence, effective_opts, synth
from bioseqdb_amd import _native as N

pytestmark = pytest.mark.gpu


def _pair(texts):
    host, dev = BwaIndex(), BwaIndex()
    for i, t in enumerate(texts):
        for x in (host, dev):
            x.add_ref_sequence(i + 1, NucleotideSequence.from_text(t))
    host.build()
    dev.build_on_device()
    for x in (host, dev):
        x.options = effective_opts(None, len(texts))
    return host, dev


def _sa(L, h):
    eb = ctypes.c_int()
    p = L.bsq_index_sa_data(h, ctypes.byref(eb))
    n = L.bsq_index_seq_len(h) + 1
    return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint32 if eb.value == 4 else ctypes.c_uint64)),
                                 shape=(n,)).copy()


def _check_same_index(host, dev, rows=3000):
    L = N.lib()
    N.check(L.bsq_index_download(dev.handle))
    assert L.bsq_index_seq_len(dev.handle) == L.bsq_index_seq_len(host.handle)
    assert L.bsq_index_primary(dev.handle) == L.bsq_index_primary(host.handle)
    a, b = _sa(L, host.handle), _sa(L, dev.handle)
    assert a.dtype == b.dtype and np.array_equal(a, b)
    n = L.bsq_index_seq_len(host.handle)
    rng = random.Random(n)
    ks = {-1, 0, n - 1, n} | {rng.randrange(-1, n + 1) for _ in range(rows)}
    c1, c2 = (ctypes.c_uint64 * 4)(), (ctypes.c_uint64 * 4)()
    for k in sorted(ks):
        N.check(L.bsq_index_occ4(host.handle, k, c1))
        N.check(L.bsq_index_occ4(dev.handle, k, c2))
        assert list(c1) == list(c2), k


def _texts_random(n, seed):
    r = random.Random(seed)
    return "".join(r.choice("ACGT") for _ in range(n))


def test_random_with_holes_and_padding():
    r = random.Random(3)
    t1 = _texts_random(120_001, 1)
    t2 = _texts_random(40_000, 2)
    t2 = t2[:9000] + "N" * 700 + t2[9700:20000] + "RY" + t2[20002:]
    t3 = _texts_random(333, 3)
    host, dev = _pair([t1, t2, t3])
    _check_same_index(host, dev)
    L = N.lib()
    rounds, tied = ctypes.c_int(), ctypes.c_uint64()
    N.check(L.bsq_index_build_stats(dev.handle, ctypes.byref(rounds), ctypes.byref(tied)))
    assert rounds.value >= 0 and tied.value < L.bsq_index_seq_len(dev.handle)
    # alignment through the device-built index equals the host-built one, row for row
    reads = [t1[p:p + 150] for p in range(0, 110_000, 997)] + [t2[p:p + 150] for p in range(0, 39_000, 1501)]
    reads = [x if i % 3 else x[::-1].translate(str.maketrans("ACGT", "TGCA")) for i, x in enumerate(reads)]
    seqs = [NucleotideSequence.from_text(x) for x in reads]
    a = host.align_sequences(seqs, host.options, first_call=5)
    b = dev.align_sequences(seqs, dev.options, first_call=5)
    assert a == b
    assert sum(len(x) for x in a) >= len(reads) - 5   # a few reads span the N run


def test_repetitive_many_rounds(monkeypatch):
    # tandem repeats and long exact copies: ties survive many doubling rounds (with the on-device SA
    # certificate: adjacent suffixes strictly increasing, every position once)
    monkeypatch.setenv("BSQ_IDX_CHECK", "1")
    unit = _texts_random(37, 9)
    block = _texts_random(5000, 10)
    t = unit * 300 + block + "ACGT" * 2000 + block + "A" * 3001 + block[:2500]
    host, dev = _pair([t])
    _check_same_index(host, dev)
    rounds = ctypes.c_int()
    N.check(N.lib().bsq_index_build_stats(dev.handle, ctypes.byref(rounds), None))
    assert rounds.value >= 7   # LCPs of ~10 kbp need h = 21 * 2^9


@pytest.mark.parametrize("text", ["A", "C", "AC", "ACG", "TTTT", "GATTACA", "ACGTACGTAC"])
def test_tiny(text):
    host, dev = _pair([text])
    _check_same_index(host, dev, rows=50)


@pytest.mark.parametrize("split", [False, True])
def test_wide_rows(monkeypatch, split):
    monkeypatch.setenv("BSQ_FORCE_WIDE", "1")
    if split:   # the bucketed first sort that texts of >= 2^32 suffixes take (3 Gbp), on a small text
        monkeypatch.setenv("BSQ_IDX_SPLIT", "1")
        monkeypatch.setenv("BSQ_IDX_CHECK", "1")
    ref = synth.make_reference(300_000, n_rows=2, n_run_every=100_000, n_run_len=200)
    texts = [t.decode() for t in ref.texts()]
    host, dev = _pair(texts)
    _check_same_index(host, dev)
    reads = synth.make_reads(ref, 400, seed=77)
    seqs = [NucleotideSequence.from_text(reads.text(i)) for i in range(reads.n)]
    assert host.align_sequences(seqs, host.options, first_call=0) == dev.align_sequences(seqs, dev.options, first_call=0)


def test_replicate_from_device_build():
    # a device-built index moves its tables into caller buffers (bsq_index_upload_into) and still aligns
    import torch
    L = N.lib()
    ref = synth.make_reference(200_000, n_rows=1)
    host, dev = _pair([t.decode() for t in ref.texts()])
    sizes = (ctypes.c_uint64 * N.N_TABLES)()
    mb = ctypes.c_uint64()
    N.check(L.bsq_index_layout(dev.handle, sizes, None, ctypes.byref(mb)))
    hs = (ctypes.c_uint64 * N.N_TABLES)()
    N.check(L.bsq_index_layout(host.handle, hs, None, ctypes.byref(mb)))
    assert list(sizes) == list(hs)
    bufs = [torch.empty(int(b), dtype=torch.uint8, device="cuda:0") if b else None for b in sizes]
    tabs = (N.Table * N.N_TABLES)(*[N.Table(t.data_ptr() if t is not None else None, int(b)) for t, b in zip(bufs, sizes)])
    N.check(L.bsq_index_upload_into(dev.handle, 0, tabs, N.N_TABLES))
    reads = synth.make_reads(ref, 300, seed=5)
    seqs = [NucleotideSequence.from_text(reads.text(i)) for i in range(reads.n)]
    assert host.align_sequences(seqs, host.options, first_call=0) == dev.align_sequences(seqs, dev.options, first_call=0)
    del dev   # the index uses the buffers: free it before them
    import gc
    gc.collect()
    del bufs


@pytest.mark.parametrize("wide", [False, True])
def test_sa_certificate_detects_corruption(monkeypatch, wide):
    """bsq_index_certify_sa (the device certificate the C3/C4 parity fixtures and bench's oracle leg run): 0
    violations for the device build and for a host build uploaded, and > 0 once two SA rows are swapped or one
    row duplicated in HBM (the SA table lives in caller-owned torch buffers via bsq_index_upload_into)."""
    import gc
    import torch
    if wide:
        monkeypatch.setenv("BSQ_FORCE_WIDE", "1")
    L = N.lib()
    ref = synth.make_reference(150_000, n_rows=2, n_run_every=60_000, n_run_len=100)
    host, dev = _pair([t.decode() for t in ref.texts()])
    host.upload()
    for x in (host, dev):
        c = x.certify_sa()
        assert c["violations"] == 0 and c["suffixes"] == L.bsq_index_seq_len(x.handle) + 1, c
    sizes = (ctypes.c_uint64 * N.N_TABLES)()
    mb = ctypes.c_uint64()
    N.check(L.bsq_index_layout(dev.handle, sizes, None, ctypes.byref(mb)))
    bufs = [torch.empty(int(b), dtype=torch.uint8, device="cuda:0") if b else None for b in sizes]
    tabs = (N.Table * N.N_TABLES)(*[N.Table(t.data_ptr() if t is not None else None, int(b)) for t, b in zip(bufs, sizes)])
    N.check(L.bsq_index_upload_into(dev.handle, 0, tabs, N.N_TABLES))
    sa = bufs[2].view(torch.int64 if wide else torch.int32)   # T_SA
    assert dev.certify_sa()["violations"] == 0
    good = sa.clone()
    n = sa.numel()
    for i in (1, n // 2, n - 2):
        sa.copy_(good)
        sa[i], sa[i + 1] = good[i + 1].item(), good[i].item()
        torch.cuda.synchronize()
        assert dev.certify_sa()["violations"] >= 1, i
    sa.copy_(good)
    sa[n // 3] = good[n // 3 + 1].item()   # one position twice, another missing
    torch.cuda.synchronize()
    assert dev.certify_sa()["violations"] >= 1
    sa.copy_(good)
    torch.cuda.synchronize()
    assert dev.certify_sa()["violations"] == 0
    del dev
    gc.collect()
    del bufs, sa, good
