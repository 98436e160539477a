"""bwa_result rows rendered on the GPU (bsq_batch_render) are byte-identical to
the host renderer (bsq_render_tsv): reference rows with N/IUPAC runs (Q3 overlay), reverse-strand rows
(Q7), clips printed as N (Q8), reads with IUPAC symbols, multi-chunk batches; and the rows' two nuclseq
columns (bsq_batch_render_nuclseqs) equal nuclseq_from_text of the printed subsequences."""
import ctypes
import random

import numpy as np
import pytest

from bioseqdb_amd import NucleotideSequence, synth
from bioseqdb_amd import _native as N
from parity_util import build_pair

pytestmark = pytest.mark.gpu


def _reads_with_iupac(reads, r):
    out = []
    for i in range(reads.n):
        t = list(reads.text(i))
        if i % 7 == 0:
            for _ in range(r.randrange(1, 3)):
                p = r.randrange(0, len(t) - 4)
                t[p:p + r.randrange(1, 4)] = r.choice("RYKNW")
        out.append("".join(t))
    return out


@pytest.mark.parametrize("chunk", [None, "700"])
def test_gpu_render_matches_host(monkeypatch, chunk):
    if chunk:
        monkeypatch.setenv("BSQ_CHUNK", chunk)
    r = random.Random(17)
    ref = synth.make_reference(400_000, n_rows=3, n_run_every=100_000, n_run_len=300)
    texts = [t.decode() for t in ref.texts()]
    texts[1] = texts[1][:5000] + "RRYY" + texts[1][5004:9000] + "N" * 40 + texts[1][9040:]
    pi, _ = build_pair(texts)
    pi.upload()
    reads = synth.make_reads(ref, 2500, seed=29)
    rtexts = _reads_with_iupac(reads, r)
    seqs = [NucleotideSequence.from_text(t) for t in rtexts]
    codes = np.concatenate([np.frombuffer(t.encode(), np.uint8) for t in rtexts])
    lut = np.full(256, 4, np.uint8)
    for c, v in zip(b"ACGT", range(4)):
        lut[c] = v
    codes = np.ascontiguousarray(lut[codes])
    offs = np.zeros(len(rtexts) + 1, np.int64)
    offs[1:] = np.cumsum([len(t) for t in rtexts])
    L = N.lib()
    b = ctypes.c_void_p()
    N.check(L.bsq_batch_create(pi.handle, len(rtexts), int(offs[-1]), ctypes.byref(b)))
    try:
        N.check(L.bsq_batch_set_reads(b, codes.ctypes.data, offs.ctypes.data, len(rtexts)))
        N.check(L.bsq_batch_run(b, ctypes.byref(pi.options), 0))
        arr = (ctypes.c_void_p * len(seqs))(*[s.ptr for s in seqs])
        p = L.bsq_render_tsv(pi.handle, L.bsq_batch_hits(b), arr)
        host = ctypes.string_at(p)
        L.bsq_free(p)
        t, n = ctypes.c_void_p(), ctypes.c_int64()
        N.check(L.bsq_batch_render(b, arr, ctypes.byref(t), ctypes.byref(n)))
        gpu = ctypes.string_at(t, n.value)
        assert n.value == len(host) and host.count(b"\n") >= 2000
        assert gpu == host
        assert b"\tf\tf\tt\t" in gpu or b"\tt\tf\tt\t" in gpu   # reverse-strand rows present
        # build_tuple_bwa's nuclseq columns (bsq_batch_render_nuclseqs) = nuclseq_from_text of the printed texts
        out, oo = ctypes.c_void_p(), ctypes.c_void_p()
        N.check(L.bsq_batch_render_nuclseqs(b, arr, ctypes.byref(out), ctypes.byref(oo)))
        rows = host.decode().splitlines()
        off = np.ctypeslib.as_array(ctypes.cast(oo, ctypes.POINTER(ctypes.c_int64)), shape=(2 * len(rows) + 1,)).copy()
        raw = ctypes.string_at(out, int(off[-1]))
        L.bsq_free(out)
        L.bsq_free(oo)
        for k, row in enumerate(rows):
            f = row.split("\t")
            for t, col in ((0, 1), (1, 5)):
                a0 = int(off[2 * k + t])
                size = int.from_bytes(raw[a0:a0 + 4], "little") >> 2
                assert raw[a0:a0 + size] == NucleotideSequence._encode(f[col]).raw, (k, col)
    finally:
        L.bsq_batch_free(b)


def test_gpu_render_overlapping_long_holes():
    """An hg38-like N-gap layout (long gaps in every row pile up on the row-relative axis, Q3): the GPU rows
    under hundreds of overlapping holes equal the host renderer's (both read the disjoint overlay segments
    of HoleIndex; tests/test_render.py pins the host against extract_reference_subseq's loop)."""
    r = random.Random(23)
    from test_render import _gapped_refs, _decode
    refs = _gapped_refs(r)
    texts = [_decode(ns)[0][:40000] for ns in refs]   # row texts without the overlay: reads come from real bases
    pi, _ = build_pair([ns.to_text() for ns in refs])
    pi.upload()
    rtexts = []
    for k in range(3000):
        row = texts[0 if k % 3 else r.randrange(len(texts))]
        p = r.randrange(0, len(row) - 150)
        rtexts.append(row[p:p + 150])
    seqs = [NucleotideSequence.from_text(t) for t in rtexts]
    codes = np.frombuffer("".join(rtexts).encode(), np.uint8)
    lut = np.full(256, 4, np.uint8)
    for c, v in zip(b"ACGT", range(4)):
        lut[c] = v
    codes = np.ascontiguousarray(lut[codes])
    offs = np.arange(len(rtexts) + 1, dtype=np.int64) * 150
    L = N.lib()
    b = ctypes.c_void_p()
    N.check(L.bsq_batch_create(pi.handle, len(rtexts), int(offs[-1]), ctypes.byref(b)))
    try:
        N.check(L.bsq_batch_set_reads(b, codes.ctypes.data, offs.ctypes.data, len(rtexts)))
        N.check(L.bsq_batch_run(b, ctypes.byref(pi.options), 0))
        arr = (ctypes.c_void_p * len(seqs))(*[s.ptr for s in seqs])
        p = L.bsq_render_tsv(pi.handle, L.bsq_batch_hits(b), arr)
        host = ctypes.string_at(p)
        L.bsq_free(p)
        t, n = ctypes.c_void_p(), ctypes.c_int64()
        N.check(L.bsq_batch_render(b, arr, ctypes.byref(t), ctypes.byref(n)))
        gpu = ctypes.string_at(t, n.value)
        assert host.count(b"\n") >= 2000 and gpu == host
        under = sum(1 for row in host.decode().splitlines() if set(row.split("\t")[1]) & set("NRYK"))
        assert under >= 100   # rows whose ref_subseq carries overlay symbols
    finally:
        L.bsq_batch_free(b)
