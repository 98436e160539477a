"""bwa_result rendering on the host (no GPU): the multi-threaded renderer gives the
same text as one thread, and ref_subseq follows extract_reference_subseq's quirks (bwa.cpp:55-68):
hole symbols overlaid at row-relative offsets on the concatenated text (Q3), later holes win."""
import ctypes
import random
import struct

from bioseqdb_amd import BwaIndex, NucleotideSequence
from bioseqdb_amd import _native as N
from bioseqdb_amd import bwa as B


def _decode(ns):
    """(pac text incl. the byte padding, [(offset, len, symbol)]) of a nuclseq varlena (sequence.h:18-38)."""
    raw = ns.raw
    nh, ln = struct.unpack_from("<II", raw, 4)
    holes = [struct.unpack_from("<qic", raw, 12 + 16 * i) for i in range(nh)]
    pac = raw[12 + 16 * nh:]
    text = "".join("ACGT"[(b >> s) & 3] for b in pac for s in (6, 4, 2, 0))
    return text, [(o, l, c.decode()) for o, l, c in holes]


def _concat(seqs):
    pac, holes = "", []
    for ns in seqs:
        t, h = _decode(ns)
        pac += t
        holes += h   # offsets stay row-relative (Q3)
    return pac, holes


def _expected_ref_subseq(seqs, rb, re, cat=None):
    pac, holes = cat or _concat(seqs)
    s = list(pac[rb:re])
    for o, l, c in holes:
        for i in range(max(o, rb), min(o + l, re)):
            s[i - rb] = c
    return "".join(s)


def _render(idx, seqs, records, read_off, cigars, threads, monkeypatch):
    monkeypatch.setenv("BSQ_RENDER_THREADS", str(threads))
    H = (N.Hit * max(len(records), 1))()
    for i, r in enumerate(records):
        for k, v in r.items():
            setattr(H[i], k, v)
    off = (ctypes.c_int64 * len(read_off))(*read_off)
    cig = (ctypes.c_uint32 * max(len(cigars), 1))(*cigars)
    hits = N.Hits(len(read_off) - 1, len(records), H, off, len(cigars), cig)
    arr = (ctypes.c_void_p * len(seqs))(*[s.ptr for s in seqs])
    L = N.lib()
    p = L.bsq_render_tsv(idx.handle, ctypes.byref(hits), arr)
    try:
        return ctypes.string_at(p).decode("latin-1")
    finally:
        L.bsq_free(p)


def test_render_threads_and_hole_overlay(monkeypatch):
    r = random.Random(4)
    texts = []
    for n in (5003, 3001, 2222):
        t = [r.choice("ACGT") for _ in range(n)]
        for _ in range(6):   # runs of N and IUPAC symbols
            o = r.randrange(0, n - 60)
            t[o:o + r.randrange(1, 50)] = r.choice("NRY") * len(t[o:o + 50])
        texts.append("".join(t[:n]))
    refs = [NucleotideSequence.from_text(t) for t in texts]
    idx = BwaIndex()
    for i, ns in enumerate(refs):
        idx.add_ref_sequence(100 + i, ns)
    idx.build()
    l_pac = N.lib().bsq_index_l_pac(idx.handle)
    reads = [NucleotideSequence.from_text("".join(r.choice("ACGT") for _ in range(150))) for _ in range(3000)]
    records, read_off, cigars = [], [0], []
    for i in range(len(reads)):
        for _ in range(r.randrange(0, 3)):
            rb = r.randrange(0, l_pac - 200)
            re = rb + r.randrange(100, 200)
            qb = r.randrange(0, 20)
            records.append(dict(ref_id=100, rb=rb, re=re, ref_match_start=rb, ref_match_end=re, ref_match_len=re - rb,
                                qb=qb, qe=150, score=r.randrange(-5, 150), rid=0, is_primary=1, is_secondary=0,
                                is_reverse=0, read_index=i, cigar_off=len(cigars), n_cigar=2))
            cigars += [(qb << 4) | 3, ((150 - qb) << 4) | 0]
        read_off.append(len(records))
    one = _render(idx, reads, records, read_off, cigars, 1, monkeypatch)
    many = _render(idx, reads, records, read_off, cigars, 8, monkeypatch)
    assert one == many and one.count("\n") == len(records) >= 2000
    rows = B.parse_tsv(one)
    for rec, row in zip(records, rows):
        assert row.ref_subseq == _expected_ref_subseq(refs, rec["rb"], rec["re"])
        assert row.cigar == f"{rec['qb']}N{150 - rec['qb']}M"   # clip op 3 prints as 'N' (Q8)
        assert row.score == rec["score"]


def _gapped_refs(r, rows=12, n=40000):
    """An hg38-like N-gap layout: every row has a long centromere-like gap plus telomere and scattered gaps of
    N and IUPAC symbols, so (Q3) the holes of all rows pile up on the shared row-relative axis."""
    texts = []
    for _ in range(rows):
        t = [r.choice("ACGT") for _ in range(n)]
        spans = [(0, r.randrange(50, 500)), (r.randrange(n // 3, n // 2), r.randrange(5000, 15000)),
                 (n - r.randrange(50, 500), n)]
        spans = [(a, a + b) if b < a else (a, b) for a, b in spans[:2]] + [spans[2]]
        spans += [(o, o + r.randrange(1, 300)) for o in (r.randrange(0, n - 300) for _ in range(40))]
        for a, b in spans:
            t[a:b] = r.choice("NNNRYK") * (min(b, n) - a)
        texts.append("".join(t[:n]))
    return [NucleotideSequence.from_text(t) for t in texts]


def test_render_overlapping_long_holes(monkeypatch):
    """Windows under hundreds of overlapping long holes (the overlay is one binary search plus the
    disjoint segments a window touches) give extract_reference_subseq's text."""
    r = random.Random(11)
    refs = _gapped_refs(r)
    idx = BwaIndex()
    for i, ns in enumerate(refs):
        idx.add_ref_sequence(7 + i, ns)
    idx.build()
    l_pac = N.lib().bsq_index_l_pac(idx.handle)
    reads = [NucleotideSequence.from_text("ACGT" * 40)]
    records, cigars = [], []
    for k in range(1500):
        rb = r.randrange(0, 45000) if k % 2 else r.randrange(0, l_pac - 400)
        re = min(rb + r.randrange(1, 400), l_pac)
        records.append(dict(ref_id=7, rb=rb, re=re, ref_match_start=rb, ref_match_end=re, ref_match_len=re - rb,
                            qb=0, qe=160, score=1, rid=0, is_primary=1, is_secondary=0, is_reverse=0, read_index=0,
                            cigar_off=0, n_cigar=1))
    cigars = [(160 << 4) | 0]
    text = _render(idx, reads, records, [0, len(records)], cigars, 4, monkeypatch)
    rows = B.parse_tsv(text)
    assert len(rows) == len(records)
    cat = _concat(refs)
    for rec, row in zip(records, rows):
        assert row.ref_subseq == _expected_ref_subseq(refs, rec["rb"], rec["re"], cat)
