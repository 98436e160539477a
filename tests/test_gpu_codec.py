"""Bulk nuclseq codec on the GPU against the oracle's restatement of
nuclseq_from_text / to_text_palloc (oracle/bwa_oracle.c, sequence.cpp:71-81,209-245): byte-identical
varlenas (holes, minstd_rand fill of hole and padding bases, zeroed padding) for ragged batches, holes
that cross lane and tile boundaries, all-hole and empty texts; nuclseq_in's errors and their order
(the reference's own test/run.py cases); decode against the oracle, including overlapping holes; and a
200 Mbp round trip."""
import ctypes
import random
import string

import numpy as np
import pytest

import oracle_py as O
from bioseqdb_amd import loader, synth
from bioseqdb_amd.bwa import InvalidTextRepresentation, NucleotideSequence

pytestmark = pytest.mark.gpu

IUPAC = "NWSMKRYBDHV"


def rand_text(rng, n, hole_rate=0.01):
    s = []
    while len(s) < n:
        if rng.random() < hole_rate:
            s += [rng.choice(IUPAC)] * rng.choice([1, 1, 2, 3, 7, 40, 300, 1500])
        else:
            s.append(rng.choice("ACGT"))
    return "".join(s[:n])


def check_batch(texts):
    got = loader.nuclseq_in_batch(texts)
    assert len(got) == len(texts)
    for t, g in zip(texts, got):
        assert g.raw == O.Nuclseq(t).raw, (len(t), t[:40])
    return got


def test_ragged_small_texts():
    rng = random.Random(1)
    texts = [rand_text(rng, n, 0.05) for n in list(range(0, 40)) + [rng.randint(0, 3000) for _ in range(400)]]
    check_batch(texts)


def test_holes_across_lanes_and_tiles():
    rng = random.Random(2)
    texts = []
    for L in (1023, 1024, 1025, 4096 + 3, 20_000):
        for sym in ("N", "R"):
            for start in (0, 3, 4, 1020, 1023, 1024):
                if start < L:
                    t = list(rand_text(rng, L, 0.0))
                    for j in range(start, min(L, start + rng.choice([1, 5, 1024, 3000]))):
                        t[j] = sym
                    texts.append("".join(t))
    texts += ["N" * 5000, "NR" * 700, "RRRRNNNN" * 100, "", "A", "N", "ACG", "NNN", "ACGTN"]
    check_batch(texts)


def test_many_reads_and_one_large_row():
    rng = random.Random(3)
    reads = [rand_text(rng, 150, 0.001) for _ in range(20_000)]
    big = rand_text(rng, 3_000_001, 0.0005)
    check_batch(reads[:10_000] + [big] + reads[10_000:])


def test_reference_test_cases():
    # test/run.py: nuclseq_accept_* round trips and the rejections with their messages
    for t in ("ACGT", "N", "RYKMSWBDHVN", ""):
        (v,) = loader.nuclseq_in_batch([t])
        assert loader.nuclseq_out_batch([v]) == [t]
        assert v.raw == NucleotideSequence.from_text(t).raw
    bad = set(string.ascii_lowercase) | (set(string.ascii_uppercase) - set("ACGTNRYKMSWBDHV")) | \
        (set(chr(i) for i in range(1, 128)) - set(string.ascii_letters))
    for ch in sorted(bad):
        with pytest.raises(InvalidTextRepresentation, match="invalid nucleotide in nuclseq_in: '"):
            loader.nuclseq_in_batch(["ACGT", "AC" + ch + "GT"])
    with pytest.raises(InvalidTextRepresentation) as e:
        loader.nuclseq_in_batch(["żółć".encode()])
    assert "'�'" in str(e.value)


def test_first_invalid_in_text_order():
    texts = ["ACGT" * 300, "ACGTx" + "A" * 5000 + "q", "ACGTNNNz"]
    with pytest.raises(InvalidTextRepresentation, match="'x'"):
        loader.nuclseq_in_batch(texts)
    # unvalidated: the bytes nuclseq_from_text gives (any non-ACGT byte is a hole symbol)
    got = loader.nuclseq_in_batch(texts, validate=False)
    for t, g in zip(texts, got):
        assert g.raw == O.Nuclseq(t).raw


def test_decode_matches_oracle_including_overlapping_holes():
    rng = random.Random(5)
    vals = check_batch([rand_text(rng, rng.randint(0, 2000), 0.03) for _ in range(300)])
    texts = loader.nuclseq_out_batch(vals)
    assert texts == [O.Nuclseq(v.to_text()).to_text() for v in vals]
    # hand-made varlenas whose holes overlap: later holes win (inplace_to_text :77-78)
    base = bytearray(O.Nuclseq("ACGTACGTACGTACGTACGT").raw)
    holes = [(2, 8, "N"), (5, 4, "R"), (0, 3, "Y")]
    size = 12 + 16 * len(holes) + 5
    raw = bytearray(size)
    raw[0:4] = (size << 2).to_bytes(4, "little")
    raw[4:8] = len(holes).to_bytes(4, "little")
    raw[8:12] = (20).to_bytes(4, "little")
    for k, (off, ln, amb) in enumerate(holes):
        p = 12 + 16 * k
        raw[p:p + 8] = off.to_bytes(8, "little")
        raw[p + 8:p + 12] = ln.to_bytes(4, "little")
        raw[p + 12] = ord(amb)
    raw[12 + 16 * len(holes):] = base[12:]
    v = NucleotideSequence(bytes(raw))
    p = O.lib().orc_nuclseq_to_text(v.ptr)
    exp = ctypes.string_at(p).decode()
    O.lib().orc_free(p)
    assert exp == "YYYNNRRRRNGTACGTACGT"
    assert loader.nuclseq_out_batch([v]) == [exp]


def test_large_round_trip():
    ref = synth.make_reference(200_000_000, n_rows=4, n_run_every=5_000_000, n_run_len=2000)
    texts = ref.texts()
    offs = np.zeros(len(texts) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(t) for t in texts])
    raw, off = loader.encode_concat(b"".join(texts), offs)
    vals = loader._split(raw, off)
    # each row against the product's per-value host codec (itself pinned to the oracle above)
    for t, v in zip(texts, vals):
        assert v.raw == NucleotideSequence._encode(t.decode()).raw
    assert [t.encode() for t in loader.nuclseq_out_batch(vals)] == texts
