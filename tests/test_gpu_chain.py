"""Chaining (mem_chain + mem_chain_flt) on repeat-rich inputs: reads whose SMEMs have many
occurrences carry more seeds and chains than k_chain_s's LDS share (12 seeds, 9 chains: align_kernels.hip), so
they are handed to k_chain<64>'s second launch; the rest stay in LDS.  Every bwa_result column must match the CPU
oracle on both paths, and the all-scratch path (BSQ_CHAIN_SCRATCH=1) must give the same rows."""
import numpy as np
import pytest

from parity_util import build_pair, compare

pytestmark = pytest.mark.gpu

ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)


def _repeat_reference(seed=7):
    rng = np.random.Generator(np.random.PCG64(seed))
    ref = rng.integers(0, 4, size=240_000, dtype=np.uint8)
    unit = rng.integers(0, 4, size=320, dtype=np.uint8)
    starts = []
    for k in range(28):   # interspersed copies of one unit, ~2 % diverged: MEMs with 2..28 occurrences
        c = unit.copy()
        m = rng.random(c.size) < 0.02
        c[m] = rng.integers(0, 4, size=int(m.sum()), dtype=np.uint8)
        if k % 3 == 0:
            c = (3 - c)[::-1]
        p = 5_000 + k * 8_000 + int(rng.integers(0, 3_000))
        ref[p:p + c.size] = c
        starts.append(p)
    tr = rng.integers(0, 4, size=37, dtype=np.uint8)   # a tandem repeat of 60 copies of a 37-mer
    ref[120_000:120_000 + 37 * 60] = np.tile(tr, 60)
    return ACGT[ref].tobytes().decode(), starts


def _reads(text, starts, n, seed=3):
    rng = np.random.Generator(np.random.PCG64(seed))
    comp = str.maketrans("ACGT", "TGCA")
    out = []
    for i in range(n):
        kind = i % 4
        if kind == 0:
            p = int(rng.integers(0, len(text) - 150))
        elif kind == 3:
            p = 120_000 + int(rng.integers(-100, 37 * 60 - 50))
        else:
            p = starts[int(rng.integers(0, len(starts)))] + int(rng.integers(-120, 300))
        r = list(text[p:p + 150])
        for j in range(len(r)):
            if rng.random() < 0.015:
                r[j] = "ACGT"[int(rng.integers(0, 4))]
        s = "".join(r)
        out.append(s.translate(comp)[::-1] if rng.random() < 0.5 else s)
    return out


def test_chain_lds_and_fallback_match_oracle(monkeypatch):
    text, starts = _repeat_reference()
    pi, oi = build_pair([text])
    reads = _reads(text, starts, 2000)
    rows, bad = compare(pi, oi, reads, first_call=17)
    assert rows > 1900
    assert not bad, bad[:20]
    # the all-scratch path (k_chain<64> on every read) gives the same rows
    monkeypatch.setenv("BSQ_CHAIN_SCRATCH", "1")
    rows2, bad2 = compare(pi, oi, reads, first_call=17)
    assert rows2 == rows
    assert not bad2, bad2[:20]


def test_chain_many_occurrence_reads():
    """Reads drawn only from the 28-copy unit and the tandem repeat: nearly all go past the LDS share."""
    text, starts = _repeat_reference(seed=11)
    pi, oi = build_pair([text])
    reads = [r for i, r in enumerate(_reads(text, starts, 1200, seed=5)) if i % 4 != 0]
    rows, bad = compare(pi, oi, reads, first_call=5)
    assert rows > 800
    assert not bad, bad[:20]
