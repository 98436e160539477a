"""Deterministic synthetic reference and read generator.

Reference: uniform i.i.d. ACGT rows (lengths multiples of 4 by default so no padding bases, Q4),
one 1,000-bp N run per 10 Mbp (holes, Q3/Q5) and 0.5% of the sequence copied as 500-5,000-bp
segments to random loci, half reverse-complemented (multi-hits, secondaries, ties).
Reads: 150 bp at a uniform start within a row, strand 50/50, 1% substitutions, 0.05%/base indels of
length 1-3, 2% random (unmappable) reads, 0.1% with one N.  numpy PCG64 streams seeded with
ref_seed=0x5EED0001 / read_seed=0x5EED0002 make every run bit-identical.
"""
from __future__ import annotations

import dataclasses
from typing import List, Optional, Tuple

import numpy as np

REF_SEED = 0x5EED0001
READ_SEED = 0x5EED0002
_ACGTN = np.frombuffer(b"ACGTN", dtype=np.uint8)


@dataclasses.dataclass
class Reference:
    rows: List[np.ndarray]          # nt codes per row: 0..3 bases, 4 = N

    def texts(self) -> List[bytes]:
        return [_ACGTN[r].tobytes() for r in self.rows]

    @property
    def total(self) -> int:
        return int(sum(len(r) for r in self.rows))


@dataclasses.dataclass
class Reads:
    codes: np.ndarray               # concatenated nt4 codes (uint8)
    offsets: np.ndarray             # int64[n+1]
    truth_row: np.ndarray           # int32, -1 for random reads
    truth_pos: np.ndarray           # int64 forward start of the source window
    truth_rev: np.ndarray           # bool

    @property
    def n(self) -> int:
        return len(self.offsets) - 1

    def text(self, i: int) -> str:
        return _ACGTN[self.codes[self.offsets[i]:self.offsets[i + 1]]].tobytes().decode()

    def subset(self, lo: int, hi: int) -> "Reads":
        o = self.offsets[lo:hi + 1]
        return Reads(self.codes[o[0]:o[-1]].copy(), (o - o[0]).astype(np.int64), self.truth_row[lo:hi],
                     self.truth_pos[lo:hi], self.truth_rev[lo:hi])


def make_reference(total_bp: int, n_rows: int = 1, seed: int = REF_SEED, n_run_every: int = 10_000_000,
                   n_run_len: int = 1000, dup_frac: float = 0.005, row_align: int = 4) -> Reference:
    rng = np.random.Generator(np.random.PCG64(seed))
    base = total_bp // n_rows
    rows = []
    for r in range(n_rows):
        L = base if r < n_rows - 1 else total_bp - base * (n_rows - 1)
        L -= L % row_align if row_align > 1 else 0
        rows.append(rng.integers(0, 4, size=L, dtype=np.uint8))
    # segmental duplications (before N runs so copies carry only bases)
    for row in rows:
        L = len(row)
        budget = int(L * dup_frac)
        while budget > 0 and L > 10_000:
            ln = int(rng.integers(500, 5001))
            src = int(rng.integers(0, L - ln))
            dst = int(rng.integers(0, L - ln))
            seg = row[src:src + ln].copy()
            if rng.random() < 0.5:
                seg = (3 - seg)[::-1]
            row[dst:dst + ln] = seg
            budget -= ln
    # N runs
    for row in rows:
        L = len(row)
        for start in range(0, L, n_run_every):
            if L - start <= n_run_len * 2 or L < n_run_every // 10:
                continue
            p = start + int(rng.integers(0, min(n_run_every, L - start) - n_run_len))
            row[p:p + n_run_len] = 4
    return Reference(rows)


def make_reads(ref: Reference, n: int, length: int = 150, seed: int = READ_SEED, sub_rate: float = 0.01,
               indel_rate: float = 0.0005, random_frac: float = 0.02, n_frac: float = 0.001) -> Reads:
    rng = np.random.Generator(np.random.PCG64(seed))
    lens = np.array([len(r) for r in ref.rows], dtype=np.int64)
    w = lens / lens.sum()
    row_of = rng.choice(len(ref.rows), size=n, p=w)
    pad = length + 8
    starts = (rng.random(n) * np.maximum(lens[row_of] - pad, 1)).astype(np.int64)
    rev = rng.random(n) < 0.5
    is_rand = rng.random(n) < random_frac
    has_n = rng.random(n) < n_frac
    win = np.empty((n, pad), dtype=np.uint8)
    for r in range(len(ref.rows)):
        sel = np.nonzero(row_of == r)[0]
        if len(sel):
            idx = starts[sel, None] + np.arange(pad)[None, :]
            win[sel] = ref.rows[r][np.minimum(idx, lens[r] - 1)]
    win[win == 4] = rng.integers(0, 4, size=int((win == 4).sum()), dtype=np.uint8)   # N-run bases -> random
    out = np.empty((n, length), dtype=np.uint8)
    n_indel = rng.poisson(indel_rate * length, size=n)
    plain = n_indel == 0
    out[plain] = win[plain, :length]
    for i in np.nonzero(~plain)[0]:
        seq = list(win[i])
        for _ in range(int(n_indel[i])):
            p = int(rng.integers(10, length - 10))
            ln = int(rng.integers(1, 4))
            if rng.random() < 0.5:
                del seq[p:p + ln]
            else:
                seq[p:p] = list(rng.integers(0, 4, size=ln, dtype=np.uint8))
        seq = (seq + [0] * length)[:length]
        out[i] = np.array(seq, dtype=np.uint8)
    subs = rng.random((n, length)) < sub_rate
    out[subs] = (out[subs] + rng.integers(1, 4, size=int(subs.sum()), dtype=np.uint8)) % 4
    out[rev] = (3 - out[rev])[:, ::-1]
    out[is_rand] = rng.integers(0, 4, size=(int(is_rand.sum()), length), dtype=np.uint8)
    hn = np.nonzero(has_n)[0]
    out[hn, rng.integers(0, length, size=len(hn))] = 4
    codes = out.reshape(-1).copy()
    offsets = np.arange(n + 1, dtype=np.int64) * length
    truth_row = np.where(is_rand, -1, row_of).astype(np.int32)
    return Reads(codes, offsets, truth_row, starts, rev & ~is_rand)
