"""Pin the CPU oracle: brute-force cross-checks and known-answer tests (no GPU).

The reference's own tests (test/run.py) cover only the nuclseq text codec, so those cases are
reproduced first; the alignment arithmetic is pinned by (a) naive suffix sorting / counting for the
FM index and SMEM intervals, (b) full-matrix DPs with the same recurrences as ksw_extend2 /
ksw_global2, (c) planted reads with known alignments.
"""
import ctypes
import random
import string

import pytest

import oracle_py as O
from bioseqdb_amd import bwa as B

OPTS = O.OrcOpts(19, 500, 1, 4, 5, 5, 100, 100, 6, 6, 1, 1)   # effective SQL defaults (Q1)
MAT = (ctypes.c_int8 * 25)(*[(1 if i == j else -4) if i < 4 and j < 4 else -1 for i in range(5) for j in range(5)])
COMP = str.maketrans("ACGT", "TGCA")


# --------------------------------------------------------------------------------------------- codec
def minstd(seed):
    x = seed % 2147483647 or 1
    while True:
        x = x * 48271 % 2147483647
        yield x


def naive_nuclseq(text: str) -> bytes:
    """Independent re-derivation of sequence.cpp:209-245 for the codec KATs."""
    holes = []
    prev = ""
    for i, c in enumerate(text):
        if c not in "ACGT":
            if c == prev:
                holes[-1][1] += 1
            else:
                holes.append([i, 1, c])
        prev = c
    n = len(text)
    nb = (n + 3) // 4
    pac = bytearray(nb)
    rng = minstd(len(holes) ^ n)
    for i, c in enumerate(text):
        v = "ACGT".index(c) if c in "ACGT" else next(rng) & 3
        pac[i >> 2] |= v << ((~i & 3) << 1)
    for i in range(n, nb * 4):
        pac[i >> 2] |= (next(rng) & 3) << ((~i & 3) << 1)
    size = 12 + 16 * len(holes) + nb
    out = bytearray((size << 2).to_bytes(4, "little") + len(holes).to_bytes(4, "little") + n.to_bytes(4, "little"))
    for off, ln, amb in holes:
        out += off.to_bytes(8, "little") + ln.to_bytes(4, "little") + amb.encode() + b"\0\0\0"
    return bytes(out + pac)


@pytest.mark.parametrize("text", ["ACGT", "N", "RYKMSWBDHVN", "", "A", "NNNNACGTNNRRRA", "ACGTACGTA", "TTTTTTTTTTT"])
def test_codec_kat(text):
    o = O.Nuclseq(text)
    assert o.raw == naive_nuclseq(text)
    assert o.to_text() == text
    p = B.NucleotideSequence.from_text(text)
    assert p.raw == o.raw and p.to_text() == text and len(p) == len(text)


def test_codec_random_equal():
    rng = random.Random(1)
    for _ in range(200):
        t = "".join(rng.choice("ACGTACGTACGTNRYKMSWBDHV") for _ in range(rng.randint(0, 300)))
        assert O.Nuclseq(t).raw == B.NucleotideSequence.from_text(t).raw == naive_nuclseq(t)


def test_codec_rejects_like_reference():
    # test/run.py:40-94: lowercase and unknown letters are rejected with this message
    for ch in string.ascii_lowercase:
        with pytest.raises(B.InvalidTextRepresentation, match=f"invalid nucleotide in nuclseq_in: '{ch}'"):
            B.NucleotideSequence.from_text(ch)
    for ch in set(string.ascii_uppercase) - set("ACGTNRYKMSWBDHV"):
        with pytest.raises(B.InvalidTextRepresentation):
            B.NucleotideSequence.from_text(ch)


def test_lrand48_stream():
    assert [O.lrand48_at(i) for i in range(4)] == [0, 2116118, 89401895, 379337186]


# ---------------------------------------------------------------------------------------- FM index
def make_index(rows):
    oi = O.OracleIndex()
    for k, t in enumerate(rows):
        oi.add_ref(k + 1, O.Nuclseq(t).raw)
    oi.build()
    return oi


def text_T(oi):
    lp = oi.l_pac
    f = "".join("ACGT"[oi_base] for oi_base in (O.lib().orc_index_pac_base(oi.h, i) for i in range(lp)))
    return f + f.translate(COMP)[::-1]


def test_sa_and_occ_vs_naive():
    rng = random.Random(2)
    rows = ["".join(rng.choice("ACGT") for _ in range(rng.randint(1, 400))) for _ in range(3)] + ["ACAC" * 30]
    oi = make_index(rows)
    T = text_T(oi)
    n = len(T)
    assert oi.seq_len == n
    # "$" sorts before every base: explicit key with $ = 0
    sa = sorted(range(n + 1), key=lambda i: [("ACGT".index(c) + 1) for c in T[i:]] + [0])
    for r in range(1, n + 1):
        assert oi.sa(r) == sa[r]
    primary = sa.index(0)
    assert oi.primary == primary
    bwt = [T[s - 1] for s in sa if s != 0]   # $-removed BWT
    for k in range(-1, n):
        kk = k - (k >= primary)
        exp = [sum(1 for c in bwt[:kk + 1] if c == b) for b in "ACGT"]
        assert oi.occ4(k) == exp, k
    assert oi.l2() == [0] + [sum(T.count(b) for b in "ACGT"[:i + 1]) for i in range(4)]


def occurrences(T, s):
    c, i = 0, T.find(s)
    while i >= 0:
        c += 1
        i = T.find(s, i + 1)
    return c


def test_smem_intervals_vs_naive_counts():
    rng = random.Random(3)
    ref = "".join(rng.choice("ACGT") for _ in range(3000))
    ref = ref[:1000] + ref[200:600] + ref[1000:]          # a duplicated segment -> multi-hit intervals
    oi = make_index([ref])
    T = text_T(oi)
    for t in range(60):
        p = rng.randrange(len(ref) - 120)
        q = list(ref[p:p + 120])
        for j in range(len(q)):
            if rng.random() < 0.03:
                q[j] = rng.choice("ACGT")
        codes = bytes("ACGT".index(c) for c in q)
        for x0, x1, x2, info in oi.collect_intv(OPTS, codes):
            b, e = info >> 32, info & 0xFFFFFFFF
            s = "".join(q[b:e])
            assert e - b >= 19
            assert x2 == occurrences(T, s)
            rows = sorted(oi.sa(r) for r in range(x0, x0 + x2))
            assert all(T[pos:pos + len(s)] == s for pos in rows)
            rc = s.translate(COMP)[::-1]
            assert sorted(oi.sa(r) for r in range(x1, x1 + x2)) == sorted(
                i for i in range(len(T)) if T.startswith(rc, i))


# ----------------------------------------------------------------------------------- DP cross-checks
NEG = -(1 << 30)


def full_extend(q, t, o_del, e_del, o_ins, e_ins, end_bonus, h0):
    """ksw_extend2 recurrences over the full matrix (no band, no z-drop)."""
    qlen, tlen = len(q), len(t)
    oe_del, oe_ins = o_del + e_del, o_ins + e_ins
    H = [0] * (qlen + 1)
    E = [0] * (qlen + 1)
    H[0] = h0
    H[1] = h0 - oe_ins if h0 > oe_ins else 0 if qlen >= 1 else 0
    for j in range(2, qlen + 1):
        H[j] = H[j - 1] - e_ins if H[j - 1] > e_ins else 0
    mx, mi, mj, gscore, gi, max_off = h0, -1, -1, -1, -1, 0
    for i in range(tlen):
        f, h1, m, mjj = 0, max(h0 - (o_del + e_del * (i + 1)), 0), 0, -1
        for j in range(qlen):
            M, e = H[j], E[j]
            H[j] = h1
            M = M + MAT[t[i] * 5 + q[j]] if M else 0
            h = max(M, e, f)
            h1 = h
            mjj = mjj if m > h else j
            m = max(m, h)
            e = max(e - e_del, max(M - oe_del, 0))
            E[j] = e
            f = max(f - e_ins, max(M - oe_ins, 0))
        H[qlen] = h1
        E[qlen] = 0
        if not (gscore > h1):
            gi = i
        gscore = max(gscore, h1)
        if m == 0:
            break
        if m > mx:
            mx, mi, mj = m, i, mjj
            max_off = max(max_off, abs(mjj - i))
    return mx, mj + 1, mi + 1, gi + 1, gscore, max_off


def test_ksw_extend2_vs_full_matrix():
    rng = random.Random(4)
    for trial in range(300):
        ql, tl = rng.randint(1, 40), rng.randint(1, 60)
        t = [rng.randrange(4) for _ in range(tl)]
        q = t[:ql] if rng.random() < 0.5 and tl >= ql else [rng.randrange(4) for _ in range(ql)]
        q = [c if rng.random() > 0.1 else rng.randrange(5) for c in q]
        h0 = rng.randint(1, 40)
        od, ed, oi_, ei = rng.choice([(6, 6, 1, 1), (6, 1, 6, 1), (3, 2, 4, 1)])
        qb, tb = bytes(q), bytes(t)
        outs = [ctypes.c_int() for _ in range(5)]
        sc = O.lib().orc_ksw_extend2(ql, qb, tl, tb, MAT, od, ed, oi_, ei, 1000, 5, 0, h0, *[ctypes.byref(o) for o in outs])
        exp = full_extend(q, t, od, ed, oi_, ei, 5, h0)
        # the banded kernel may stop early when the band empties; scores and maxima must agree
        assert (sc, outs[0].value, outs[1].value) == exp[:3], (trial, sc, [o.value for o in outs], exp)


def full_global(q, t, o_del, e_del, o_ins, e_ins):
    qlen, tlen = len(q), len(t)
    oe_del, oe_ins = o_del + e_del, o_ins + e_ins
    H = [0] + [-(o_ins + e_ins * j) for j in range(1, qlen + 1)]
    E = [NEG] * (qlen + 1)
    for i in range(tlen):
        f, h1 = NEG, -(o_del + e_del * (i + 1))
        for j in range(qlen):
            m, e = H[j], E[j]
            H[j] = h1
            m += MAT[t[i] * 5 + q[j]]
            h = max(m, e, f)
            h1 = h
            e = max(e - e_del, m - oe_del)
            E[j] = e
            f = max(f - e_ins, m - oe_ins)
        H[qlen] = h1
        E[qlen] = NEG
    return H[qlen]


def cigar_score(cig, q, t, o_del, e_del, o_ins, e_ins):
    i = j = s = 0
    for c in cig:
        ln, op = c >> 4, c & 0xF
        if op == 0:
            for _ in range(ln):
                s += MAT[t[i] * 5 + q[j]]
                i += 1
                j += 1
        elif op == 1:
            s -= o_ins + e_ins * ln
            j += ln
        else:
            s -= o_del + e_del * ln
            i += ln
    assert i == len(t) and j == len(q)
    return s


def test_ksw_global2_vs_full_matrix():
    rng = random.Random(5)
    for trial in range(300):
        tl = rng.randint(1, 50)
        t = [rng.randrange(4) for _ in range(tl)]
        q = list(t)
        for _ in range(rng.randint(0, 4)):
            k = rng.randrange(len(q) + 1)
            if rng.random() < 0.5 and len(q) > 1:
                del q[min(k, len(q) - 1)]
            else:
                q.insert(k, rng.randrange(4))
        q = [c if rng.random() > 0.05 else rng.randrange(4) for c in q]
        od, ed, oi_, ei = rng.choice([(6, 6, 1, 1), (6, 1, 6, 1), (3, 2, 4, 1)])
        n = ctypes.c_int()
        cig = (ctypes.c_uint32 * 256)()
        sc = O.lib().orc_ksw_global2(len(q), bytes(q), tl, bytes(t), MAT, od, ed, oi_, ei, 200, ctypes.byref(n), cig, 256)
        assert sc == full_global(q, t, od, ed, oi_, ei), trial
        assert cigar_score(list(cig)[:n.value], q, t, od, ed, oi_, ei) == sc


def _detour_free(t, q, od, ed, oi_, ei):
    """dp_wave.hip detour_free: S beats every path with >= 2 insertions (bound) and, exactly, every path with one
    insertion and one deletion (a detour along diagonal +1 or -1)."""
    n = len(t)
    s0 = [MAT[t[k] * 5 + q[k]] for k in range(n)]
    S = sum(s0)
    if S <= (n - 2) * max(MAT) - (oi_ + od + 2 * (ei + ed)):
        return False
    x = -10 ** 9
    for shift in (1, -1):
        c = mn = 0
        for b in range(n):
            mn = min(mn, c)
            x = max(x, c - mn - s0[b])
            if b + 1 < n:
                c += (MAT[t[b] * 5 + q[b + 1]] if shift == 1 else MAT[t[b + 1] * 5 + q[b]]) - s0[b]
    return x < oi_ + ei + od + ed


def test_diagonal_shortcut_theorem():
    """dev_common.h diagonal_wins() and dp_wave.hip detour_free(): for an n x n ksw_global2 whose gapless diagonal
    scores S above (n-1)*mat_max - oe_ins - oe_del, or above every detour (exact for one insertion + one
    deletion, bounded for more), the DP (oracle, full traceback) returns exactly "nM" with score S, for every
    band.  The reg2aln kernels skip the DP on those predicates."""
    rng = random.Random(12)
    mat_max = max(MAT)
    hits = [0, 0]
    for trial in range(4000):
        n = rng.choice([1, 2, 3, 5, 8, 20, 60, 150])
        t = [rng.randrange(4) for _ in range(n)]
        q = list(t)
        for _ in range(rng.choice([0, 1, 1, 2, 2, 3, 4, 5, 6])):
            k = rng.randrange(n)
            q[k] = rng.randrange(5) if rng.random() < 0.2 else (q[k] + rng.randint(1, 3)) % 4
        if rng.random() < 0.3 and n > 8:   # low-complexity stretches: off-diagonal paths score well
            s = rng.randrange(n - 4)
            for k in range(s, min(n, s + rng.randint(3, 12))):
                t[k] = q[k] = t[s]
        od, ed, oi_, ei = rng.choice([(6, 6, 1, 1), (6, 1, 6, 1), (3, 2, 4, 1), (0, 1, 0, 1), (1, 0, 0, 1)])
        diag = sum(MAT[t[i] * 5 + q[i]] for i in range(n))
        simple = diag > (n - 1) * mat_max - (oi_ + ei) - (od + ed)
        exact = _detour_free(t, q, od, ed, oi_, ei)
        assert exact or not simple, trial   # the exact form decides everything the simple bound does
        if not exact:
            continue
        hits[simple] += 1
        for w in (0, 1, 3, 8, 100):
            nc = ctypes.c_int()
            cig = (ctypes.c_uint32 * 512)()
            sc = O.lib().orc_ksw_global2(n, bytes(q), n, bytes(t), MAT, od, ed, oi_, ei, w, ctypes.byref(nc), cig, 512)
            assert sc == diag, (trial, w)
            assert list(cig)[:nc.value] == [n << 4], (trial, w, list(cig)[:nc.value])
    assert hits[1] > 1000 and hits[0] > 150   # both the simple bound and the detour scan carry weight


# ------------------------------------------------------------------------------- planted reads (KAT)
def test_planted_reads():
    rng = random.Random(6)
    ref = "".join(rng.choice("ACGT") for _ in range(100_000))
    oi = make_index([ref])
    lp = oi.l_pac

    def align(read, k=0):
        return B.parse_tsv(oi.align_tsv(OPTS, O.Nuclseq(read).raw, O.lrand48_at(k)))

    p = 31_337
    r = ref[p:p + 150]
    m = align(r)
    assert len(m) == 1
    m = m[0]
    assert (m.ref_match_begin, m.ref_match_end, m.cigar, m.score, m.is_primary, m.is_reverse) == (p, p + 150, "150M", 150, True, False)
    assert m.ref_subseq == r and m.query_subseq == r and m.ref_id == 1
    m = align(r.translate(COMP)[::-1])[0]
    assert m.is_reverse and m.ref_match_begin == 2 * lp - p - 150 and m.cigar == "150M" and m.score == 150
    mm = list(r)
    mm[70] = "A" if mm[70] != "A" else "C"
    m = align("".join(mm))[0]
    assert m.cigar == "150M" and m.score == 150 - 1 - 4
    dl = r[:100] + r[101:]           # read lacks one reference base: deletion costs o_del + e_del = 12
    m = align(dl)[0]
    assert "1D" in m.cigar and m.score == 149 - 12 and m.ref_match_len == 150
    ins = r[:80] + "G" + r[80:149]   # one inserted base: o_ins + e_ins = 2
    m = align(ins)[0]
    assert "1I" in m.cigar and m.score == 149 - 2
    pre = [rng.choice("ACGT") for _ in range(40)]
    pre[39] = "A" if r[39] != "A" else "C"          # force the soft clip to end exactly at 40
    clip = "".join(pre) + r[40:]
    m = align(clip)[0]
    assert m.cigar.endswith("110M") and m.cigar.startswith("40N") and m.query_match_begin == 40   # Q8: clip prints N
    assert align("ACGT" * 4) == []                                  # shorter than min_seed_len


# ---- ksw_align2 score (mem_seed_sw, the long-read seed filter) -------------------------------------------
def _mat(a=1, b=4):
    mat = []
    for i in range(5):
        for j in range(5):
            mat.append(-1 if i == 4 or j == 4 else (a if i == j else -b))
    return (ctypes.c_int8 * 25)(*mat)


def _gotoh_local(q, t, mat, od, ed, oi, ei):
    """Plain affine-gap Smith-Waterman (E: deletion along the target, F: insertion along the query)."""
    best = 0
    H = [0] * (len(q) + 1)
    E = [0] * (len(q) + 1)
    for i in range(len(t)):
        diag, f = 0, 0
        newH = [0] * (len(q) + 1)
        for j in range(len(q)):
            h = max(diag + mat[t[i] * 5 + q[j]], E[j], f, 0)
            diag = H[j]
            newH[j] = h
            best = max(best, h)
            E[j] = max(E[j] - ed, h - od - ed, 0)
            f = max(f - ei, h - oi - ei, 0)
        H = newH
    return best


def _ksw(q, t, mat, od=6, ed=6, oi=1, ei=1):
    qa, ta = bytes(q), bytes(t)
    return O.lib().orc_ksw_align2_score(len(q), qa, len(t), ta, mat, od, ed, oi, ei)


def test_ksw_align2_score_identity_and_bounds():
    import random
    mat = _mat()
    r = random.Random(11)
    for n in (1, 7, 8, 9, 31, 64, 150, 199):
        s = [r.randrange(4) for _ in range(n)]
        assert _ksw(s, s, mat) == n
    for _ in range(60):
        q = [r.randrange(4) for _ in range(r.randrange(5, 90))]
        t = [r.randrange(4) for _ in range(r.randrange(5, 90))]
        if r.random() < 0.5:   # related pair with an insertion and mismatches
            t = q[: len(q) // 2] + q[len(q) // 2 + 3:]
            t = [x if r.random() > 0.05 else (x + 1) % 4 for x in t]
        g = _gotoh_local(q, t, list(mat), 6, 6, 1, 1)
        k = _ksw(q, t, mat)
        assert 0 <= k <= g   # the striped kernel's lazy F never raises the maximum or E
        # without insertions (a prohibitive open penalty) F never fires: the striped result is the optimum
        assert _ksw(q, t, mat, oi=1000) == _gotoh_local(q, t, list(mat), 6, 6, 1000, 1)



def test_integer_band_formulas_equal_double():
    """dev_common.h idiv_plus: (x + k*d) / d in C integers equals libbwa's (int)((double)x / d + k) for the
    band / gap-length formulas (cal_max_gap, ksw_extend2's max_ins/max_del, bwa_gen_cigar2, infer_bw)."""
    def c_div(a, d):   # C: truncation toward zero
        q = abs(a) // d
        return q if a >= 0 else -q
    for d in range(1, 70):
        for k in (1, 2):
            for x in list(range(-3000, 3001)) + [2 ** 30 - 7, -(2 ** 30) + 5]:
                assert c_div(x + k * d, d) == int(x / d + k), (x, d, k)
