"""The oracle's extension trace (orc_ext_trace, ORC_PROFILE builds), which tools/ext_model.py replays to choose
k_extend's read order.  CPU only: a profile build of oracle/bwa_oracle.c in a
temporary directory, loaded on its own (the suite's cached oracle library is not touched)."""
import ctypes
import os
import random
import subprocess

import pytest

import oracle_py as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def prof_lib(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("orcprof") / "liboracle_prof.so")
    subprocess.run(["gcc", "-O1", "-fPIC", "-shared", "-DORC_PROFILE", "-o", so,
                    os.path.join(ROOT, "oracle", "bwa_oracle.c"), "-lpthread", "-lm"], check=True)
    L = ctypes.CDLL(so)
    P = ctypes.c_void_p
    for name, res, args in (
            ("orc_nuclseq_from_text", P, [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]),
            ("orc_free", None, [P]),
            ("orc_index_new", P, []),
            ("orc_index_free", None, [P]),
            ("orc_index_add_ref", None, [P, ctypes.c_int64, P]),
            ("orc_index_build", ctypes.c_int, [P]),
            ("orc_profile_get", None, [ctypes.POINTER(ctypes.c_uint64)]),
            ("orc_ext_trace", ctypes.c_int, [P, ctypes.POINTER(O.OrcOpts), P, ctypes.c_int, ctypes.c_int64,
                                             ctypes.POINTER(ctypes.c_int32), ctypes.c_int])):
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    return L


def test_ext_trace_records_one_sided_extension(prof_lib):
    L = prof_lib
    rng = random.Random(7)
    text = "".join(rng.choice("ACGT") for _ in range(20000))
    size = ctypes.c_size_t()
    p = L.orc_nuclseq_from_text(text.encode(), len(text), ctypes.byref(size))
    raw = ctypes.create_string_buffer(ctypes.string_at(p, size.value), size.value)
    L.orc_free(p)
    idx = L.orc_index_new()
    try:
        L.orc_index_add_ref(idx, 1, ctypes.addressof(raw))
        assert L.orc_index_build(idx) == 0
        # 100 bases from position 5000 with one mismatch at query position 70: the longest seed is [0, 70), so the
        # read is extended to the right only (through the mismatch and the remaining 29 bases)
        read = list(text[5000:5100])
        read[70] = {"A": "C", "C": "G", "G": "T", "T": "A"}[read[70]]
        codes = bytes("ACGT".index(c) for c in read)
        qb = ctypes.create_string_buffer(codes, len(codes))
        opts = O.OrcOpts(19, 500, 1, 4, 5, 5, 100, 100, 6, 6, 1, 1)
        before = (ctypes.c_uint64 * 20)()
        L.orc_profile_get(before)
        cap = 1 << 16
        buf = (ctypes.c_int32 * cap)()
        m = L.orc_ext_trace(idx, ctypes.byref(opts), ctypes.addressof(qb), len(codes), 0, buf, cap)
        after = (ctypes.c_uint64 * 20)()
        L.orc_profile_get(after)
    finally:
        L.orc_index_free(idx)
    assert 0 < m < cap and m % 4 == 0
    recs = [tuple(buf[k:k + 4]) for k in range(0, m, 4)]
    ext = [r for r in recs if r[0] >= 10]   # kinds 1-4 are the seeding trace
    chains = [r for r in ext if r[0] == 20]
    seeds = [r for r in ext if r[0] == 21]
    sides = [r[1] for r in ext if r[0] == 22]
    calls = [r for r in ext if r[0] == 10]
    rows = [r for r in ext if r[0] == 11]
    assert len(chains) == 1 and chains[0][1] >= 1 and chains[0][2] == 70   # seeds, longest seed
    first = next(r for r in seeds if r[1] == 0)
    assert (first[2], first[3]) == (0, 70)   # the first extended seed: qbeg 0, 70 bases
    assert sides == [1] and len(calls) >= 1 and calls[0][1] == 30   # right side only, query window 30 bases
    # every row of every ksw_extend2 call is recorded, with its band's cells
    assert len(rows) == after[16] - before[16]
    assert sum(r[1] for r in rows) == after[17] - before[17]
    assert all(r[1] == max(r[3] - r[2], 0) for r in rows)
