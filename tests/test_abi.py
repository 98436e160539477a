"""The C-ABI library loads and exports every symbol include/bsq.h declares (no GPU needed)."""
import ctypes
import os
import re

import pytest

from bioseqdb_amd import _native
from bioseqdb_amd import BsqError, BwaIndex, NucleotideSequence

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "bsq.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(bsq_[a-z0-9_]+)\s*\(", src)))


def test_every_declared_symbol_is_exported():
    L = ctypes.CDLL(_native.LIB_PATH)
    names = declared_functions()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_bindings_cover_header():
    assert set(declared_functions()) == set(_native.SIGNATURES)


def test_version_and_lrand48():
    L = _native.lib()
    assert b"gfx950" in L.bsq_version()
    # glibc lrand48 from the unseeded state: 0, 2116118, 89401895, ...
    assert [L.bsq_lrand48_at(i) for i in range(3)] == [0, 2116118, 89401895]


def test_hit_struct_layout_matches_header():
    assert ctypes.sizeof(_native.Hit) == 72   # gcc: sizeof(bsq_hit)
    assert ctypes.sizeof(_native.Opts) == 48


def test_no_device_fails_loudly_without_fallback(gpu_available):
    if gpu_available:
        pytest.skip("GPU present")
    idx = BwaIndex()
    idx.add_ref_sequence(1, NucleotideSequence.from_text("ACGT" * 100))
    idx.build()
    with pytest.raises(BsqError) as e:
        idx.align_sequence(NucleotideSequence.from_text("ACGT" * 10))
    assert e.value.code == _native.BSQ_E_NODEV


def test_index_same_refs_content_check():
    """bsq_index_same_refs, the backend cache's confirmation of a digest hit: same rows -> 1; a changed base,
    id, hole or row order -> 0 (host indexes, no GPU needed)."""
    L = _native.lib()

    def idx(rows):
        h = ctypes.c_void_p()
        _native.check(L.bsq_index_create(ctypes.byref(h)))
        keep = []
        for rid, t in rows:
            ns = NucleotideSequence.from_text(t)
            keep.append(ns)
            _native.check(L.bsq_index_add_ref(h, rid, ns.ptr))
        return h, keep

    base = [(1, "ACGTTGCA" * 50 + "NNNN" + "GATTACA" * 30), (2, "CCGGTTAA" * 40)]
    a, ka = idx(base)
    variants = {
        "same": (base, 1),
        "base": ([(1, "ACGTTGCA" * 50 + "NNNN" + "GATTACA" * 29 + "GATTACC"), base[1]], 0),
        "id": ([(3, base[0][1]), base[1]], 0),
        "hole": ([(1, base[0][1].replace("NNNN", "NNNR")), base[1]], 0),
        "order": ([base[1], base[0]], 0),
    }
    try:
        for name, (rows, want) in variants.items():
            b, kb = idx(rows)
            try:
                assert L.bsq_index_same_refs(a, b) == want, name
            finally:
                L.bsq_index_free(b)
        assert L.bsq_index_same_refs(a, None) == -1
    finally:
        L.bsq_index_free(a)


def test_library_is_up_to_date_with_its_sources():
    """The prebuilt libbsq.so travels to the GPU box as it is: it must not be older than any source or header
    it is built from (make -q: nothing to rebuild)."""
    import shutil
    import subprocess
    if not shutil.which("make"):
        pytest.skip("no make")
    r = subprocess.run(["make", "-q", "-C", os.path.join(ROOT, "bioseqdb_amd", "csrc")], capture_output=True)
    assert r.returncode == 0, "libbsq.so is stale: run make -C bioseqdb_amd/csrc"


def test_index_same_refs_built_vs_fresh():
    """A built (cached) index against a fresh one given the same rows: still the same rows."""
    L = _native.lib()
    a, b = BwaIndex(), BwaIndex()
    for x in (a, b):
        x.add_ref_sequence(7, NucleotideSequence.from_text("ACGTTGCANNGATTACA" * 40))
    a.build()
    assert L.bsq_index_same_refs(a.handle, b.handle) == 1

