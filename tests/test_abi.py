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
