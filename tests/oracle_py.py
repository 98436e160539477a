"""ctypes bindings of the CPU oracle (oracle/liboracle.so).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module, as the
checker / CPU baseline of the alignment path (see oracle/oracle.h for what it restates).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB = os.path.join(ORACLE_DIR, "liboracle.so")


class OrcOpts(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "min_seed_len", "max_occ", "a", "b", "pen_clip3", "pen_clip5", "zdrop", "w", "o_del", "e_del", "o_ins",
        "e_ins")]


class OrcRegion(ctypes.Structure):
    _fields_ = [("rb", ctypes.c_int64), ("re", ctypes.c_int64)] + [(n, ctypes.c_int32) for n in (
        "qb", "qe", "rid", "score", "truesc", "sub", "csub", "sub_n", "w", "seedcov", "secondary", "seedlen0",
        "n_comp", "flag", "is_rev", "n_cigar")] + [("cigar", ctypes.c_uint32 * 64), ("hash", ctypes.c_uint64)]


_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        sig = {
            "orc_nuclseq_from_text": (P, [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]),
            "orc_nuclseq_to_text": (P, [P]),
            "orc_free": (None, [P]),
            "orc_index_new": (P, []),
            "orc_index_free": (None, [P]),
            "orc_index_add_ref": (None, [P, ctypes.c_int64, P]),
            "orc_index_build": (ctypes.c_int, [P]),
            "orc_index_build_from_sa": (ctypes.c_int, [P, P, ctypes.c_int]),
            "orc_sa_violations": (ctypes.c_uint64, []),
            "orc_index_l_pac": (ctypes.c_int64, [P]),
            "orc_index_seq_len": (ctypes.c_int64, [P]),
            "orc_index_primary": (ctypes.c_int64, [P]),
            "orc_index_occ4": (None, [P, ctypes.c_int64, ctypes.POINTER(ctypes.c_uint64)]),
            "orc_index_sa": (ctypes.c_int64, [P, ctypes.c_int64]),
            "orc_index_l2": (None, [P, ctypes.POINTER(ctypes.c_uint64)]),
            "orc_index_pac_base": (ctypes.c_int, [P, ctypes.c_int64]),
            "orc_lrand48_at": (ctypes.c_int64, [ctypes.c_uint64]),
            "orc_align_tsv": (P, [P, ctypes.POINTER(OrcOpts), P, ctypes.c_int64]),
            "orc_align_regions": (ctypes.c_int, [P, ctypes.POINTER(OrcOpts), P, ctypes.c_int, ctypes.c_int64,
                                                 ctypes.POINTER(OrcRegion), ctypes.c_int]),
            "orc_collect_intv": (ctypes.c_int, [P, ctypes.POINTER(OrcOpts), P, ctypes.c_int,
                                                ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]),
            "orc_seed_batch": (ctypes.c_int64, [P, ctypes.POINTER(OrcOpts), P, P, ctypes.c_int, ctypes.c_int,
                                                ctypes.POINTER(ctypes.c_uint64)]),
            "orc_align_batch": (ctypes.c_int64, [P, ctypes.POINTER(OrcOpts), P, P, ctypes.c_int, ctypes.c_uint64,
                                                 ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]),
            "orc_algo_bytes": (None, [ctypes.POINTER(ctypes.c_uint64)]),
            "orc_ksw_align2_score": (ctypes.c_int, [ctypes.c_int, P, ctypes.c_int, P, P] + [ctypes.c_int] * 4),
            "orc_ksw_extend2": (ctypes.c_int, [ctypes.c_int, P, ctypes.c_int, P, P] + [ctypes.c_int] * 8 +
                                [ctypes.POINTER(ctypes.c_int)] * 5),
            "orc_ksw_global2": (ctypes.c_int, [ctypes.c_int, P, ctypes.c_int, P, P] + [ctypes.c_int] * 5 +
                                [ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_uint32), ctypes.c_int]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def opts_from(o) -> OrcOpts:
    return OrcOpts(*[getattr(o, n) for n, _ in OrcOpts._fields_])


class Nuclseq:
    """Oracle-side nuclseq value (varlena bytes produced by the oracle's restated codec)."""

    def __init__(self, text: str):
        size = ctypes.c_size_t()
        b = text.encode("latin-1")
        p = lib().orc_nuclseq_from_text(b, len(b), ctypes.byref(size))
        self.raw = ctypes.string_at(p, size.value)
        lib().orc_free(p)
        self._buf = ctypes.create_string_buffer(self.raw, len(self.raw))

    @property
    def ptr(self) -> int:
        return ctypes.addressof(self._buf)

    def to_text(self) -> str:
        p = lib().orc_nuclseq_to_text(self.ptr)
        t = ctypes.string_at(p).decode("latin-1")
        lib().orc_free(p)
        return t


class OracleIndex:
    def __init__(self):
        self.h = lib().orc_index_new()
        self._keep = []

    def __del__(self):
        if getattr(self, "h", None):
            try:
                lib().orc_index_free(self.h)
            except Exception:   # interpreter shutdown
                pass
            self.h = None

    def add_ref(self, ref_id: int, raw: bytes) -> None:
        buf = ctypes.create_string_buffer(raw, len(raw))
        self._keep.append(buf)
        lib().orc_index_add_ref(self.h, ref_id, ctypes.addressof(buf))

    def build(self) -> None:
        assert lib().orc_index_build(self.h) == 0

    def build_from_sa(self, sa_ptr: int, elem_bytes: int) -> dict:
        """FM tables from an outside suffix array, certified on the host first (range, one primary row,
        adjacent suffixes strictly increasing => the unique SA of T$); returns the certificate."""
        import time
        t0 = time.perf_counter()
        rc = lib().orc_index_build_from_sa(self.h, sa_ptr, elem_bytes)
        cert = {"suffixes": self.seq_len + 1 if rc == 0 else None, "violations": int(lib().orc_sa_violations()),
                "rc": rc, "host_s": round(time.perf_counter() - t0, 2)}
        assert rc == 0, f"suffix array rejected by the host certificate: {cert}"
        return cert

    @property
    def l_pac(self) -> int:
        return lib().orc_index_l_pac(self.h)

    @property
    def seq_len(self) -> int:
        return lib().orc_index_seq_len(self.h)

    @property
    def primary(self) -> int:
        return lib().orc_index_primary(self.h)

    def sa(self, row: int) -> int:
        return lib().orc_index_sa(self.h, row)

    def occ4(self, k: int):
        c = (ctypes.c_uint64 * 4)()
        lib().orc_index_occ4(self.h, k, c)
        return list(c)

    def l2(self):
        c = (ctypes.c_uint64 * 5)()
        lib().orc_index_l2(self.h, c)
        return list(c)

    def align_tsv(self, opts: OrcOpts, raw_read: bytes, lrand_id: int) -> str:
        buf = ctypes.create_string_buffer(raw_read, len(raw_read))
        p = lib().orc_align_tsv(self.h, ctypes.byref(opts), ctypes.addressof(buf), lrand_id)
        if not p:
            raise RuntimeError("oracle: unsupported read")
        t = ctypes.string_at(p).decode("latin-1")
        lib().orc_free(p)
        return t

    def regions(self, opts: OrcOpts, codes: bytes, lrand_id: int, max_regs: int = 256):
        out = (OrcRegion * max_regs)()
        buf = ctypes.create_string_buffer(codes, max(len(codes), 1))
        n = lib().orc_align_regions(self.h, ctypes.byref(opts), ctypes.addressof(buf), len(codes), lrand_id, out,
                                    max_regs)
        return [out[i] for i in range(min(n, max_regs))]

    def collect_intv(self, opts: OrcOpts, codes: bytes, max_n: int = 4096):
        out = (ctypes.c_uint64 * (4 * max_n))()
        buf = ctypes.create_string_buffer(codes, max(len(codes), 1))
        n = lib().orc_collect_intv(self.h, ctypes.byref(opts), ctypes.addressof(buf), len(codes), out, max_n)
        return [tuple(out[4 * i:4 * i + 4]) for i in range(min(n, max_n))]


def lrand48_at(pos: int) -> int:
    return lib().orc_lrand48_at(pos)
