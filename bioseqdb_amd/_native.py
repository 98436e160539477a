"""ctypes bindings of libbsq.so (include/bsq.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (``make -C bioseqdb_amd/csrc``).
Loading fails loudly when it is missing: the alignment path has no Python or CPU fallback.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BSQ_LIB") or os.path.join(_HERE, "libbsq.so")   # BSQ_LIB: experiment builds only

BSQ_OK = 0
BSQ_E_INVALID = -1
BSQ_E_NOMEM = -2
BSQ_E_HIP = -3
BSQ_E_NODEV = -4
BSQ_E_UNSUPPORTED = -5


class BsqError(RuntimeError):
    """Raised for a negative libbsq status code (mirrors the reference's ereport(ERROR))."""

    def __init__(self, code: int, message: str):
        super().__init__(f"libbsq error {code}: {message}")
        self.code = code


class Opts(ctypes.Structure):
    """bsq_opts: the effective mem_opt_t fields (extension.cpp:220-231)."""

    _fields_ = [(n, ctypes.c_int32) for n in (
        "min_seed_len", "max_occ", "a", "b", "pen_clip3", "pen_clip5", "zdrop", "w",
        "o_del", "e_del", "o_ins", "e_ins")]


class Hit(ctypes.Structure):
    _fields_ = [
        ("ref_id", ctypes.c_int64), ("rb", ctypes.c_int64), ("re", ctypes.c_int64),
        ("ref_match_start", ctypes.c_int32), ("ref_match_end", ctypes.c_int32),
        ("ref_match_len", ctypes.c_int32), ("qb", ctypes.c_int32), ("qe", ctypes.c_int32),
        ("score", ctypes.c_int32), ("rid", ctypes.c_int32),
        ("is_primary", ctypes.c_uint8), ("is_secondary", ctypes.c_uint8),
        ("is_reverse", ctypes.c_uint8), ("pad0", ctypes.c_uint8),
        ("read_index", ctypes.c_int32), ("cigar_off", ctypes.c_uint32), ("n_cigar", ctypes.c_uint32),
    ]


class Table(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("bytes", ctypes.c_uint64)]


N_TABLES = 8


class Hits(ctypes.Structure):
    _fields_ = [
        ("n_reads", ctypes.c_int32), ("n_hits", ctypes.c_int64), ("hits", ctypes.POINTER(Hit)),
        ("read_off", ctypes.POINTER(ctypes.c_int64)), ("n_cigar", ctypes.c_int64),
        ("cigar", ctypes.POINTER(ctypes.c_uint32)),
    ]


# every symbol include/bsq.h declares: name -> (restype, argtypes)
_P = ctypes.c_void_p
SIGNATURES = {
    "bsq_last_error": (ctypes.c_char_p, []),
    "bsq_version": (ctypes.c_char_p, []),
    "bsq_device_count": (ctypes.c_int, []),
    "bsq_nuclseq_from_text": (_P, [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]),
    "bsq_nuclseq_to_text": (_P, [_P]),
    "bsq_index_create": (ctypes.c_int, [ctypes.POINTER(_P)]),
    "bsq_index_free": (None, [_P]),
    "bsq_index_add_ref": (ctypes.c_int, [_P, ctypes.c_int64, _P]),
    "bsq_index_build": (ctypes.c_int, [_P, ctypes.c_int]),
    "bsq_index_upload": (ctypes.c_int, [_P, ctypes.c_int]),
    "bsq_index_l_pac": (ctypes.c_int64, [_P]),
    "bsq_index_seq_len": (ctypes.c_int64, [_P]),
    "bsq_index_primary": (ctypes.c_int64, [_P]),
    "bsq_index_n_refs": (ctypes.c_int32, [_P]),
    "bsq_index_same_refs": (ctypes.c_int, [_P, _P]),
    "bsq_index_sa": (ctypes.c_int64, [_P, ctypes.c_int64]),
    "bsq_index_occ4": (ctypes.c_int, [_P, ctypes.c_int64, ctypes.POINTER(ctypes.c_uint64)]),
    "bsq_index_sa_data": (_P, [_P, ctypes.POINTER(ctypes.c_int)]),
    "bsq_lrand48_at": (ctypes.c_int64, [ctypes.c_uint64]),
    "bsq_align_batch": (ctypes.c_int, [_P, ctypes.POINTER(Opts), ctypes.POINTER(_P), ctypes.c_int32,
                                       ctypes.c_uint64, ctypes.POINTER(ctypes.POINTER(Hits))]),
    "bsq_hits_free": (None, [ctypes.POINTER(Hits)]),
    "bsq_index_release_pool": (ctypes.c_int, [_P]),
    "bsq_render_tsv": (_P, [_P, ctypes.POINTER(Hits), ctypes.POINTER(_P)]),
    "bsq_index_ref_subseq": (ctypes.c_int64, [_P, ctypes.c_int64, ctypes.c_int64, ctypes.c_char_p]),
    "bsq_free": (None, [_P]),
    "bsq_batch_create": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int64, ctypes.POINTER(_P)]),
    "bsq_batch_free": (None, [_P]),
    "bsq_batch_set_reads": (ctypes.c_int, [_P, _P, _P, ctypes.c_int32]),
    "bsq_batch_run": (ctypes.c_int, [_P, ctypes.POINTER(Opts), ctypes.c_uint64]),
    "bsq_batch_hits": (ctypes.POINTER(Hits), [_P]),
    "bsq_batch_stage_ms": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_float), ctypes.c_int]),
    "bsq_stage_name": (ctypes.c_char_p, [ctypes.c_int]),
    "bsq_batch_stage_bytes": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_double), ctypes.c_int]),
    "bsq_batch_stage_work": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_double), ctypes.c_int]),
    "bsq_batch_seed": (ctypes.c_int, [_P, _P]),
    "bsq_index_layout": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64), _P, ctypes.POINTER(ctypes.c_uint64)]),
    "bsq_index_upload_into": (ctypes.c_int, [_P, ctypes.c_int, _P, ctypes.c_int]),
    "bsq_index_import": (ctypes.c_int, [_P, ctypes.c_uint64, ctypes.c_int, _P, ctypes.c_int, ctypes.POINTER(_P)]),
    "bsq_batch_intervals": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.POINTER(ctypes.c_int64)),
                                           ctypes.POINTER(ctypes.POINTER(ctypes.c_uint64)),
                                           ctypes.POINTER(ctypes.c_int64)]),
    "bsq_batch_retried": (ctypes.c_int64, [_P]),
    "bsq_batch_sort_guard": (ctypes.c_int64, [_P]),
    "bsq_sort_guard_total": (ctypes.c_int64, []),
    "bsq_batch_copy_records": (ctypes.c_int, [_P, _P, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]),
    "bsq_index_build_device": (ctypes.c_int, [_P, ctypes.c_int]),
    "bsq_batch_run_many": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_int, ctypes.POINTER(Opts),
                                          ctypes.POINTER(ctypes.c_uint64)]),
    "bsq_batch_run_rounds": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_int, ctypes.POINTER(Opts),
                                            ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]),
    "bsq_batch_render": (ctypes.c_int, [_P, _P, ctypes.POINTER(_P), ctypes.POINTER(ctypes.c_int64)]),
    "bsq_index_download": (ctypes.c_int, [_P]),
    "bsq_index_build_stats": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_uint64)]),
    "bsq_index_certify_sa": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "bsq_nuclseq_encode_batch": (ctypes.c_int, [ctypes.c_int, _P, _P, ctypes.c_int64, ctypes.c_int,
                                                ctypes.POINTER(_P), ctypes.POINTER(_P)]),
    "bsq_nuclseq_decode_batch": (ctypes.c_int, [ctypes.c_int, _P, ctypes.c_int64, ctypes.POINTER(_P),
                                                ctypes.POINTER(_P)]),
    "bsq_nuclseq_codec_ms": (ctypes.c_int, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
    "bsq_batch_set_nuclseqs": (ctypes.c_int, [_P, _P, ctypes.c_int32]),
    "bsq_batch_render_nuclseqs": (ctypes.c_int, [_P, _P, ctypes.POINTER(_P), ctypes.POINTER(_P)]),
    "bsq_fasta_parse": (ctypes.c_int, [_P, ctypes.c_int64, ctypes.POINTER(_P), ctypes.POINTER(_P), ctypes.POINTER(_P),
                                       ctypes.POINTER(_P), ctypes.POINTER(ctypes.c_int64)]),
    "bsq_index_device_tables": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int), _P, ctypes.c_int]),
    "bsq_group_create": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.POINTER(_P)]),
    "bsq_group_free": (None, [_P]),
    "bsq_group_size": (ctypes.c_int, [_P]),
    "bsq_group_replicate": (ctypes.c_int, [_P, _P, ctypes.POINTER(ctypes.c_double)]),
    "bsq_group_run": (ctypes.c_int, [_P, ctypes.POINTER(Opts), _P, ctypes.c_int32, ctypes.c_uint64]),
    "bsq_group_hits": (ctypes.POINTER(Hits), [_P]),
    "bsq_group_render_nuclseqs": (ctypes.c_int, [_P, _P, ctypes.POINTER(_P), ctypes.POINTER(_P)]),
    "bsq_group_set_slots": (ctypes.c_int, [_P, ctypes.c_int]),
    "bsq_group_run_rounds": (ctypes.c_int, [_P, ctypes.POINTER(Opts), ctypes.c_int32, ctypes.c_uint64, ctypes.c_int]),
    "bsq_group_set_exchange": (ctypes.c_int, [_P, ctypes.c_int]),
    "bsq_batch_set_record_route": (ctypes.c_int, [_P, ctypes.c_int]),
    "bsq_xchg_unique_id": (ctypes.c_int, [_P]),
    "bsq_xchg_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, _P, ctypes.c_int, ctypes.POINTER(_P)]),
    "bsq_xchg_free": (None, [_P]),
    "bsq_batch_run_rounds_x": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_int, ctypes.POINTER(Opts),
                                              ctypes.POINTER(ctypes.c_uint64), ctypes.c_int, _P]),
    "bsq_xchg_finish": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double)]),
    "bsq_xchg_view": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int, ctypes.POINTER(Hits)]),
    "bsq_xchg_set_index": (ctypes.c_int, [_P, _P]),
    "bsq_xchg_wire_check": (ctypes.c_int, [_P, _P, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                           ctypes.POINTER(ctypes.c_int64)]),
    "bsq_group_segments": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.POINTER(Hits)), ctypes.POINTER(ctypes.c_int32),
                                          ctypes.c_int]),
    "bsq_pipeline_create": (ctypes.c_int, [_P, ctypes.c_int, ctypes.POINTER(_P)]),
    "bsq_pipeline_free": (None, [_P]),
    "bsq_pipeline_slots": (ctypes.c_int, [_P]),
    "bsq_pipeline_submit": (ctypes.c_int, [_P, ctypes.POINTER(Opts), _P, ctypes.c_int32, ctypes.c_uint64, ctypes.c_int]),
    "bsq_pipeline_next": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.POINTER(Hits)), ctypes.POINTER(_P),
                                         ctypes.POINTER(ctypes.POINTER(ctypes.c_int64))]),
    "bsq_pipeline_release": (ctypes.c_int, [_P]),
    "bsq_pipeline_submit_deferred": (ctypes.c_int, [_P, ctypes.POINTER(Opts), _P, ctypes.c_int32, ctypes.c_uint64,
                                                    ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]),
    "bsq_pipeline_wait_staged": (ctypes.c_int, [_P, ctypes.c_int64]),
}

_lib = None


def lib() -> ctypes.CDLL:
    """Load libbsq.so (fails loudly if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `make -C bioseqdb_amd/csrc` "
                              "(or __graft_entry__.build()); there is no fallback implementation")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(code: int) -> None:
    if code != BSQ_OK:
        raise BsqError(code, lib().bsq_last_error().decode(errors="replace"))
