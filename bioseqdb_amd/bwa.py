"""Host-side mirror of bioseqdb's alignment interface over the libbsq C-ABI.

Reference interface being mirrored (same names, argument meaning and error behaviour):
  * ``NucleotideSequence`` / ``nuclseq_in``            bioseqdb/sequence.h:18-38, extension.cpp:46-61
  * ``bwa_opts()`` incl. the ROW field-order quirk Q1  bioseqdb/bioseqdb--0.0.0.sql:160-194
  * ``BwaIndex`` (add_ref_sequence/build/align_sequence) bioseqdb/bwa.h:32-48, bwa.cpp:80-181
  * ``BwaMatch`` / ``bwa_result`` rows                  bwa.h:15-30, bioseqdb--0.0.0.sql:196-212
  * ``nuclseq_search_bwa`` / ``nuclseq_multi_search_bwa`` extension.cpp:311-378
The SQL strings of the reference become Python iterables of ``(id, nuclseq)`` rows (the SPI cursor
of extension.cpp:156-195); rows with a NULL (None) id or sequence are skipped, non-integer ids raise
``DatatypeMismatch`` like ``expected column of integers``.  All alignment work runs in the HIP
kernels of libbsq; without a GPU, aligning raises ``BsqError`` (no CPU fallback).
"""
from __future__ import annotations

import ctypes
import dataclasses
import hashlib
import os
import re
import struct
from collections import OrderedDict
from typing import Iterable, Iterator, List, Optional, Sequence, Tuple

from . import _native
from ._native import BsqError, Opts, check, lib

ALLOWED_NUCLEOTIDES = "ACGTNWSMKRYBDHV"   # sequence.h:46
_INVALID_NUCLEOTIDE = re.compile(f"[^{ALLOWED_NUCLEOTIDES}]", re.S)


class InvalidTextRepresentation(ValueError):
    pass


class InvalidParameterValue(ValueError):
    pass


class DatatypeMismatch(TypeError):
    pass


class NucleotideSequence:
    """A ``nuclseq`` value: the exact varlena bytes of sequence.h:18-38."""

    __slots__ = ("raw", "_buf")

    def __init__(self, raw: bytes):
        self.raw = bytes(raw)
        self._buf = ctypes.create_string_buffer(self.raw, len(self.raw))

    @classmethod
    def from_text(cls, text: str) -> "NucleotideSequence":
        """nuclseq_in (extension.cpp:46-61): validates the alphabet then nuclseq_from_text."""
        if len(text) > 0x7FFFFFFF // 4:
            raise InvalidParameterValue("provided sequence is too long")
        bad = _INVALID_NUCLEOTIDE.search(text)
        if bad:
            raise InvalidTextRepresentation(f"invalid nucleotide in nuclseq_in: '{bad.group(0)}'")
        return cls._encode(text)

    @classmethod
    def _encode(cls, text: str) -> "NucleotideSequence":
        b = text.encode("latin-1")
        size = ctypes.c_size_t()
        p = lib().bsq_nuclseq_from_text(b, len(b), ctypes.byref(size))
        if not p:
            raise MemoryError("bsq_nuclseq_from_text failed")
        try:
            return cls(ctypes.string_at(p, size.value))
        finally:
            lib().bsq_free(p)

    @property
    def ptr(self) -> int:
        return ctypes.addressof(self._buf)

    def __len__(self) -> int:
        return int.from_bytes(self.raw[8:12], "little")

    @property
    def holes_num(self) -> int:
        return int.from_bytes(self.raw[4:8], "little")

    def to_text(self) -> str:
        p = lib().bsq_nuclseq_to_text(self.ptr)
        try:
            return ctypes.string_at(p).decode("latin-1")
        finally:
            lib().bsq_free(p)

    def __str__(self) -> str:
        return self.to_text()

    def __repr__(self) -> str:
        t = self.to_text()
        return f"NucleotideSequence({t[:20]!r}{'...' if len(t) > 20 else ''})"

    def __eq__(self, other) -> bool:
        return isinstance(other, NucleotideSequence) and self.raw == other.raw

    def __hash__(self) -> int:
        return hash(self.raw)


@dataclasses.dataclass(frozen=True)
class BwaOptions:
    """The SQL composite ``bwa_options`` (bioseqdb--0.0.0.sql:160-173), field order included."""

    min_seed_len: Optional[int] = 19
    max_occ: Optional[int] = None
    match_score: Optional[int] = 1
    mismatch_penalty: Optional[int] = 4
    pen_clip3: Optional[int] = 5
    pen_clip5: Optional[int] = 5
    zdrop: Optional[int] = 100
    bandwidth: Optional[int] = 100
    o_del: Optional[int] = 6
    e_del: Optional[int] = 1
    o_ins: Optional[int] = 6
    e_ins: Optional[int] = 1


def bwa_opts(min_seed_len=19, max_occ=None, match_score=1, mismatch_penalty=4, pen_clip3=5, pen_clip5=5,
             zdrop=100, bandwidth=100, o_del=6, o_ins=6, e_del=1, e_ins=1) -> BwaOptions:
    """``bwa_opts()`` (bioseqdb--0.0.0.sql:175-194).

    Reproduces quirk Q1: the function builds ``ROW(..., o_del, o_ins, e_del, e_ins)`` but the type's
    fields are ``(..., o_del, e_del, o_ins, e_ins)``; the positional ROW->composite cast therefore
    stores the ``o_ins`` argument in ``e_del`` and the ``e_del`` argument in ``o_ins``.
    """
    return BwaOptions(min_seed_len, max_occ, match_score, mismatch_penalty, pen_clip3, pen_clip5, zdrop,
                      bandwidth, o_del, o_ins, e_del, e_ins)


def effective_opts(opts: Optional[BwaOptions], n_refs: int) -> Opts:
    """get_opt_or over the composite (extension.cpp:197-231): NULL -> default, negative -> error."""
    if opts is None:
        opts = bwa_opts()

    def get(name: str, default: int) -> int:
        v = getattr(opts, name)
        if v is None:
            return default
        v = int(v)
        if v < 0:
            raise InvalidParameterValue(f"bwa_opt {name} must be nonnegative")
        return v

    return Opts(
        min_seed_len=get("min_seed_len", 19), max_occ=get("max_occ", max(500, n_refs * 2)),
        a=get("match_score", 1), b=get("mismatch_penalty", 4), pen_clip3=get("pen_clip3", 5),
        pen_clip5=get("pen_clip5", 5), zdrop=get("zdrop", 100), w=get("bandwidth", 100),
        o_del=get("o_del", 6), e_del=get("e_del", 1), o_ins=get("o_ins", 6), e_ins=get("e_ins", 1))


@dataclasses.dataclass
class BwaMatch:
    """bwa.h:15-30; together with query_id one ``bwa_result`` row."""

    ref_id: int
    ref_subseq: str
    ref_match_begin: int
    ref_match_end: int
    ref_match_len: int
    query_subseq: str
    query_match_begin: int
    query_match_end: int
    query_match_len: int
    is_primary: bool
    is_secondary: bool
    is_reverse: bool
    cigar: str
    score: int


BWA_RESULT_COLUMNS = ("ref_id", "ref_subseq", "ref_match_start", "ref_match_end", "ref_match_len", "query_id",
                      "query_subseq", "query_match_start", "query_match_end", "query_match_len", "is_primary",
                      "is_secondary", "is_reverse", "cigar", "score")


class _CallCounter:
    """Position in the backend's lrand48 stream: mem_align1 draws one value per call (Q10)."""

    value = 0


def lrand48_calls() -> int:
    return _CallCounter.value


def reset_lrand48(calls: int = 0) -> None:
    _CallCounter.value = int(calls)


def parse_tsv(tsv: str) -> List[BwaMatch]:
    out = []
    for line in tsv.splitlines():
        f = line.split("\t")
        out.append(BwaMatch(int(f[0]), f[1], int(f[2]), int(f[3]), int(f[4]), f[5], int(f[6]), int(f[7]),
                            int(f[8]), f[9] == "t", f[10] == "t", f[11] == "t", f[12], int(f[13])))
    return out


class BwaIndex:
    """bwa.h:32-48 over libbsq: references are concatenated on the host, indexed, copied to HBM once."""

    def __init__(self, device: int = 0):
        h = ctypes.c_void_p()
        check(lib().bsq_index_create(ctypes.byref(h)))
        self._h = h
        self._refs: List[NucleotideSequence] = []
        self.device = device
        self.options: Optional[Opts] = None
        self._uploaded = False
        self._built = False

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                lib().bsq_index_free(h)
            except Exception:   # interpreter shutdown (cached indexes): the process releases everything
                pass
            self._h = None

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._h

    def add_ref_sequence(self, ref_id: int, seq: NucleotideSequence) -> None:
        check(lib().bsq_index_add_ref(self._h, int(ref_id), seq.ptr))
        self._refs.append(seq)

    def build(self, threads: int = 0) -> None:
        check(lib().bsq_index_build(self._h, threads))
        self._built = True

    def build_on_device(self) -> None:
        """BwaIndex::build on the GPU (suffix sort + BWT in HBM); leaves it uploaded."""
        check(lib().bsq_index_build_device(self._h, self.device))
        self._built = True
        self._uploaded = True

    def certify_sa(self) -> dict:
        """The device certificate of the suffix array in HBM (bsq_index_certify_sa): range, every position
        once, adjacent suffixes strictly increasing; violations == 0 proves it is the SA of T$."""
        import time
        n, bad = ctypes.c_uint64(), ctypes.c_uint64()
        t0 = time.perf_counter()
        check(lib().bsq_index_certify_sa(self._h, ctypes.byref(n), ctypes.byref(bad)))
        return {"suffixes": int(n.value), "violations": int(bad.value),
                "device_s": round(time.perf_counter() - t0, 3)}

    def upload(self) -> None:
        if not self._uploaded and self.l_pac > 0:
            check(lib().bsq_index_upload(self._h, self.device))
            self._uploaded = True

    @property
    def l_pac(self) -> int:
        return lib().bsq_index_l_pac(self._h)

    @property
    def n_refs(self) -> int:
        return lib().bsq_index_n_refs(self._h)

    def align_sequences(self, seqs: Sequence[NucleotideSequence], opts: Opts,
                        first_call: Optional[int] = None) -> List[List[BwaMatch]]:
        """BwaIndex::align_sequence for a cursor batch; consumes one lrand48 value per read."""
        n = len(seqs)
        if self.l_pac <= 0:   # bwa.cpp:142-143: empty reference -> no matches, no mem_align1 call
            return [[] for _ in range(n)]
        self.upload()
        if first_call is None:
            first_call = _CallCounter.value
        arr = (ctypes.c_void_p * max(n, 1))(*[s.ptr for s in seqs])
        out = ctypes.POINTER(_native.Hits)()
        check(lib().bsq_align_batch(self._h, ctypes.byref(opts), arr, n, first_call, ctypes.byref(out)))
        try:
            p = lib().bsq_render_tsv(self._h, out, arr)
            try:
                text = ctypes.string_at(p).decode("latin-1")
            finally:
                lib().bsq_free(p)
            rows = parse_tsv(text)
            res: List[List[BwaMatch]] = [[] for _ in range(n)]
            it = iter(rows)
            for i in range(n):
                cnt = out.contents.read_off[i + 1] - out.contents.read_off[i]
                res[i] = [next(it) for _ in range(cnt)]
        finally:
            lib().bsq_hits_free(out)
        _CallCounter.value = first_call + n
        return res

    def align_sequence(self, seq: NucleotideSequence, opts: Optional[Opts] = None) -> List[BwaMatch]:
        return self.align_sequences([seq], opts or self.options or effective_opts(None, self.n_refs))[0]


Row = Tuple[Optional[int], Optional[NucleotideSequence]]


def _iterate_nuclseq_table(rows: Iterable[Row]) -> Iterator[Tuple[int, NucleotideSequence]]:
    """iterate_nuclseq_table (extension.cpp:156-195): type checks, NULLs skipped."""
    for row in rows:
        rid, seq = row[0], row[1]
        if rid is not None and not isinstance(rid, int):
            raise DatatypeMismatch("expected column of integers")
        if seq is not None and not isinstance(seq, NucleotideSequence):
            raise DatatypeMismatch("expected column of nuclseqs")
        if rid is None or seq is None:
            continue
        yield rid, seq


class _IndexCache:
    """Cross-call index cache: the reference rebuilds the index from
    ``reference_sql`` on every call (extension.cpp:326,359); here an index is keyed by a digest of its
    rows (ids and nuclseq bytes, in cursor order) and the device, so repeated calls over the same
    reference skip the build and the upload.  Options are per call and are not part of the key.
    ``BSQ_INDEX_CACHE`` = number of indexes kept (default 2, 0 disables)."""

    def __init__(self):
        self._d: "OrderedDict[tuple, BwaIndex]" = OrderedDict()
        self.hits = 0
        self.builds = 0

    @staticmethod
    def capacity() -> int:
        return max(0, int(os.environ.get("BSQ_INDEX_CACHE", "2")))

    def get(self, rows: List[Tuple[int, NucleotideSequence]], device: int) -> BwaIndex:
        h = hashlib.blake2b(digest_size=20)
        for rid, seq in rows:
            h.update(struct.pack("<qQ", rid, len(seq.raw)))
            h.update(seq.raw)
        key = (h.digest(), len(rows), device)
        cap = self.capacity()
        if cap and key in self._d:
            self._d.move_to_end(key)
            self.hits += 1
            return self._d[key]
        idx = BwaIndex(device)
        for rid, seq in rows:
            idx.add_ref_sequence(rid, seq)
        if rows and lib().bsq_device_count() > device:
            idx.build_on_device()   # suffix sort + BWT in HBM (bsq_index_build_device)
        else:
            idx.build()             # same tables from the host build (alignment itself needs the GPU)
        self.builds += 1
        if cap:
            self._d[key] = idx
            while len(self._d) > cap:
                self._d.popitem(last=False)
        return idx

    def clear(self) -> None:
        self._d.clear()
        self.hits = self.builds = 0


INDEX_CACHE = _IndexCache()


def bwa_index_from_query(reference_rows: Iterable[Row], opts: Optional[BwaOptions], device: int = 0) -> BwaIndex:
    """bwa_index_from_query (extension.cpp:211-236), through the cross-call cache."""
    rows = list(_iterate_nuclseq_table(reference_rows))
    idx = INDEX_CACHE.get(rows, device)
    idx.options = effective_opts(opts, len(rows))
    return idx


def _rows(query_id: Optional[int], matches: List[BwaMatch]) -> List[tuple]:
    """build_tuple_bwa (extension.cpp:282-305): query_id NULL for the single-query function."""
    return [(m.ref_id, m.ref_subseq, m.ref_match_begin, m.ref_match_end, m.ref_match_len, query_id,
             m.query_subseq, m.query_match_begin, m.query_match_end, m.query_match_len, m.is_primary,
             m.is_secondary, m.is_reverse, m.cigar, m.score) for m in matches]


def nuclseq_search_bwa(query_sequence: NucleotideSequence, reference_rows: Iterable[Row],
                       opts: Optional[BwaOptions] = None, device: int = 0) -> List[tuple]:
    """nuclseq_search_bwa(NUCLSEQ, CSTRING, bwa_options) RETURNS SETOF bwa_result (extension.cpp:311-343)."""
    if query_sequence is None:   # LANGUAGE C STRICT
        return []
    idx = bwa_index_from_query(reference_rows, opts, device)
    return _rows(None, idx.align_sequence(query_sequence))


def nuclseq_multi_search_bwa(query_rows: Iterable[Row], reference_rows: Iterable[Row],
                             opts: Optional[BwaOptions] = None, device: int = 0,
                             batch_reads: int = 1 << 20) -> List[tuple]:
    """nuclseq_multi_search_bwa(CSTRING, CSTRING, bwa_options) (extension.cpp:345-378).

    The reference fetches the query cursor one row at a time; here rows are aligned in batches of
    ``batch_reads`` on the GPU with identical per-read results and lrand48 stream positions."""
    idx = bwa_index_from_query(reference_rows, opts, device)
    out: List[tuple] = []
    ids: List[int] = []
    seqs: List[NucleotideSequence] = []

    def flush():
        if seqs:
            for qid, ms in zip(ids, idx.align_sequences(seqs, idx.options)):
                out.extend(_rows(qid, ms))
            ids.clear()
            seqs.clear()

    for qid, seq in _iterate_nuclseq_table(query_rows):
        ids.append(qid)
        seqs.append(seq)
        if len(seqs) >= batch_reads:
            flush()
    flush()
    return out
