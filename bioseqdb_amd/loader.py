"""Bulk nuclseq codec and FASTA loader over libbsq.

Mirrors, for whole batches:
  * ``nuclseq_in`` / ``nuclseq_out`` (bioseqdb/extension.cpp:46-67; sequence.cpp:71-81, 209-245):
    ``nuclseq_in_batch`` / ``nuclseq_out_batch`` run on the GPU (csrc/codec_gpu.hip), with the same
    bytes as the per-value path and the same errors, raised for the first offending text in order;
  * the bioseqdb-import tool (bioseqdb-import/main.cpp:18-76) up to its INSERTs: ``parse_fasta`` gives the
    (name, sequence) records it would insert, ``import_fasta`` also encodes them as nuclseq values.
There is no CPU fallback: without a device the codec raises ``BsqError`` (BSQ_E_NODEV).
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Sequence, Tuple, Union

import numpy as np

from ._native import BsqError, check, lib
from .bwa import InvalidParameterValue, InvalidTextRepresentation, NucleotideSequence

Text = Union[str, bytes]


def _raise(rc: int) -> None:
    if rc == 0:
        return
    msg = lib().bsq_last_error().decode("utf-8", errors="replace")
    if msg.startswith("invalid nucleotide in nuclseq_in"):
        raise InvalidTextRepresentation(msg)
    if msg.startswith("provided sequence is too long"):
        raise InvalidParameterValue(msg)
    check(rc)


def _take(ptr: ctypes.c_void_p, nbytes: int) -> bytes:
    # (ctypes.string_at takes a C int size: texts of 2 GiB and more are copied through a sized array)
    try:
        if not nbytes:
            return b""
        addr = ptr.value if isinstance(ptr, ctypes.c_void_p) else ptr
        return bytes((ctypes.c_char * nbytes).from_address(addr))
    finally:
        lib().bsq_free(ptr)


def _take_i64(ptr: ctypes.c_void_p, count: int) -> np.ndarray:
    try:
        return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_int64)), shape=(count,)).copy()
    finally:
        lib().bsq_free(ptr)


def encode_concat(data: Union[bytes, np.ndarray], offs: np.ndarray, device: int = 0,
                  validate: bool = True) -> Tuple[bytes, np.ndarray]:
    """Concatenated texts (``data[offs[i]:offs[i+1]]``) -> (concatenated varlenas, their offsets)."""
    offs = np.ascontiguousarray(offs, dtype=np.int64)
    n = len(offs) - 1
    buf = data if isinstance(data, np.ndarray) else np.frombuffer(data, dtype=np.uint8)
    buf = np.ascontiguousarray(buf)
    out, oo = ctypes.c_void_p(), ctypes.c_void_p()
    _raise(lib().bsq_nuclseq_encode_batch(device, buf.ctypes.data if buf.size else None, offs.ctypes.data, n,
                                          int(validate), ctypes.byref(out), ctypes.byref(oo)))
    off = _take_i64(oo, n + 1)
    return _take(out, int(off[n])), off


def _split(raw: bytes, off: np.ndarray) -> List[NucleotideSequence]:
    res = []
    for i in range(len(off) - 1):
        a = int(off[i])
        size = int.from_bytes(raw[a:a + 4], "little") >> 2
        res.append(NucleotideSequence(raw[a:a + size]))
    return res


def nuclseq_in_batch(texts: Sequence[Text], device: int = 0, validate: bool = True) -> List[NucleotideSequence]:
    """``nuclseq_in`` of every text, on the GPU."""
    bs = [t.encode("latin-1") if isinstance(t, str) else bytes(t) for t in texts]
    offs = np.zeros(len(bs) + 1, dtype=np.int64)
    if bs:
        offs[1:] = np.cumsum([len(b) for b in bs])
    raw, off = encode_concat(b"".join(bs), offs, device, validate)
    return _split(raw, off)


def nuclseq_out_batch(seqs: Sequence[NucleotideSequence], device: int = 0) -> List[str]:
    """``nuclseq_out`` of every value, on the GPU."""
    n = len(seqs)
    ptrs = (ctypes.c_void_p * max(n, 1))(*[s.ptr for s in seqs])
    txt, to = ctypes.c_void_p(), ctypes.c_void_p()
    _raise(lib().bsq_nuclseq_decode_batch(device, ptrs, n, ctypes.byref(txt), ctypes.byref(to)))
    off = _take_i64(to, n + 1)
    t = _take(txt, int(off[n])).decode("latin-1")
    return [t[int(off[i]):int(off[i + 1])] for i in range(n)]


def codec_ms() -> Tuple[float, float]:
    """(kernel ms, whole-call ms) of this thread's last bulk encode/decode."""
    k, c = ctypes.c_double(), ctypes.c_double()
    lib().bsq_nuclseq_codec_ms(ctypes.byref(k), ctypes.byref(c))
    return k.value, c.value


def parse_fasta_concat(data: bytes) -> Tuple[bytes, np.ndarray, List[str]]:
    """FASTA bytes -> (concatenated sequences, offsets, names) as bioseqdb-import reads them."""
    s, so, nm, no = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    n = ctypes.c_int64()
    rc = lib().bsq_fasta_parse(data, len(data), ctypes.byref(s), ctypes.byref(so), ctypes.byref(nm),
                               ctypes.byref(no), ctypes.byref(n))
    if rc != 0:
        raise BsqError(rc, "bsq_fasta_parse failed")
    soff = _take_i64(so, n.value + 1)
    noff = _take_i64(no, n.value + 1)
    seq = _take(s, int(soff[-1]))
    nb = _take(nm, int(noff[-1]))
    return seq, soff, [nb[int(noff[i]):int(noff[i + 1])].decode("utf-8", errors="surrogateescape")
                       for i in range(n.value)]


def parse_fasta(data: bytes) -> List[Tuple[str, bytes]]:
    seq, off, names = parse_fasta_concat(data)
    return [(names[i], seq[int(off[i]):int(off[i + 1])]) for i in range(len(names))]


def import_fasta(path: Union[str, os.PathLike], device: int = 0) -> List[Tuple[str, NucleotideSequence]]:
    """bioseqdb-import without the database: every record of the file as (name, nuclseq), encoded on the
    GPU in one batch (validation as nuclseq_in, which the reference's INSERT applies)."""
    with open(path, "rb") as f:
        data = f.read()
    seq, off, names = parse_fasta_concat(data)
    raw, voff = encode_concat(seq, off, device, True)
    return list(zip(names, _split(raw, voff)))
