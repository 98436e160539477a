"""Index replication: an index imported from another index's device tables and
metadata aligns byte-identically to the original (the broadcast itself is torch.distributed's)."""
import ctypes

import numpy as np
import pytest

from bioseqdb_amd import NucleotideSequence, synth
from bioseqdb_amd import _native as N
from parity_util import build_pair

pytestmark = pytest.mark.gpu


def _align(L, h, opts, seqs, first_call):
    arr = (ctypes.c_void_p * len(seqs))(*[s.ptr for s in seqs])
    out = ctypes.POINTER(N.Hits)()
    N.check(L.bsq_align_batch(h, ctypes.byref(opts), arr, len(seqs), first_call, ctypes.byref(out)))
    H = out.contents
    hits = ctypes.string_at(H.hits, H.n_hits * ctypes.sizeof(N.Hit)) if H.n_hits else b""
    cig = ctypes.string_at(H.cigar, H.n_cigar * 4) if H.n_cigar else b""
    off = ctypes.string_at(H.read_off, (len(seqs) + 1) * 8)
    L.bsq_hits_free(out)
    return hits, cig, off


@pytest.mark.parametrize("wide", [False, True])
def test_import_matches_original(monkeypatch, wide):
    import torch
    if wide:
        monkeypatch.setenv("BSQ_FORCE_WIDE", "1")
    L = N.lib()
    ref = synth.make_reference(600_000, n_rows=2, n_run_every=200_000, n_run_len=300)
    reads = synth.make_reads(ref, 1200, seed=51)
    pi, _ = build_pair([t.decode() for t in ref.texts()])
    sizes = (ctypes.c_uint64 * N.N_TABLES)()
    mb = ctypes.c_uint64()
    N.check(L.bsq_index_layout(pi.handle, sizes, None, ctypes.byref(mb)))
    meta = ctypes.create_string_buffer(mb.value)
    N.check(L.bsq_index_layout(pi.handle, sizes, meta, ctypes.byref(mb)))
    dev = torch.device("cuda", 0)
    src = [torch.empty(int(b), dtype=torch.uint8, device=dev) if b else None for b in sizes]
    T = lambda bufs: (N.Table * N.N_TABLES)(*[N.Table(t.data_ptr() if t is not None else None, int(b))
                                             for t, b in zip(bufs, sizes)])
    N.check(L.bsq_index_upload_into(pi.handle, 0, T(src), N.N_TABLES))
    dst = [t.clone() if t is not None else None for t in src]   # stands in for the broadcast
    torch.cuda.synchronize()
    imp = ctypes.c_void_p()
    N.check(L.bsq_index_import(meta, mb.value, 0, T(dst), N.N_TABLES, ctypes.byref(imp)))
    try:
        assert L.bsq_index_n_refs(imp) == 2 and L.bsq_index_l_pac(imp) == L.bsq_index_l_pac(pi.handle)
        seqs = [NucleotideSequence.from_text(reads.text(i)) for i in range(reads.n)]
        a = _align(L, pi.handle, pi.options, seqs, 17)
        b = _align(L, imp, pi.options, seqs, 17)
        assert len(a[0]) > 1000 * ctypes.sizeof(N.Hit)
        if a != b:   # say which records differ
            import numpy as np
            ha = np.frombuffer(a[0], np.uint8).reshape(-1, ctypes.sizeof(N.Hit))
            hb = np.frombuffer(b[0], np.uint8).reshape(-1, ctypes.sizeof(N.Hit))
            diff = np.where((ha != hb).any(1))[0] if ha.shape == hb.shape else None
            ex = ""
            if diff is not None and len(diff):
                k = int(diff[0])
                ra = N.Hit.from_buffer_copy(a[0][k * ctypes.sizeof(N.Hit):(k + 1) * ctypes.sizeof(N.Hit)])
                rb = N.Hit.from_buffer_copy(b[0][k * ctypes.sizeof(N.Hit):(k + 1) * ctypes.sizeof(N.Hit)])
                ex = {f: (getattr(ra, f), getattr(rb, f)) for f, _ in N.Hit._fields_ if getattr(ra, f) != getattr(rb, f)}
            raise AssertionError(f"{ex} hits {ha.shape} vs {hb.shape}, differing {None if diff is None else (len(diff), diff[:8].tolist())}, "
                                 f"cigar equal {a[1] == b[1]}, offsets equal {a[2] == b[2]}")
    finally:
        L.bsq_index_free(imp)
        del src, dst
