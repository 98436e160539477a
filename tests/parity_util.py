"""Shared helpers for parity tests: run the same inputs through libbsq (GPU) and the oracle (CPU)."""
from __future__ import annotations

import oracle_py as O
from bioseqdb_amd import BwaIndex, NucleotideSequence, effective_opts
from bioseqdb_amd import bwa as B

FIELDS = ("ref_id", "ref_subseq", "ref_match_begin", "ref_match_end", "ref_match_len", "query_subseq",
          "query_match_begin", "query_match_end", "query_match_len", "is_primary", "is_secondary", "is_reverse",
          "cigar", "score")


def build_pair(ref_texts, ids=None, opts=None):
    ids = ids or list(range(1, len(ref_texts) + 1))
    pi = BwaIndex()
    oi = O.OracleIndex()
    for rid, t in zip(ids, ref_texts):
        ns = NucleotideSequence.from_text(t)
        on = O.Nuclseq(t)
        assert ns.raw == on.raw
        pi.add_ref_sequence(rid, ns)
        oi.add_ref(rid, on.raw)
    pi.options = effective_opts(opts, len(ref_texts))
    pi.build()
    oi.build()
    return pi, oi


def oracle_from_device_sa(pi, oi, label):
    """The oracle's FM tables for a device-built index at the BASELINE sizes, where the oracle's own suffix sort
    is too slow: from the GPU's suffix array, but only after two independent certificates -- the device one
    (bsq_index_certify_sa: range, every position once, adjacent suffixes increasing) and the oracle's host one
    inside orc_index_build_from_sa (range, one primary row, adjacent suffixes strictly increasing => a
    permutation).  Either proves the SA is the unique SA of T$, so a wrong SA cannot reach both sides of the
    parity check.  Both certificates are appended to gpurun_out/sa_certificates.jsonl (kept under profiles/)."""
    import ctypes
    import json
    import os
    from bioseqdb_amd import _native as N
    L = N.lib()
    dev = pi.certify_sa()
    assert dev["violations"] == 0 and dev["suffixes"] == L.bsq_index_seq_len(pi.handle) + 1, dev
    N.check(L.bsq_index_download(pi.handle))
    eb = ctypes.c_int()
    sa = L.bsq_index_sa_data(pi.handle, ctypes.byref(eb))
    host = oi.build_from_sa(sa, eb.value)
    assert host["violations"] == 0 and host["suffixes"] == dev["suffixes"], host
    assert oi.primary == L.bsq_index_primary(pi.handle)
    rec = {"config": label, "sa_elem_bytes": eb.value, "device": dev, "host": host}
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "sa_certificates.jsonl"), "a") as f:
        f.write(json.dumps(rec) + "\n")
    print(f"[sa certificate] {label}: {json.dumps(rec)}", flush=True)
    return rec


def compare(pi, oi, read_texts, first_call=0, opts=None):
    """Returns (n_rows_checked, mismatches[list of (read, field, gpu, oracle)])."""
    o = pi.options if opts is None else opts
    oo = O.opts_from(o)
    seqs = [NucleotideSequence.from_text(t) for t in read_texts]
    got = pi.align_sequences(seqs, o, first_call=first_call)
    bad = []
    rows = 0
    for i, t in enumerate(read_texts):
        exp = B.parse_tsv(oi.align_tsv(oo, seqs[i].raw, O.lrand48_at(first_call + i)))
        g = got[i]
        if len(g) != len(exp):
            bad.append((i, "n_rows", len(g), len(exp)))
            continue
        for a, e in zip(g, exp):
            rows += 1
            for f in FIELDS:
                if f == "ref_subseq" and e.is_reverse:
                    continue   # Q7: the reference reads out of bounds on reverse rows
                if getattr(a, f) != getattr(e, f):
                    bad.append((i, f, getattr(a, f), getattr(e, f)))
    return rows, bad


def _oracle_batch_tsv(oi, oo, raws, first_call, threads=0):
    """orc_align_tsv_batch: the oracle's rows of every read, read order, on all host cores."""
    import ctypes
    import os
    n = len(raws)
    bufs = [ctypes.create_string_buffer(r, len(r)) for r in raws]
    ptrs = (ctypes.c_void_p * max(n, 1))(*[ctypes.addressof(b) for b in bufs])
    cnt = (ctypes.c_int64 * max(n, 1))()
    L = O.lib()
    f = L.orc_align_tsv_batch
    f.restype = ctypes.c_void_p
    f.argtypes = [ctypes.c_void_p, ctypes.POINTER(O.OrcOpts), ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64,
                  ctypes.c_int, ctypes.c_void_p]
    p = f(oi.h, ctypes.byref(oo), ptrs, n, first_call, threads or min(16, os.cpu_count() or 1), cnt)
    assert p, "oracle: unsupported read"
    try:
        text = ctypes.string_at(p).decode("latin-1")
    finally:
        L.orc_free(p)
    return text, list(cnt)[:n]


def gpu_batch_tsv(pi, seqs, opts, first_call):
    """bsq_align_batch + bsq_render_tsv over the whole batch: (text, rows per read)."""
    import ctypes
    from bioseqdb_amd import _native as N
    L = N.lib()
    n = len(seqs)
    pi.upload()
    arr = (ctypes.c_void_p * max(n, 1))(*[s.ptr for s in seqs])
    out = ctypes.POINTER(N.Hits)()
    N.check(L.bsq_align_batch(pi.handle, ctypes.byref(opts), arr, n, first_call, ctypes.byref(out)))
    try:
        p = L.bsq_render_tsv(pi.handle, out, arr)
        try:
            text = ctypes.string_at(p).decode("latin-1")
        finally:
            L.bsq_free(p)
        ro = out.contents.read_off
        counts = [ro[i + 1] - ro[i] for i in range(n)]
    finally:
        L.bsq_hits_free(out)
    return text, counts


def compare_tsv(got_text, got_counts, exp_text, exp_counts, limit=50):
    """Row-by-row comparison of two bwa_result TSVs in read order; the oracle prints '*' as ref_subseq on
    reverse-strand rows (Q7), where that column is skipped.  Returns (rows, mismatches)."""
    bad = []
    g_lines = got_text.splitlines()
    e_lines = exp_text.splitlines()
    gi = ei = 0
    rows = 0
    for r, (gc, ec) in enumerate(zip(got_counts, exp_counts)):
        if gc != ec:
            bad.append((r, "n_rows", gc, ec))
        else:
            for k in range(gc):
                a, e = g_lines[gi + k], e_lines[ei + k]
                rows += 1
                if a != e:
                    fa, fe = a.split("\t"), e.split("\t")
                    for j, (x, y) in enumerate(zip(fa, fe)):
                        if x != y and not (j == 1 and y == "*"):
                            bad.append((r, FIELDS[j], x[:60], y[:60]))
        gi += gc
        ei += ec
        if len(bad) >= limit:
            break
    if len(got_counts) != len(exp_counts):
        bad.append((-1, "n_reads", len(got_counts), len(exp_counts)))
    return rows, bad


def compare_batch(pi, oi, seqs, first_call=0, opts=None):
    """The whole batch through the GPU (bsq_align_batch + bsq_render_tsv) against the oracle's batch TSV.
    `seqs` are NucleotideSequence values; returns (rows, mismatches)."""
    o = pi.options if opts is None else opts
    got, gc = gpu_batch_tsv(pi, seqs, o, first_call)
    exp, ec = _oracle_batch_tsv(oi, O.opts_from(o), [s.raw for s in seqs], first_call)
    return compare_tsv(got, gc, exp, ec)
