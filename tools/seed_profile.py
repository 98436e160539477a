#!/usr/bin/env python3
"""Seeding work profile on the CPU (no GPU): bwt_extend calls of mem_collect_intv by phase and by
interval class, from the oracle built with -DORC_PROFILE, on the C3 shape (synthetic 100 Mbp
reference, 150 bp reads).  Usage: python tools/seed_profile.py [ref_bp] [reads]"""
import ctypes, os, subprocess, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from bioseqdb_amd import synth
from bioseqdb_amd import _native as N
import oracle_py as O

ref_bp = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
nreads = int(sys.argv[2]) if len(sys.argv) > 2 else 3000
so = "/tmp/liboracle_prof.so"
subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-DORC_PROFILE", "-o", so, os.path.join(ROOT, "oracle", "bwa_oracle.c"),
                "-lpthread", "-lm"], check=True)
O.LIB = so
P = O.lib()
L = N.lib()
ref = synth.make_reference(ref_bp)
reads = synth.make_reads(ref, nreads)
idx = ctypes.c_void_p()
N.check(L.bsq_index_create(ctypes.byref(idx)))
oi = O.OracleIndex()
keep = []
for i, t in enumerate(ref.texts()):
    size = ctypes.c_size_t()
    p = L.bsq_nuclseq_from_text(t, len(t), ctypes.byref(size))
    buf = ctypes.create_string_buffer(ctypes.string_at(p, size.value), size.value)
    keep.append(buf)
    N.check(L.bsq_index_add_ref(idx, i + 1, ctypes.addressof(buf)))
    oi.add_ref(i + 1, bytes(buf.raw))
N.check(L.bsq_index_build(idx, 0))
eb = ctypes.c_int()
oi.build_from_sa(L.bsq_index_sa_data(idx, ctypes.byref(eb)), eb.value)
opts = O.opts_from(type("o", (), dict(min_seed_len=19, max_occ=500, a=1, b=4, pen_clip3=5, pen_clip5=5, zdrop=100,
                                        w=100, o_del=6, e_del=6, o_ins=1, e_ins=1))())
codes = np.ascontiguousarray(reads.codes); offs = np.ascontiguousarray(reads.offsets)
ck = ctypes.c_uint64()
P.orc_seed_batch(oi.h, ctypes.byref(opts), codes.ctypes.data, offs.ctypes.data, reads.n, 1, ctypes.byref(ck))
c = (ctypes.c_uint64 * 16)()
P.orc_profile_get(c)
names = ["fwd<=11", "fwd u1", "fwd rank", "bwd<=11", "bwd u1", "bwd rank", "strat<=11", "strat u1", "strat rank",
         "bwd levels with a lone unique entry", "", "",
         "bwd rank, string of 12 bases", "bwd rank, 13 bases", "bwd rank, 14 bases", "bwd rank, 15 bases"]
tot = sum(c[:9])
for k, nm in enumerate(names):
    if not nm:
        continue
    print(f"{nm:38s} {c[k] / reads.n:8.1f} per read" + (f"  {100 * c[k] / tot:5.1f}%" if k < 9 else ""))
