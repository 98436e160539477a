#!/usr/bin/env python3
"""Extension work profile on the CPU (no GPU): ksw_extend2 rows and cells over the C3 shape (synthetic 100 Mbp
reference, 150 bp reads, the effective SQL options), and the rows / cells that follow the one-column tail condition
(the band is the query's last column alone, its left neighbour's H is 0 and the row reached the query's end: every
later row only decays that column's E, so no output of the call can change).  The oracle built with -DORC_PROFILE.
Usage: python tools/ext_profile.py [ref_bp] [reads]"""
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
# the effective SQL defaults (bench.default_opts: the bwa_opts() field-order quirk Q1 gives e_del = 6, o_ins = 1)
opts = O.OrcOpts(19, 500, 1, 4, 5, 5, 100, 100, 6, 6, 1, 1)
codes = np.ascontiguousarray(reads.codes); offs = np.ascontiguousarray(reads.offsets)
ck = ctypes.c_uint64()
P.orc_align_batch(oi.h, ctypes.byref(opts), codes.ctypes.data, offs.ctypes.data, reads.n, 0, 1, ctypes.byref(ck))
c = (ctypes.c_uint64 * 20)()
P.orc_profile_get(c)
n = reads.n
print(f"{n} reads: ksw_extend2 rows {c[16] / n:.1f} per read, cells {c[17] / n:.1f} ({c[17] / max(c[16], 1):.1f} per row)")
print(f"  after the one-column tail condition: rows {c[18] / n:.1f} per read ({100 * c[18] / max(c[16], 1):.1f} %), "
      f"cells {c[19] / n:.1f} ({100 * c[19] / max(c[17], 1):.1f} %)")
