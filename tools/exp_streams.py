"""Experiment: S concurrent sub-batches (own stream + workspace each, one host thread each) vs one batch."""
import ctypes, sys, threading, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from bioseqdb_amd import synth
from bioseqdb_amd import _native as N
import bench

L = N.lib()
ref = synth.make_reference(100_000_000)
reads = synth.make_reads(ref, 1_000_000)
idx = ctypes.c_void_p()
N.check(L.bsq_index_create(ctypes.byref(idx)))
keep = []
for i, t in enumerate(ref.texts()):
    size = ctypes.c_size_t()
    p = L.bsq_nuclseq_from_text(t, len(t), ctypes.byref(size))
    buf = ctypes.create_string_buffer(ctypes.string_at(p, size.value), size.value)
    L.bsq_free(p); keep.append(buf)
    N.check(L.bsq_index_add_ref(idx, i + 1, ctypes.addressof(buf)))
N.check(L.bsq_index_build_device(idx, 0))
opts = bench.default_opts(1)
for S in [int(x) for x in sys.argv[1:]] or [1, 2, 3]:
    subs = [reads.subset(reads.n * k // S, reads.n * (k + 1) // S) for k in range(S)]
    bs = []
    for sub in subs:
        b = ctypes.c_void_p()
        N.check(L.bsq_batch_create(idx, sub.n, int(sub.offsets[-1]), ctypes.byref(b)))
        c = np.ascontiguousarray(sub.codes); o = np.ascontiguousarray(sub.offsets)
        N.check(L.bsq_batch_set_reads(b, c.ctypes.data, o.ctypes.data, sub.n))
        bs.append(b)
    def run_all():
        th = [threading.Thread(target=lambda b=b, k=k: N.check(L.bsq_batch_run(b, ctypes.byref(opts), reads.n * k // S)))
              for k, b in enumerate(bs)]
        for t in th: t.start()
        for t in th: t.join()
    run_all()
    t0 = time.perf_counter()
    for _ in range(6): run_all()
    dt = (time.perf_counter() - t0) / 6
    print(f"S={S}: {reads.n / dt / 1e6:.2f} M reads/s ({dt * 1e3:.1f} ms/step)", flush=True)
    for b in bs: L.bsq_batch_free(b)
