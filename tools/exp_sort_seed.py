"""Experiment (GPU box): how much of the seeding kernel's time is divergence between the reads of a wave?
Times lone 1M-read seeding launches (bsq_batch_seed, C2/C3 reference) with the reads in their own order and
re-ordered by keys that group similar reads into the same waves: the per-read interval count of a first run (an
upper bound: perfect knowledge of the work), the synthetic truth (random vs mapping reads), and a cheap predictor.
Prints one JSON line per ordering.  python tools/exp_sort_seed.py [reads]"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bioseqdb_amd import _native as N, synth  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    L = N.lib()
    ref = synth.make_reference(100_000_000)
    reads = synth.make_reads(ref, n, seed=synth.READ_SEED)
    idx = ctypes.c_void_p()
    N.check(L.bsq_index_create(ctypes.byref(idx)))
    keep = []
    for i, t in enumerate(ref.texts()):
        size = ctypes.c_size_t()
        p = L.bsq_nuclseq_from_text(t, len(t), ctypes.byref(size))
        buf = ctypes.create_string_buffer(ctypes.string_at(p, size.value), size.value)
        L.bsq_free(p)
        keep.append(buf)
        N.check(L.bsq_index_add_ref(idx, i + 1, ctypes.addressof(buf)))
    N.check(L.bsq_index_build_device(idx, 0))
    opts = N.Opts(19, 500, 1, 4, 5, 5, 100, 100, 6, 6, 1, 1)

    def run(perm, label, reps=5):
        codes = np.ascontiguousarray(reads.codes.reshape(n, -1)[perm].reshape(-1))
        offs = np.arange(n + 1, dtype=np.int64) * (len(codes) // n)
        b = ctypes.c_void_p()
        N.check(L.bsq_batch_create(idx, n, int(offs[-1]), ctypes.byref(b)))
        N.check(L.bsq_batch_set_reads(b, codes.ctypes.data, offs.ctypes.data, n))
        N.check(L.bsq_batch_seed(b, ctypes.byref(opts)))
        ts = []
        for _ in range(reps):
            N.check(L.bsq_batch_seed(b, ctypes.byref(opts)))
            ms = (ctypes.c_float * 6)()
            L.bsq_batch_stage_ms(b, ms, 6)
            ts.append(ms[0])
        ro = ctypes.POINTER(ctypes.c_int64)()
        iv = ctypes.POINTER(ctypes.c_uint64)()
        nt = ctypes.c_int64()
        N.check(L.bsq_batch_intervals(b, ctypes.byref(ro), ctypes.byref(iv), ctypes.byref(nt)))
        cnt = np.diff(np.ctypeslib.as_array(ro, shape=(n + 1,)).copy())
        L.bsq_batch_free(b)
        print(json.dumps({"order": label, "seed_ms": sorted(ts)[len(ts) // 2], "runs": [round(t, 3) for t in ts],
                          "intervals": int(cnt.sum())}), flush=True)
        return cnt

    base = np.arange(n)
    cnt = run(base, "as generated")
    run(np.argsort(cnt, kind="stable"), "by interval count (first run)")
    run(np.argsort(-cnt, kind="stable"), "by interval count, descending")
    run(np.argsort(reads.truth_row < 0, kind="stable"), "mapping reads first, random reads last (truth)")
    rng = np.random.default_rng(1)
    run(rng.permutation(n), "shuffled")


if __name__ == "__main__":
    main()
