"""A trip model of the seeding kernels' schedules, from the oracle's per-call seeding trace (orc_seed_trace).

Each bwt_smem1 call is (forward trips, backward trips), each bwt_seed_strategy1 call its trips, counted the way
smem.hip's kernels take them (bwa_oracle.c tr_push).  A wave of 64 lanes advances one trip at a time; a schedule
decides which lanes wait for which.  Printed per schedule: wave trips per 64 reads (lower = fewer dependent memory
round trips per read at equal occupancy), and the fraction of lane-trips doing work.
  lds     k_smem_lds: pass-1 calls aligned by ordinal (forward max + backward max per call), pass-2 calls by mem index,
          seed-strategy calls by ordinal; one read per lane
  merged  the same with one loop for forward and backward (max of the sum per call)
  lanes   k_smem_lanes: persistent lanes, one call per lane per outer step (smem calls: forward max + backward max;
          seed-strategy calls beside them), a lane takes its next read when done (R reads per lane)
  lanesm  lanes with the merged loop
  ideal   no lane ever waits (each lane's own trips; the wave ends with its busiest lane)
python tools/seed_model.py [waves] [reads_per_lane]   (CPU; builds the C3 100 Mbp index on the host)"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_py as O  # noqa: E402
from bioseqdb_amd import BwaIndex, NucleotideSequence, synth  # noqa: E402
from bioseqdb_amd._native import lib  # noqa: E402


BWD_POS = [0, 0, 0]


def traces(n_reads, ref_bp=100_000_000, walk=True):
    ref = synth.make_reference(ref_bp)
    pi, oi = BwaIndex(), O.OracleIndex()
    for i, t in enumerate(ref.texts()):
        ns = NucleotideSequence.from_text(t.decode())
        pi.add_ref_sequence(i + 1, ns)
        oi.add_ref(i + 1, ns.raw)
    pi.build(threads=0)
    eb = ctypes.c_int()
    oi.build_from_sa(lib().bsq_index_sa_data(pi.handle, ctypes.byref(eb)), eb.value)
    reads = synth.make_reads(ref, n_reads, seed=synth.READ_SEED)
    oo = O.OrcOpts(19, 500, 1, 4, 5, 5, 100, 100, 6, 6, 1, 1)
    f = O.lib().orc_seed_trace
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.POINTER(O.OrcOpts), ctypes.c_void_p, ctypes.c_int,
                  ctypes.POINTER(ctypes.c_int32), ctypes.c_int]
    buf = (ctypes.c_int32 * 65536)()
    out = []
    for r in range(n_reads):
        q = bytes(reads.codes[reads.offsets[r]:reads.offsets[r + 1]])
        qb = ctypes.create_string_buffer(q, len(q))
        m = f(oi.h, ctypes.byref(oo), ctypes.addressof(qb), len(q), buf, 65536)
        calls = []
        for k in range(0, m, 4):
            kind, a, b, idx = buf[k], buf[k + 1], buf[k + 2], buf[k + 3]
            if kind == 4:   # backward positions of the preceding smem call: all, with <= 2 entries, one unique entry
                for j, v in enumerate((a, b, idx)):
                    BWD_POS[j] += v
                continue
            if kind == 3:   # seed strategy: trips before uniqueness, then the walk (2 trips) or one per step
                calls.append((3, a + (min(b, 2) if walk else b), 0, idx))
            else:
                calls.append((kind, a, b, idx))
        out.append(calls)
    return out


def wave_lds(reads, merged):
    t = 0
    for kind in (1, 2, 3):
        by = {}
        for calls in reads:
            for c in calls:
                if c[0] == kind:
                    by.setdefault(c[3], []).append(c)
        for _, cs in sorted(by.items()):
            if kind == 3:
                t += max(c[1] for c in cs)
            elif merged:
                t += max(c[1] + c[2] for c in cs)
            else:
                t += max(c[1] for c in cs) + max(c[2] for c in cs)
    return t


def wave_lanes(lanes_reads, merged):
    queues = [[c for calls in rs for c in calls] for rs in lanes_reads]
    pos = [0] * len(queues)
    t = 0
    while any(p < len(q) for p, q in zip(pos, queues)):
        sm, ss = [], []
        for i, q in enumerate(queues):
            if pos[i] < len(q):
                c = q[pos[i]]
                (ss if c[0] == 3 else sm).append(c)
                pos[i] += 1
        if sm:
            t += max(c[1] + c[2] for c in sm) if merged else max(c[1] for c in sm) + max(c[2] for c in sm)
        if ss:
            t += max(c[1] for c in ss)
    return t


def main():
    waves = int(sys.argv[1]) if len(sys.argv) > 1 else 48
    rpl = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    n = waves * 64 * rpl
    tr = traces(n)
    work = sum(sum(c[1] + c[2] for c in calls) for calls in tr)
    res = {}
    for name in ("lds", "merged"):
        tot = 0
        for w in range(waves * rpl):
            tot += wave_lds(tr[w * 64:(w + 1) * 64], name == "merged")
        res[name] = tot
    # tools/exp_sort_seed.py's measured orderings (C2 lds: 10.57 ms as generated, 9.31 ms sorted descending by
    # interval count): the same schedule over reads sorted by their number of calls and by their trips
    for name, key in (("lds_bycalls", lambda c: -len(c)), ("lds_bytrips", lambda c: -sum(x[1] + x[2] for x in c))):
        st = sorted(tr, key=key)
        res[name] = sum(wave_lds(st[w * 64:(w + 1) * 64], False) for w in range(waves * rpl))
    for name in ("lanes", "lanesm"):
        tot = 0
        for w in range(waves):
            lanes = [[tr[(w * 64 + l) + 64 * waves * k] for k in range(rpl)] for l in range(64)]
            tot += wave_lanes(lanes, name == "lanesm")
        res[name] = tot
    ideal = 0
    for w in range(waves):
        ideal += max(sum(sum(c[1] + c[2] for c in tr[(w * 64 + l) + 64 * waves * k]) for k in range(rpl)) for l in range(64))
    res["ideal"] = ideal
    print(f"{n} reads, {waves} waves x {rpl} reads per lane; lane work {work / n:.1f} trips per read")
    print(f"  backward positions per read {BWD_POS[0] / n:.1f}: {BWD_POS[1] / max(BWD_POS[0], 1):.3f} with <= 2 list "
          f"entries, {BWD_POS[2] / max(BWD_POS[0], 1):.3f} with one unique entry")
    for k, v in res.items():
        print(f"  {k:7s} wave trips per 64 reads {v * 64 / n:8.1f}   useful lane-trips {work / (v * 64):.3f}")


if __name__ == "__main__":
    main()
