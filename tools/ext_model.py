"""A lockstep model of k_extend's schedules, from the oracle's per-read extension trace (orc_ext_trace, an
ORC_PROFILE build): every mem_chain2aln call, every seed it visits (skipped or not), every extension side and
every ksw_extend2 call with the cells of each of its rows (bwa_oracle.c tr_push kinds 20/21/22/10/11).

A wave of 64 lanes runs nested loops in lockstep: a loop runs as many iterations as its busiest active lane, and
an iteration costs its body once whatever the number of active lanes.  Costs are VALU wave-instructions (`C_*`
below; the cell loop is 57 per two cells, tools/dp_cell_isa.py), so `util` is the model's lane utilisation
(useful lane-instructions / 64 x wave-instructions; the GPU measures 39 % for k_extend, SQ counters).
  current  k_extend today: each wave takes the next 64 reads of the work-sorted order, one read per lane;
           chains, seeds, sides, band retries, rows and cells all in lockstep
  merged   the current schedule with one loop over a seed's ksw_extend2 calls (left band tries, then right ones)
           instead of a loop per side: a lane extending only left and one extending only right run together
  calls    a task loop at call granularity: each trip every lane runs its next ksw_extend2 call (rows and cells
           in lockstep with the other lanes' calls); a lane whose read is done takes the next read of the order;
           the per-read finish (dedup / patch / primary marking) moved to a kernel of its own (one read per lane)
  rows     the same at row granularity: each trip every lane runs one row of its current call; a lane whose call
           ended sets up its next call (and, when needed, its next seed / chain / read) in that trip
python tools/ext_model.py [reads] [ref_bp]   (CPU; builds the C3-shaped index on the host)"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import oracle_py as O  # noqa: E402
from bioseqdb_amd import BwaIndex, NucleotideSequence, synth  # noqa: E402
from bioseqdb_amd._native import lib  # noqa: E402

C_PAIR = 57      # two cells of the unrolled cell loop
C_ROW = 90       # band update, z-drop test, the row's E/H bookkeeping and the beg/end scans
C_CALL = 300     # ksw_extend2 set-up: band clamp, first row, profile / target accessors, result
C_SEED = 120     # the skip test against the read's regions and the region record
C_CHAIN = 400    # chain window and seed order
C_READ = 900     # read start: descriptors, query staged in LDS
C_FINISH = 1500  # dedup / patch / primary marking per read


def traces(n_reads, ref_bp):
    so = "/tmp/liboracle_prof.so"
    import subprocess
    subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-DORC_PROFILE", "-o", so,
                    os.path.join(ROOT, "oracle", "bwa_oracle.c"), "-lpthread", "-lm"], check=True)
    O.LIB = so
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
    oo = O.OrcOpts(19, 500, 1, 4, 5, 5, 100, 100, 6, 6, 1, 1)   # the effective SQL options (Q1: e_del 6, o_ins 1)
    f = O.lib().orc_ext_trace
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.POINTER(O.OrcOpts), ctypes.c_void_p, ctypes.c_int, ctypes.c_int64,
                  ctypes.POINTER(ctypes.c_int32), ctypes.c_int]
    cap = 1 << 20
    buf = (ctypes.c_int32 * cap)()
    out = []
    for r in range(n_reads):
        q = bytes(reads.codes[reads.offsets[r]:reads.offsets[r + 1]])
        qb = ctypes.create_string_buffer(q, len(q))
        m = f(oi.h, ctypes.byref(oo), ctypes.addressof(qb), len(q), r, buf, cap)
        chains = []
        for k in range(0, m, 4):
            kind, a, b, d = buf[k], buf[k + 1], buf[k + 2], buf[k + 3]
            if kind == 20:
                chains.append({"n": a, "best": b, "seeds": []})
            elif kind == 21:
                chains[-1]["seeds"].append({"skip": a, "qbeg": b, "slen": d, "sides": [[], []], "cur": None})
            elif kind == 22:   # side a: 0 left, 1 right
                chains[-1]["seeds"][-1]["cur"] = a
            elif kind == 10:
                sd = chains[-1]["seeds"][-1]
                sd["sides"][sd["cur"]].append([])
            elif kind == 11:
                sd = chains[-1]["seeds"][-1]
                sd["sides"][sd["cur"]][-1].append(a)
        est = sum(max(len(q) - c["best"], 0) + 4 for c in chains)
        out.append({"len": len(q), "chains": chains, "key": (min(len(chains), 63) << 18) | min(est, 262143)})
    return out


def pairs(c):
    return (c + 1) // 2


def lockstep_calls(calls):
    """64 (or fewer) ksw_extend2 calls side by side: rows in lockstep, each row's cell loop as long as its widest
    active lane.  Returns (wave cost, useful lane cost)."""
    calls = [c for c in calls if c is not None]
    if not calls:
        return 0, 0
    w = C_CALL
    u = C_CALL * len(calls)
    nrow = max(len(c) for c in calls)
    for i in range(nrow):
        act = [c[i] for c in calls if i < len(c)]
        w += C_ROW + C_PAIR * max(pairs(x) for x in act)
        u += C_ROW * len(act) + C_PAIR * sum(pairs(x) for x in act)
    return w, u


def flat_calls(rd):
    """a read's ksw_extend2 calls in order, each with the control it needs first ('chain' / 'seed')"""
    out = []
    for c in rd["chains"]:
        first = True
        for s in c["seeds"]:
            for side in s["sides"]:
                for call in side:
                    out.append((first, call))
                    first = False
    return out


def model_current(reads, merged=False):
    W = U = 0
    order = sorted(range(len(reads)), key=lambda i: -reads[i]["key"])
    for b in range(0, len(order), 64):
        grp = [reads[i] for i in order[b:b + 64]]
        W += C_READ + C_FINISH
        U += (C_READ + C_FINISH) * len(grp)
        nch = max(len(r["chains"]) for r in grp)
        for ci in range(nch):
            ch = [r["chains"][ci] for r in grp if ci < len(r["chains"])]
            W += C_CHAIN
            U += C_CHAIN * len(ch)
            nsd = max(len(c["seeds"]) for c in ch)
            for si in range(nsd):
                sd = [c["seeds"][si] for c in ch if si < len(c["seeds"])]
                W += C_SEED
                U += C_SEED * len(sd)
                if merged:   # one loop over the seed's calls, left tries then right tries
                    seq = [[c for side in s["sides"] for c in side] for s in sd]
                    for t in range(max((len(x) for x in seq), default=0)):
                        w, u = lockstep_calls([x[t] if t < len(x) else None for x in seq])
                        W += w
                        U += u
                    continue
                for side in (0, 1):   # left, then right (a side list holds 0, 1 or 2 band tries)
                    sides = [s["sides"][side] for s in sd]
                    ntry = max((len(x) for x in sides), default=0)
                    for t in range(ntry):
                        w, u = lockstep_calls([x[t] if t < len(x) else None for x in sides])
                        W += w
                        U += u
    return W, U


def model_readflat(reads):
    """64 reads per wave as today, but one loop over each read's ksw_extend2 calls (all chains, seeds, sides and
    band tries flattened): trip t runs the t-th call of every lane, with the control before it"""
    W = U = 0
    order = sorted(range(len(reads)), key=lambda i: -reads[i]["key"])
    for b in range(0, len(order), 64):
        grp = [flat_calls(reads[i]) for i in order[b:b + 64]]
        W += C_READ + C_FINISH
        U += (C_READ + C_FINISH) * len(grp)
        for t in range(max((len(x) for x in grp), default=0)):
            cur = [x[t][1] if t < len(x) else None for x in grp]
            first = any(t < len(x) and x[t][0] for x in grp)
            W += C_SEED + (C_CHAIN if first else 0)
            U += C_SEED * sum(c is not None for c in cur)
            w, u = lockstep_calls(cur)
            W += w
            U += u
    U += sum(C_CHAIN * len(r["chains"]) for r in reads)
    return W, U


def model_merged(reads):
    return model_current(reads, merged=True)


def model_calls(reads):
    W = U = 0
    order = sorted(range(len(reads)), key=lambda i: -reads[i]["key"])
    queue = [flat_calls(reads[i]) for i in order]
    # finish kernel: one read per lane, 64 reads per wave
    W += C_FINISH * ((len(order) + 63) // 64)
    U += C_FINISH * len(order)
    # one wave per 64 lanes drawing reads from the order (waves interleave, so model one wave per 64-read chunk pool)
    for b in range(0, len(queue), 64 * 8):
        pool = list(reversed(queue[b:b + 64 * 8]))
        lanes = [[] for _ in range(64)]
        while True:
            for lane in lanes:
                if not lane and pool:
                    lane.extend(pool.pop())
                    lane.insert(0, "read")
            if not any(lanes):
                break
            cur, ctl_read, ctl_chain = [], False, False
            for lane in lanes:
                if lane and lane[0] == "read":
                    lane.pop(0)
                    ctl_read = True
                if lane:
                    first, call = lane.pop(0)
                    ctl_chain = ctl_chain or first
                    cur.append(call)
            n = len(cur)
            W += C_SEED + (C_READ if ctl_read else 0) + (C_CHAIN if ctl_chain else 0)
            U += C_SEED * n
            w, u = lockstep_calls(cur)
            W += w
            U += u
    U += sum(C_READ for _ in order) + sum(C_CHAIN * len(r["chains"]) for r in reads)
    return W, U


def model_rows(reads):
    W = U = 0
    order = sorted(range(len(reads)), key=lambda i: -reads[i]["key"])
    queue = [flat_calls(reads[i]) for i in order]
    W += C_FINISH * ((len(order) + 63) // 64)
    U += C_FINISH * len(order)
    for b in range(0, len(queue), 64 * 8):
        pool = list(reversed(queue[b:b + 64 * 8]))
        calls = [[] for _ in range(64)]   # a lane's remaining calls of its read
        rows = [None] * 64                # a lane's remaining rows of its current call
        while True:
            ctl_call = ctl_read = ctl_chain = False
            act = []
            for i in range(64):
                if rows[i] is None or not rows[i]:
                    if not calls[i] and pool:
                        calls[i] = list(pool.pop())
                        ctl_read = True
                    if calls[i]:
                        first, call = calls[i].pop(0)
                        ctl_chain = ctl_chain or first
                        ctl_call = True
                        rows[i] = list(call)
                        U += C_CALL + C_SEED
                    else:
                        rows[i] = None
                if rows[i]:
                    act.append(rows[i].pop(0))
            if not act and not ctl_call:
                if all(r is None for r in rows) and not pool:
                    break
            W += (C_CALL + C_SEED if ctl_call else 0) + (C_READ if ctl_read else 0) + (C_CHAIN if ctl_chain else 0)
            if act:
                W += C_ROW + C_PAIR * max(pairs(x) for x in act)
                U += C_ROW * len(act) + C_PAIR * sum(pairs(x) for x in act)
    U += sum(C_READ for _ in order) + sum(C_CHAIN * len(r["chains"]) for r in reads)
    return W, U


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    ref_bp = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000_000
    reads = traces(n, ref_bp)
    key_study(reads)
    ncalls = sum(len(flat_calls(r)) for r in reads)
    nrows = sum(len(c) for r in reads for _, c in flat_calls(r))
    ncells = sum(sum(c) for r in reads for _, c in flat_calls(r))
    nch = sum(len(r["chains"]) for r in reads)
    print(f"{n} reads: {nch / n:.2f} chains, {ncalls / n:.2f} ksw_extend2 calls, {nrows / n:.1f} rows, "
          f"{ncells / n:.0f} cells per read")
    for keyname in ("previous key", "round-5 key"):
        if keyname == "round-5 key":   # k_ext_key today: chains, sides of the first extended seed, its left extent / 8, est
            for r in reads:
                qb, sl = next(((sd["qbeg"], sd["slen"]) for c in r["chains"] for sd in c["seeds"] if not sd["skip"]),
                              (0, r["len"]))
                sides = (qb > 0) + (qb + sl != r["len"])
                r["key"] = (min(len(r["chains"]), 63) << 24) | (sides << 22) | (min(qb >> 3, 63) << 16) | \
                    min(r["key"] & 262143, 65535)
        print(f" schedules over the {keyname}'s order:")
        run_schedules(reads, n)


def run_schedules(reads, n):
    base = None
    for name, fn in (("current", model_current), ("merged", model_merged), ("readflat", model_readflat), ("calls", model_calls), ("rows", model_rows)):
        W, U = fn(reads)
        base = base or W
        print(f"  {name:8s} wave-instructions per 64 reads {W * 64 / n:9.0f}  "
              f"util {U / (64 * W):.3f}  time x{W / base:.3f}")



def key_study(reads):
    """the current schedule under other sort keys: what a better work estimate would be worth"""
    import numpy as np
    rows = np.array([sum(len(c) for _, c in flat_calls(r)) for r in reads])
    est = np.array([r["key"] & 262143 for r in reads])
    print(f"  rows per read: mean {rows.mean():.1f} sd {rows.std():.1f}; corr(rows, est) {np.corrcoef(rows, est)[0, 1]:.3f}")
    W0, _ = model_current(reads)
    def sides(r):   # extension sides of the first seed that is extended
        for c in r["chains"]:
            for sd in c["seeds"]:
                if not sd["skip"]:
                    return [sum(len(x) for x in side) for side in sd["sides"]]
        return []

    est_of = lambda r: r["key"] & 262143

    def top(r):   # the first extended seed: (qbeg, len)
        for c in r["chains"]:
            for sd in c["seeds"]:
                if not sd["skip"]:
                    return sd["qbeg"], sd["slen"]
        return 0, r["len"]

    def nsides(r):
        qb, sl = top(r)
        return (qb > 0) + (qb + sl != r["len"])

    def kind(r):
        qb, sl = top(r)
        return (qb > 0) | (qb + sl != r["len"]) << 1

    def lb(r, sh=3):
        return min(top(r)[0] >> sh, 63)

    def rb(r, sh=3):
        qb, sl = top(r)
        return min((r["len"] - qb - sl) >> sh, 63)

    for name, kf in (("rows", lambda r: sum(len(c) for _, c in flat_calls(r))),
                     ("cells", lambda r: sum(sum(c) for _, c in flat_calls(r))),
                     ("sides,est", lambda r: (nsides(r) << 16) | min(est_of(r), 65535)),
                     ("sides,lb,est", lambda r: (nsides(r) << 22) | (lb(r) << 16) | min(est_of(r), 65535)),
                     ("sides,lb,rb", lambda r: (nsides(r) << 22) | (lb(r) << 16) | rb(r)),
                     ("sides,lb4,est", lambda r: (nsides(r) << 22) | (lb(r, 2) << 16) | min(est_of(r), 65535)),
                     ("sides,lb,rb4", lambda r: (nsides(r) << 22) | (lb(r) << 16) | rb(r, 2)),
                     ("sides,max,est", lambda r: (nsides(r) << 22) | (max(lb(r), rb(r)) << 16) | min(est_of(r), 65535)),
                     ("kind,max,est", lambda r: (kind(r) << 22) | (max(lb(r), rb(r)) << 16) | min(est_of(r), 65535)),
                     ("sides,max4,est", lambda r: (nsides(r) << 22) | (max(lb(r, 2), rb(r, 2)) << 16) | min(est_of(r), 65535)),
                     ("sides,max,min", lambda r: (nsides(r) << 22) | (max(lb(r), rb(r)) << 16) | min(lb(r), rb(r))),
                     ("max,est", lambda r: (max(lb(r), rb(r)) << 16) | min(est_of(r), 65535)),
                     ("kind,max4,est", lambda r: (kind(r) << 22) | (max(lb(r, 2), rb(r, 2)) << 16) | min(est_of(r), 65535)),
                     ("kind,lb,rb", lambda r: (kind(r) << 22) | (lb(r) << 16) | rb(r)),
                     ("kind,lb,est", lambda r: (kind(r) << 22) | (lb(r) << 16) | min(est_of(r), 65535)),
                     ("kind,max,min", lambda r: (kind(r) << 22) | (max(lb(r), rb(r)) << 16) | min(lb(r), rb(r)))):
        saved = [r["key"] for r in reads]
        for r in reads:
            r["key"] = (min(len(r["chains"]), 63) << 26) | min(kf(r), (1 << 26) - 1)
        W, U = model_current(reads)
        for r, k in zip(reads, saved):
            r["key"] = k
        print(f"  current, sorted by {name:11s}: util {U / (64 * W):.3f}  time x{W / W0:.3f}")


if __name__ == "__main__":
    main()
