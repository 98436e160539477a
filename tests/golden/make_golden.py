"""Regenerates the committed golden fixtures (inputs + oracle outputs).  Run from the repo root:
    python tests/golden/make_golden.py
The fixtures pin the oracle against regressions (tests/test_golden.py::test_oracle_reproduces_golden) and
give the GPU path a fixed input/output set (tests/test_golden.py::test_gpu_matches_golden, marked gpu).  The
expected outputs are the oracle's own, so they pin the oracle against itself and the GPU against the oracle,
not either against libbwa (absent here).  Inputs are stored as text so they do not depend
on the generator's numpy version."""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

import oracle_py as O  # noqa: E402

OPTS = dict(min_seed_len=19, max_occ=500, a=1, b=4, pen_clip3=5, pen_clip5=5, zdrop=100, w=100, o_del=6, e_del=6,
            o_ins=1, e_ins=1)


def main():
    rng = random.Random(20250218)
    rows = []
    for L, nh in ((40_003, 3), (25_001, 2), (29, 1)):
        s = [rng.choice("ACGT") for _ in range(L)]
        for _ in range(nh):
            p = rng.randrange(L - 13)
            ch = rng.choice("NRYKMSWBDHV")
            for j in range(p, p + rng.randint(1, 12)):
                s[j] = ch
        rows.append("".join(s))
    # a duplicated segment (secondary hits) and an inverted copy
    seg = rows[0][5000:6200]
    rows[1] = rows[1][:3000] + seg + rows[1][3000 + len(seg):]
    comp = str.maketrans("ACGTNRYKMSWBDHV", "TGCANYRMKSWVHDB")
    rows[1] = rows[1][:9000] + seg.translate(comp)[::-1] + rows[1][9000 + len(seg):]
    cat = "".join(rows)
    reads = []
    for i in range(400):
        L = rng.choice([150] * 6 + [100, 75, 40, 20])
        p = rng.randrange(len(cat) - L)
        r = list(cat[p:p + L])
        for j in range(L):
            if rng.random() < 0.015:
                r[j] = rng.choice("ACGT")
        if rng.random() < 0.08:
            q = rng.randrange(10, max(L - 10, 11))
            if rng.random() < 0.5:
                del r[q:q + rng.randint(1, 3)]
            else:
                r[q:q] = [rng.choice("ACGT") for _ in range(rng.randint(1, 3))]
        r = "".join(c if c in "ACGTN" else "N" for c in r)
        if rng.random() < 0.5:
            r = r.translate(comp)[::-1]
        if rng.random() < 0.03:
            r = "".join(rng.choice("ACGT") for _ in range(L))
        reads.append(r)
    oi = O.OracleIndex()
    for k, t in enumerate(rows):
        oi.add_ref(100 + k, O.Nuclseq(t).raw)
    oi.build()
    oo = O.OrcOpts(*OPTS.values())
    first_call = 17
    out = []
    for i, r in enumerate(reads):
        for line in oi.align_tsv(oo, O.Nuclseq(r).raw, O.lrand48_at(first_call + i)).splitlines():
            out.append(f"{i}\t{line}")
    with open(os.path.join(HERE, "g1_input.json"), "w") as f:
        json.dump({"ref_ids": [100, 101, 102], "refs": rows, "reads": reads, "first_call": first_call,
                   "opts": OPTS}, f)
    with open(os.path.join(HERE, "g1_expected.tsv"), "w") as f:
        f.write("\n".join(out) + "\n")
    print(len(reads), "reads,", len(out), "rows")


if __name__ == "__main__":
    main()
