"""Kernel + copy timeline of the pipelined cursor (tools/cursor_probe.sh output).

    python3 tools/cursor_timeline.py gpurun_out/<tag>/cur

Splits the trace into the with-columns cursor (first k_col_lens launch to the last) and the records-only cursor
after it, and prints per phase: wall span, union of kernel busy time, kernel time by kernel family, and the copies
(count, bytes, summed duration) by direction.
"""
import csv
import glob
import sys
from collections import defaultdict


def load(d, kind):
    f = glob.glob(f"{d}/**/*{kind}.csv", recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def family(name):
    for k in ("k_col_lens", "k_sub_write", "k_enc_", "k_dec_", "k_smem_lds", "k_codes_wave", "k_chain", "k_extend",
              "k_ext_key", "k_r2a_key", "k_reg2aln_diag", "k_reg2aln_g", "k_reg2aln_w", "k_counts", "k_pack",
              "rocprim", "hipcub"):
        if k in name:
            return k
    return name.split("(")[0][-40:]


def main(d):
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in load(d, "kernel_trace")]
    cs = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", "?"), int(r.get("Bytes", 0) or 0))
          for r in load(d, "memory_copy_trace")]
    cl = [k for k in ks if "k_col_lens" in k[2]]
    if not cl:
        print("no k_col_lens launches")
        return
    t0 = min(k[0] for k in cl) - 60_000_000   # the with-columns phase starts with alignment ahead of the first columns
    t1 = max(k[1] for k in cl)
    t2 = max(k[1] for k in ks)
    for label, a, b in (("with columns", t0, t1), ("records only", t1, t2)):
        kk = [k for k in ks if k[0] >= a and k[1] <= b]
        cc = [c for c in cs if c[0] >= a and c[1] <= b]
        span = (b - a) / 1e6
        busy = union([(s, e) for s, e, _ in kk]) / 1e6
        fam = defaultdict(float)
        for s, e, n in kk:
            fam[family(n)] += (e - s) / 1e6
        print(f"== {label}: span {span:.1f} ms, kernel busy (union) {busy:.1f} ms ({busy / span:.0%})")
        for n, t in sorted(fam.items(), key=lambda x: -x[1])[:16]:
            print(f"   {n:28s} {t:9.2f} ms")
        dirs = defaultdict(lambda: [0, 0, 0.0])
        for s, e, dr, by in cc:
            x = dirs[dr]
            x[0] += 1; x[1] += by; x[2] += (e - s) / 1e6
        for dr, (n, by, t) in dirs.items():
            print(f"   copies {dr:24s} n {n:6d}  {by / 1e6:9.1f} MB  {t:8.2f} ms  busy {union([(s, e) for s, e, d_, _ in cc if d_ == dr]) / 1e6:8.2f} ms")


if __name__ == "__main__":
    main(sys.argv[1])
