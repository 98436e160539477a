#!/usr/bin/env python3
"""tools/sq_deep.sh passes -> per-kernel JSON: where a kernel's wave cycles go (issue by class, waits) and the average
in-flight latency of its LDS and VMEM instructions (SQ_INST_LEVEL_x / SQ_INSTS_x, both in quad-cycles per the guide's
SQ units).  Usage: sq_deep_from_pmc.py <out dir> <config> <round tag>"""
import csv
import glob
import json
import os
import sys


def main(root, cfg, tag):
    tot = {}
    for f in glob.glob(os.path.join(root, f"sqd_{cfg}_p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            d = tot.setdefault(k, {})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    res = {"round": tag, "config": cfg, "basis": "one lone launch (--streams 1), sums over the kernel's dispatches", "kernels": {}}
    for k, c in tot.items():
        wc = c.get("SQ_WAVE_CYCLES", 0)
        if wc <= 0:
            continue
        e = {x: c[x] for x in sorted(c)}
        for a in ("WAIT_ANY", "WAIT_INST_ANY", "ACTIVE_INST_ANY", "ACTIVE_INST_VALU", "ACTIVE_INST_LDS", "ACTIVE_INST_VMEM",
                  "ACTIVE_INST_SCA", "WAIT_INST_LDS"):
            if "SQ_" + a in c:
                e["frac_" + a.lower()] = round(c["SQ_" + a] / wc, 4)
        if c.get("SQ_INSTS_LDS"):
            e["lds_latency_qcycles"] = round(c.get("SQ_INST_LEVEL_LDS", 0) / c["SQ_INSTS_LDS"], 1)
        if c.get("SQ_INSTS_VMEM_RD"):
            e["vmem_latency_qcycles"] = round(c.get("SQ_INST_LEVEL_VMEM", 0) / (c["SQ_INSTS_VMEM_RD"] + c.get("SQ_INSTS_VMEM_WR", 0)), 1)
        if c.get("SQ_ACTIVE_INST_VALU") and c.get("SQ_THREAD_CYCLES_VALU"):
            e["valu_lane_util"] = round(c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"]), 4)
        if c.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_bank_conflict_frac"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"], 4)
        res["kernels"][k] = e
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
