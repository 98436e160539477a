#!/usr/bin/env python3
"""Per-stage SQ counters of one lone launch (tools/sq_round.sh passes) -> JSON for bench.py's `kernels.*.sq`.

Derived per stage (kernels as in traffic_from_pmc.py):
  valu_lane_util = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU)   active lanes per issued VALU cycle
  valu_busy      = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES                 share of resident-wave cycles issuing VALU
  wait_frac      = SQ_WAIT_ANY / SQ_WAVE_CYCLES                         share of wave cycles waiting on anything
Usage: sq_from_pmc.py <out dir> <config> <round tag>
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from traffic_from_pmc import KERNELS  # noqa: E402


def main(root, cfg, tag):
    tot = {}
    for f in glob.glob(os.path.join(root, f"sq_{cfg}_p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            for stage, pats in KERNELS.items():
                if any(p in k for p in pats):
                    d = tot.setdefault(stage, {})
                    d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    res = {"round": tag, "config": cfg, "basis": "one lone launch of the config's reads (--streams 1), sums over its dispatches",
           "stages": {}}
    for stage, c in tot.items():
        e = dict(c)
        if c.get("SQ_ACTIVE_INST_VALU"):
            e["valu_lane_util"] = round(c.get("SQ_THREAD_CYCLES_VALU", 0) / (64.0 * c["SQ_ACTIVE_INST_VALU"]), 4)
        if c.get("SQ_WAVE_CYCLES"):
            e["valu_busy"] = round(c.get("SQ_ACTIVE_INST_VALU", 0) / c["SQ_WAVE_CYCLES"], 4)
            e["wait_frac"] = round(c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"], 4)
        res["stages"][stage] = e
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
