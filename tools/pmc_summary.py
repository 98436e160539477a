#!/usr/bin/env python3
"""Summarise rocprofv3 PMC csv output: per kernel, the sum of each counter over its dispatches."""
import csv, glob, os, sys, collections

def main(root, filt=""):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if filt and filt not in k:
                continue
            k = k.split("(")[0][:70]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add((f, r["Dispatch_Id"]))
    for k in sorted(agg):
        print(k, "dispatches(all passes)=%d" % len(disp[k]))
        for c in sorted(agg[k]):
            print("    %-28s %.6g" % (c, agg[k][c]))

if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
