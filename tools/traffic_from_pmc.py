#!/usr/bin/env python3
"""Per-launch HBM traffic of the alignment kernels from rocprofv3 PMC passes (tools/profile_round.sh).

FETCH_SIZE / WRITE_SIZE are summed per dispatch (KB -> bytes).  Correction (MI355X_MICROARCH.md, HBM
section: calibrate non-streaming widths on a known byte count): tools/calib_fetch.hip measured on the
same box gives FETCH_SIZE = 1.00 x bytes for random 64-B block gathers (the occ rank query, the
dominant access of every kernel here) and 0.5 x for 16-B/lane coalesced streaming; the kernels'
accesses are gathers, so the factor applied is the gather64 ratio.  Writes are taken as reported.
Usage: traffic_from_pmc.py <profile dir> <out json> <round tag>
"""
import csv, glob, json, os, sys

# stage -> kernels its HIP events bracket (the sorts' rocprim kernels are negligible and not counted)
KERNELS = {"smem": ["k_codes_wave", "k_smem_lds<", "k_smem_lanes<", "k_smem_sm", "k_pack_reads", "k_intv_sort"], "chain": ["k_chain_s", "k_chain<"],
           "extend": ["k_ext_key", "k_extend<"],
           "reg2aln": ["k_r2a_key", "k_reg2aln_diag", "k_reg2aln_g<16>", "k_reg2aln_g<32>", "bsq::k_reg2aln_w"]}


def per_dispatch(d, counter):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            out.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]) * 1024.0)
    return out


def main(root, dst, tag):
    cal = sorted((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"]) * 1024.0)
                 for f in glob.glob(os.path.join(root, "calib", "**", "*counter_collection.csv"), recursive=True)
                 for r in csv.DictReader(open(f)))
    cal = [c for c in cal if c[1].startswith("k_")]
    gib = float(1 << 30)
    names = ["stream_4G", "gather64_4G", "gather16_4G", "stream_96M_warm", "gather64_96M", "gather16_96M"]
    calib = {names[i]: round(c[2] / (gib if i != 3 else 96 * (1 << 20)), 4) for i, c in enumerate(cal[:6])}
    corr = calib.get("gather64_4G", 1.0)
    fetch, write = per_dispatch(os.path.join(root, "fetch"), "FETCH_SIZE"), per_dispatch(os.path.join(root, "write"), "WRITE_SIZE")
    # the profiled run: `--timed-only --streams 1 --steps 1 --warmup 0`, so every dispatch of a stage kernel belongs
    # to the one lone launch over all the reads (C4: ten 1M-read workspace chunks, one dispatch each)
    try:
        bj = json.load(open(os.path.join(root, "fetch.json")))
        rpl = bj["config"]["reads_per_launch"]
        launches = bj["steps"] * bj["config"]["streams"]
    except (OSError, KeyError, ValueError):
        rpl, launches = 1000000, 1
    res = {"round": tag, "reads_per_launch": rpl, "fetch_correction": 1.0 / corr,
           "calibration_fetch_size_over_bytes": calib, "kernels": {}}
    for stage, pats in KERNELS.items():
        fb = wb = 0.0
        names = []
        for pat in pats:
            fk = [k for k in fetch if pat in k]
            wk = [k for k in write if pat in k]
            if not fk or not wk:
                continue
            fb += sum(sum(fetch[k]) for k in fk) / launches
            wb += sum(sum(write[k]) for k in wk) / launches
            names.append(fk[0].split("(")[0])
        if names:
            res["kernels"][stage] = {"kernel": " + ".join(names), "fetch_bytes": fb / corr, "write_bytes": wb,
                                     "traffic_bytes": fb / corr + wb}
    json.dump(res, open(dst, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
