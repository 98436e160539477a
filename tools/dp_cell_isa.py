#!/usr/bin/env python3
"""Instructions per ksw_extend2 DP cell in k_extend<true, 1> (bench.py EXT_VALU_PER_CELL), counted in the gfx950 ISA.

Compiles align_kernels.hip to device assembly (CPU only), takes k_extend<true, 1>, and lists its innermost loops
that read the per-row score profile (v_bfe_u32) and are short (the DP cell loop, unrolled by two): instructions
by class, and VALU per cell.  Usage: python3 tools/dp_cell_isa.py
"""
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src = os.path.join(ROOT, "bioseqdb_amd", "csrc", "align_kernels.hip")
    with tempfile.TemporaryDirectory() as d:
        asm = os.path.join(d, "ak.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only",
                        "-S", "-o", asm, src], check=True)
        lines = open(asm).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_ZN3bsq8k_extendILb1ELi1EE.*:", l))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    L = lines[start:end]
    for h, l in enumerate(L):
        if "Inner Loop Header" not in l:
            continue
        j = h
        while not re.match(r"^\.LBB\S+:", L[j]):
            j -= 1
        lab = L[j].split(":")[0]
        k = h
        while k < len(L) and not (("s_cbranch" in L[k] or "s_branch" in L[k]) and L[k].strip().endswith(lab)):
            k += 1
        body = [x.strip() for x in L[j + 1:k + 1] if x.strip() and not x.strip().startswith(";") and not x.startswith(".")]
        if len(body) > 200 or not any(x.startswith("v_bfe_u32") for x in body):
            continue
        nv = sum(x.startswith("v_") for x in body)
        ns = sum(x.startswith("s_") for x in body)
        nd = sum(x.startswith("ds_") for x in body)
        cells = sum(x.startswith("v_bfe_u32") for x in body)
        print(f"{lab}: {len(body)} instructions ({nv} VALU, {ns} SALU, {nd} LDS) for {cells} cells: "
              f"{nv / cells:.1f} VALU per cell")


if __name__ == "__main__":
    main()
