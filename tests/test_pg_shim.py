"""The drop-in BwaIndex shim (bioseqdb_amd/pg/bwa_bsq.cpp) compiles and links against libbsq with
plain g++ (no Postgres headers needed), and reports a missing GPU as BsqFailure, not a crash."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

MAIN = r'''
#include "bwa_bsq.h"
#include <cstdio>
#include <cstdlib>
#include <cstring>
int main() {
    size_t sz = 0;
    const char *rt = "ACGTTGCAACGTAGGCTAGCTAGGATCGATCGATTTACG", *qt = "GCAACGTAGGCTAGCTAGGATCG";
    void *ref = bsq_nuclseq_from_text(rt, strlen(rt), &sz);
    void *q = bsq_nuclseq_from_text(qt, strlen(qt), &sz);
    BwaIndex idx;
    idx.options->max_occ = 500;
    idx.add_ref_sequence(42, *static_cast<const NucleotideSequence *>(ref));
    idx.build();
    int rc = 0;
    try {
        auto m = idx.align_sequence(*static_cast<const NucleotideSequence *>(q));
        printf("rows %zu\n", m.size());
        rc = m.size() == 1 ? 0 : 3;
    } catch (const BsqFailure &e) {
        printf("failure %d %s\n", e.code, e.what());
        rc = e.code == BSQ_E_NODEV ? 0 : 2;
    }
    free(ref); free(q);
    return rc;
}
'''


def test_shim_compiles_links_and_runs(tmp_path):
    src = tmp_path / "main.cpp"
    src.write_text(MAIN)
    exe = tmp_path / "shim_test"
    pg = os.path.join(ROOT, "bioseqdb_amd", "pg")
    libdir = os.path.join(ROOT, "bioseqdb_amd")
    subprocess.run(["g++", "-std=c++17", "-O1", f"-I{pg}", f"-I{os.path.join(ROOT, 'include')}", str(src),
                    os.path.join(pg, "bwa_bsq.cpp"), f"-L{libdir}", "-lbsq", f"-Wl,-rpath,{libdir}", "-o", str(exe)],
                   check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
