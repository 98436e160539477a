"""The drop-in BwaIndex (bioseqdb_amd/pg/bwa_bsq.{h,cpp}, replacing bioseqdb/bwa.{h,cpp}) compiled with plain g++
against libbsq.  CPU: it links, builds an index and reports a missing GPU as BsqFailure (no crash, no CPU
fallback).  GPU: every BwaMatch field of align_sequence / align_sequences against the oracle, with IUPAC holes
in the reference rows and in the reads, padding bases (Q4) and the lrand48 stream continuing across calls."""
import os
import random
import subprocess

import pytest

import oracle_py as O
from bioseqdb_amd import NucleotideSequence, effective_opts
from bioseqdb_amd import bwa as B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# Reads "<n_refs> <max_occ>" then ref texts and read texts (one per line), aligns the reads as one batch with
# align_sequences, then one by one with align_sequence, printing every BwaMatch as a TSV row.
MAIN = r'''
#include "bwa_bsq.h"
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>
static void print(const BwaMatch &m) {
    printf("%lld\t%s\t%d\t%d\t%d\t%s\t%d\t%d\t%d\t%s\t%s\t%s\t%s\t%d\n", (long long)m.ref_id, m.ref_subseq.c_str(),
           m.ref_match_begin, m.ref_match_end, m.ref_match_len, m.query_subseq.c_str(), m.query_match_begin,
           m.query_match_end, m.query_match_len, m.is_primary ? "t" : "f", m.is_secondary ? "t" : "f",
           m.is_reverse ? "t" : "f", m.cigar.c_str(), m.score);
}
int main() {
    int n_refs = 0, n_reads = 0, max_occ = 0;
    std::cin >> n_refs >> n_reads >> max_occ;
    std::vector<void *> refs, reads;
    std::string t;
    BwaIndex idx;
    idx.options->max_occ = max_occ;
    idx.options->o_ins = 1; idx.options->e_del = 6; idx.options->e_ins = 1;   // bwa_opts() defaults after Q1
    for (int i = 0; i < n_refs; ++i) {
        std::cin >> t;
        size_t sz = 0;
        refs.push_back(bsq_nuclseq_from_text(t.data(), t.size(), &sz));
        idx.add_ref_sequence(1000 + 7 * i, *static_cast<const NucleotideSequence *>(refs.back()));
    }
    for (int i = 0; i < n_reads; ++i) {
        std::cin >> t;
        size_t sz = 0;
        reads.push_back(bsq_nuclseq_from_text(t.data(), t.size(), &sz));
    }
    try {
        idx.build();
        std::vector<const NucleotideSequence *> batch;
        for (void *r : reads) batch.push_back(static_cast<const NucleotideSequence *>(r));
        for (const auto &ms : idx.align_sequences(batch)) { for (const auto &m : ms) print(m); printf("--\n"); }
        for (const auto *r : batch) { for (const auto &m : idx.align_sequence(*r)) print(m); printf("--\n"); }
    } catch (const BsqFailure &e) {
        printf("failure %d %s\n", e.code, e.what());
        return e.code == BSQ_E_NODEV ? 3 : 2;
    }
    for (void *p : refs) bsq_free(p);
    for (void *p : reads) bsq_free(p);
    return 0;
}
'''


@pytest.fixture(scope="module")
def shim_exe(tmp_path_factory):
    d = tmp_path_factory.mktemp("shim")
    src = d / "main.cpp"
    src.write_text(MAIN)
    exe = d / "shim_test"
    pg = os.path.join(ROOT, "bioseqdb_amd", "pg")
    libdir = os.path.join(ROOT, "bioseqdb_amd")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", f"-I{pg}", f"-I{os.path.join(ROOT, 'include')}",
                    str(src), os.path.join(pg, "bwa_bsq.cpp"), f"-L{libdir}", "-lbsq", f"-Wl,-rpath,{libdir}", "-o",
                    str(exe)], check=True)
    return str(exe)


def _run(exe, refs, reads, max_occ=500):
    inp = f"{len(refs)} {len(reads)} {max_occ}\n" + "\n".join(refs + reads) + "\n"
    return subprocess.run([exe], input=inp, capture_output=True, text=True, timeout=300)


def test_shim_links_and_reports_no_device(shim_exe, gpu_available):
    r = _run(shim_exe, ["ACGTTGCAACGTAGGCTAGCTAGGATCGATCGATTTACG"], ["GCAACGTAGGCTAGCTAGGATCG"])
    if gpu_available:
        assert r.returncode == 0, r.stdout + r.stderr
    else:
        assert r.returncode == 3 and r.stdout.startswith("failure -4"), r.stdout + r.stderr


@pytest.mark.gpu
def test_shim_matches_oracle(shim_exe):
    rng = random.Random(3)
    refs = []
    for L in (90_001, 33, 60_002, 45_003):   # lengths not multiples of 4: padding bases (Q4)
        s = [rng.choice("ACGT") for _ in range(L)]
        for _ in range(L // 9000):
            p = rng.randrange(max(L - 50, 1))
            ch = rng.choice("NRYKMSWBDHV")
            for j in range(p, min(p + rng.randint(1, 40), L)):
                s[j] = ch
        refs.append("".join(s))
    cat = "".join(refs)
    comp = str.maketrans("ACGTNRYKMSWBDHV", "TGCANYRMKSWVHDB")
    reads = []
    for _ in range(400):
        L = rng.choice([150, 150, 120, 70, 36])
        p = rng.randrange(len(cat) - L)
        r = [c if rng.random() > 0.015 else rng.choice("ACGTN") for c in cat[p:p + L]]
        r = "".join(r)
        reads.append(r.translate(comp)[::-1] if rng.random() < 0.5 else r)
    r = _run(shim_exe, refs, reads, max_occ=500)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr
    blocks = r.stdout.split("--\n")[:-1]
    assert len(blocks) == 2 * len(reads)
    oi = O.OracleIndex()
    for i, t in enumerate(refs):
        oi.add_ref(1000 + 7 * i, O.Nuclseq(t).raw)
    oi.build()
    oo = O.opts_from(effective_opts(None, len(refs)))
    bad, rows = [], 0
    for k, blk in enumerate(blocks):   # batch pass: lrand48 calls 0..n-1; single pass: n..2n-1
        exp = B.parse_tsv(oi.align_tsv(oo, NucleotideSequence.from_text(reads[k % len(reads)]).raw, O.lrand48_at(k)))
        got = B.parse_tsv(blk)
        if len(got) != len(exp):
            bad.append((k, "n_rows", len(got), len(exp)))
            continue
        for g, e in zip(got, exp):
            rows += 1
            for f in ("ref_id", "ref_subseq", "ref_match_begin", "ref_match_end", "ref_match_len", "query_subseq",
                      "query_match_begin", "query_match_end", "query_match_len", "is_primary", "is_secondary",
                      "is_reverse", "cigar", "score"):
                if f == "ref_subseq" and e.is_reverse:
                    continue   # Q7
                if getattr(g, f) != getattr(e, f):
                    bad.append((k, f, getattr(g, f), getattr(e, f)))
    assert rows > 600
    assert not bad, bad[:10]
