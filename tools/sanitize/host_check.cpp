// host_check.cpp -- ASan/UBSan driver for the host code of the path ("Host: ASan/UBSan build of the
// oracle and shim").  Built by tools/sanitize/Makefile with -fsanitize=address,undefined together with the
// host-only translation units of libbsq (index_build.cpp: nuclseq codec + host index build; render.cpp: bwa_result
// rendering, Q3/Q7/Q8; fasta.cpp: bioseqdb-import's reader) and the CPU oracle (oracle/bwa_oracle.c).  The HIP
// side cannot run under a sanitizer here (no GPU, and GPU ASan is not available on the pool).
//
// Every check compares two independent implementations, so the run is also a differential test:
//   * nuclseq codec: libbsq vs oracle bytes, text round trips (holes, IUPAC runs, empty and 1-base texts);
//   * host index: suffix array and occ of libbsq's parallel host build vs the oracle's own suffix sort;
//   * rendering: bsq_render_tsv / bsq_index_ref_subseq over synthetic regions on both strands and across holes;
//   * FASTA: bsq_fasta_parse on ragged input;
//   * oracle alignment: orc_align_tsv_batch on 4 threads over planted and random reads.
// Exit status 0 = every check passed and no sanitizer report (the sanitizers abort on the first finding).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../include/bsq.h"
#include "../../bioseqdb_amd/csrc/bsq_index.h"
#include "../../oracle/oracle.h"

static int fails = 0;
#define CHECK(c, ...)                                     \
    do {                                                  \
        if (!(c)) {                                       \
            ++fails;                                      \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                 \
            fputc('\n', stderr);                          \
        }                                                 \
    } while (0)

static std::string rand_text(std::mt19937_64 &rng, size_t len, double hole_rate)
{
    static const char iupac[] = "NRYKMSWBDHV";
    std::string s(len, 'A');
    for (size_t i = 0; i < len; ++i) s[i] = "ACGT"[rng() & 3];
    for (size_t i = 0; i < len; ++i) {
        if ((double)(rng() % 1000000) / 1e6 < hole_rate) {
            const char c = iupac[rng() % 11];
            const size_t run = 1 + rng() % 12;
            for (size_t j = i; j < len && j < i + run; ++j) s[j] = c;
        }
    }
    return s;
}

static void check_codec(std::mt19937_64 &rng)
{
    for (int t = 0; t < 400; ++t) {
        const size_t len = t < 8 ? (size_t)t : rng() % 700;
        const std::string s = rand_text(rng, len, t % 3 ? 0.01 : 0.2);
        size_t a = 0, b = 0;
        void *x = bsq_nuclseq_from_text(s.data(), s.size(), &a);
        uint8_t *y = orc_nuclseq_from_text(s.data(), s.size(), &b);
        CHECK(x && y && a == b && memcmp(x, y, a) == 0, "codec bytes differ (len %zu)", len);
        char *u = bsq_nuclseq_to_text(x);
        char *v = orc_nuclseq_to_text(y);
        CHECK(u && v && s == u && s == v, "round trip differs (len %zu)", len);
        free(x); orc_free(y); free(u); orc_free(v);
    }
}

static void check_index_render(std::mt19937_64 &rng)
{
    for (int t = 0; t < 6; ++t) {
        std::vector<std::string> rows;
        const int n_rows = 1 + (int)(rng() % 4);
        for (int r = 0; r < n_rows; ++r) rows.push_back(rand_text(rng, rng() % 4000 + (t == 0 ? 0 : 5), 0.002));
        bsq_index idx;
        orc_index *oi = orc_index_new();
        std::vector<std::vector<uint8_t>> ns;
        for (int r = 0; r < n_rows; ++r) {
            size_t sz = 0;
            void *p = bsq_nuclseq_from_text(rows[r].data(), rows[r].size(), &sz);
            ns.emplace_back((uint8_t *)p, (uint8_t *)p + sz);
            free(p);
            idx.h.add_ref(100 + r, ns.back().data());
            orc_index_add_ref(oi, 100 + r, ns.back().data());
        }
        std::string err;
        CHECK(idx.h.build(4, err) == 0, "host build: %s", err.c_str());
        CHECK(orc_index_build(oi) == 0, "oracle build");
        const uint64_t n = idx.h.seq_len;
        CHECK((int64_t)n == orc_index_seq_len(oi), "seq_len");
        if (n) {
            CHECK((int64_t)idx.h.primary == orc_index_primary(oi), "primary");
            for (uint64_t r = 1; r <= n; ++r) CHECK((int64_t)idx.h.sa(r) == orc_index_sa(oi, (int64_t)r), "sa[%llu]", (unsigned long long)r);
            uint64_t c[4], d[4];
            for (int64_t k = -1; k <= (int64_t)n; ++k) {
                idx.h.occ4((uint64_t)k, c);
                orc_index_occ4(oi, k, d);
                CHECK(memcmp(c, d, sizeof c) == 0, "occ4(%lld)", (long long)k);
            }
            // rendering over synthetic regions: both strands, every hole overlay, every CIGAR op
            const int64_t lp = idx.h.l_pac;
            std::vector<bsq_hit> hits;
            std::vector<uint32_t> cig;
            std::vector<int64_t> off(1, 0);
            std::vector<std::vector<uint8_t>> reads;
            for (int q = 0; q < 50; ++q) {
                const std::string rt = rand_text(rng, 20 + rng() % 150, 0.01);
                size_t sz = 0;
                void *p = bsq_nuclseq_from_text(rt.data(), rt.size(), &sz);
                reads.emplace_back((uint8_t *)p, (uint8_t *)p + sz);
                free(p);
                const int nh = (int)(rng() % 3);
                for (int k = 0; k < nh && lp > 40; ++k) {
                    bsq_hit h{};
                    const bool rev = rng() & 1;
                    const int64_t len = 1 + (int64_t)(rng() % 30);
                    const int64_t rb = (int64_t)(rng() % (uint64_t)(lp - len)) + (rev ? lp : 0);
                    h.rb = rb; h.re = rb + len; h.qb = 0; h.qe = (int32_t)std::min<int64_t>(len, (int64_t)rt.size());
                    h.rid = 0; h.ref_id = 100; h.is_reverse = rev; h.is_primary = k == 0; h.is_secondary = k != 0;
                    h.read_index = q; h.score = (int32_t)len; h.cigar_off = (uint32_t)cig.size(); h.n_cigar = 3;
                    cig.push_back(1u << 4 | 3); cig.push_back((uint32_t)(len - 1) << 4 | 0); cig.push_back(2u << 4 | 1);
                    hits.push_back(h);
                    std::string out((size_t)len, '?');
                    CHECK(bsq_index_ref_subseq(&idx, h.rb, h.re, &out[0]) == len, "ref_subseq");
                }
                off.push_back((int64_t)hits.size());
            }
            std::vector<const void *> rp;
            for (auto &r : reads) rp.push_back(r.data());
            bsq_hits H{(int32_t)reads.size(), (int64_t)hits.size(), hits.data(), off.data(), (int64_t)cig.size(), cig.data()};
            char *tsv = bsq_render_tsv(&idx, &H, rp.data());
            size_t lines = 0;
            for (const char *p = tsv; p && *p; ++p) lines += *p == '\n';
            CHECK(tsv && lines == hits.size(), "render rows %zu vs %zu", lines, hits.size());
            free(tsv);
            CHECK(bsq_index_ref_subseq(&idx, -1, 5, nullptr) == -1 && bsq_index_ref_subseq(&idx, 0, 2 * lp + 1, nullptr) == -1,
                  "ref_subseq range checks");
        }
        // oracle alignment of planted and random reads on 4 threads
        if (n) {
            std::string cat;
            for (auto &r : rows) cat += r;
            std::vector<std::vector<uint8_t>> rq;
            for (int q = 0; q < 60; ++q) {
                std::string s;
                if (q % 3 && cat.size() > 200) {
                    const size_t p = rng() % (cat.size() - 150);
                    s = cat.substr(p, 40 + rng() % 110);
                    for (char &c : s) if (rng() % 60 == 0) c = "ACGTN"[rng() % 5];
                } else s = rand_text(rng, rng() % 160, 0.0);
                size_t sz = 0;
                uint8_t *p = orc_nuclseq_from_text(s.data(), s.size(), &sz);
                rq.emplace_back(p, p + sz);
                orc_free(p);
            }
            std::vector<const uint8_t *> qp;
            for (auto &r : rq) qp.push_back(r.data());
            const orc_opts o{19, 500, 1, 4, 5, 5, 100, 100, 6, 6, 1, 1};
            std::vector<int64_t> rows_per((size_t)qp.size());
            char *t4 = orc_align_tsv_batch(oi, &o, qp.data(), (int)qp.size(), 17, 4, rows_per.data());
            char *t1 = orc_align_tsv_batch(oi, &o, qp.data(), (int)qp.size(), 17, 1, rows_per.data());
            CHECK(t4 && t1 && strcmp(t4, t1) == 0, "oracle batch differs between 4 threads and 1");
            orc_free(t4); orc_free(t1);
        }
        orc_index_free(oi);
    }
}

static void check_fasta(std::mt19937_64 &rng)
{
    for (int t = 0; t < 50; ++t) {
        std::string f;
        const int nrec = (int)(rng() % 6);
        for (int r = 0; r < nrec; ++r) {
            f += ">rec" + std::to_string(r) + (rng() & 1 ? "\r\n" : "\n");
            const int nl = (int)(rng() % 4);
            for (int l = 0; l < nl; ++l) f += rand_text(rng, rng() % 90, 0.01) + "\n";
        }
        if (rng() & 1) f += "acgt";   // last line without a newline, lower case
        char *seq = nullptr, *names = nullptr;
        int64_t *so = nullptr, *no = nullptr, nr = 0;
        CHECK(bsq_fasta_parse(f.data(), (int64_t)f.size(), &seq, &so, &names, &no, &nr) == BSQ_OK, "fasta parse");
        CHECK(nr >= 0 && nr <= nrec + 1, "fasta records %lld", (long long)nr);
        free(seq); free(so); free(names); free(no);
    }
}

int main()
{
    std::mt19937_64 rng(20261016);
    check_codec(rng);
    check_index_render(rng);
    check_fasta(rng);
    printf("host_check: %s (%d failures)\n", fails ? "FAILED" : "ok", fails);
    return fails ? 1 : 0;
}
