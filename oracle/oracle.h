/*
 * oracle.h -- CPU oracle for the bioseqdb BWA alignment path.  TEST INFRASTRUCTURE ONLY.
 *
 * This is a clean-room restatement in plain C of
 *   - the bioseqdb wrapper (reference: bioseqdb/bwa.cpp, bioseqdb/extension.cpp,
 *     bioseqdb/sequence.{h,cpp}, bioseqdb/bioseqdb--0.0.0.sql), and
 *   - the third-party libbwa functions it calls (lh3/bwa, branch `Apache2`, unpinned in the
 *     reference: Dockerfile:6, .github/workflows/ci.yml:21).  libbwa is NOT vendored under
 *     /root/reference and is not present in this container; its algorithm is restated from the
 *     published BWA-MEM 0.7.x sources (bwt.c, bwamem.c, ksw.c, bntseq.c, bwa.c, kbtree.h,
 *     ksort.h) as written down in SURVEY.md Appendix A.
 *
 * Attribution: restates BWA (lh3/bwa, Apache License 2.0) and klib (MIT License); see NOTICE.
 *
 * Parity status: the reference's own tests (test/run.py) pin nothing on the alignment path and
 * ship no golden vectors, and libbwa cannot be built here.  The oracle is pinned by brute-force
 * cross-checks (FM counts, SMEMs, full-matrix DP) and planted-truth known-answer tests under
 * tests/, so alignment parity is "parity unpinned" against libbwa itself.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
 * and only as the checker / CPU baseline, never as the product path.
 */
#ifndef BSQ_ORACLE_H
#define BSQ_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- nuclseq codec (reference: bioseqdb/sequence.cpp:209-245, :71-81) ---------------------- */
/* Encodes `text` (len bytes) into the nuclseq varlena layout; returns malloc'd buffer, size in *out_size. */
uint8_t *orc_nuclseq_from_text(const char *text, size_t len, size_t *out_size);
/* Renders a nuclseq to text (malloc'd, NUL-terminated). */
char *orc_nuclseq_to_text(const uint8_t *nuclseq);
void orc_free(void *p);

/* ---- options: the *effective* mem_opt_t fields bioseqdb sets (extension.cpp:220-231) ---------- */
typedef struct {
    int32_t min_seed_len, max_occ, a, b, pen_clip3, pen_clip5, zdrop, w, o_del, e_del, o_ins, e_ins;
} orc_opts;

/* ---- BwaIndex (reference: bioseqdb/bwa.h:32-48, bwa.cpp:82-128) ------------------------------ */
typedef struct orc_index orc_index;
orc_index *orc_index_new(void);
void orc_index_free(orc_index *idx);
void orc_index_add_ref(orc_index *idx, int64_t id, const uint8_t *nuclseq);
/* Builds BWT/occ/SA with the oracle's own suffix sort. Returns 0 on success. */
int orc_index_build(orc_index *idx);
/* Builds BWT/occ/SA from an externally supplied suffix array of T$ (n+1 entries; sa_bytes = 4 or 8).
 * Used by the BASELINE-size parity fixtures and bench.py's cpu_baseline leg to skip the oracle's own
 * O(n log n) sort on 100 Mbp / 3 Gbp inputs.  The SA is certified on the host first (16 threads): every
 * value in [0, n], exactly one row 0, and adjacent rows' suffixes of T$ strictly increasing -- which
 * makes it a permutation and so the unique suffix array.  Returns 0 on success, -1 for a range/primary
 * fault, -2 for order violations (their count: orc_sa_violations). */
int orc_index_build_from_sa(orc_index *idx, const void *sa, int sa_bytes);
/* Order violations found by the last orc_index_build_from_sa (0 after a certified build). */
uint64_t orc_sa_violations(void);
int64_t orc_index_l_pac(const orc_index *idx);
int64_t orc_index_seq_len(const orc_index *idx);
int64_t orc_index_primary(const orc_index *idx);
/* Logical FM queries (restated bwt_occ4 / bwt_sa) for tests. */
void orc_index_occ4(const orc_index *idx, int64_t k, uint64_t cnt[4]);
int64_t orc_index_sa(const orc_index *idx, int64_t k);
void orc_index_l2(const orc_index *idx, uint64_t l2[5]);
/* 2-bit base of the concatenated forward text T[0..l_pac). */
int orc_index_pac_base(const orc_index *idx, int64_t pos);

/* ---- lrand48 stream (Q10) --------------------------------------------------------------------- */
/* Value returned by the (pos+1)-th call of glibc lrand48() from the unseeded state (X0 = 0). */
int64_t orc_lrand48_at(uint64_t pos);

/* ---- alignment ------------------------------------------------------------------------------- */
/* Aligns one nuclseq read (reference: BwaIndex::align_sequence, bwa.cpp:141-181) with the given
 * lrand48 value.  Returns a malloc'd TSV text, one line per bwa_result row (query_id excluded):
 *   ref_id ref_subseq ref_match_start ref_match_end ref_match_len query_subseq
 *   query_match_start query_match_end query_match_len is_primary is_secondary is_reverse cigar score
 * ref_subseq is "*" on reverse-strand rows (Q7: the reference reads out of bounds there). */
char *orc_align_tsv(const orc_index *idx, const orc_opts *opt, const uint8_t *nuclseq_read, int64_t lrand_id);

/* orc_align_tsv over n reads (nuclseq pointers) on `threads` POSIX threads, read r with lrand48 call
 * first_call + r; the rows concatenated in read order, rows_per_read[r] = rows of read r.  NULL if a read
 * is unsupported.  malloc'd (orc_free). */
char *orc_align_tsv_batch(const orc_index *idx, const orc_opts *opt, const uint8_t *const *reads, int n,
                          uint64_t first_call, int threads, int64_t *rows_per_read);

/* Raw alignment regions after mem_align1 (+ mem_reg2aln) for stage-level parity tests. */
typedef struct {
    int64_t rb, re;
    int32_t qb, qe, rid, score, truesc, sub, csub, sub_n, w, seedcov, secondary, seedlen0, n_comp;
    int32_t flag, is_rev, n_cigar;
    uint32_t cigar[64];
    uint64_t hash;
} orc_region;
/* Aligns nt4-coded query (values 0..4); writes up to max_regs regions; returns the number of regions
 * (which may exceed max_regs). */
int orc_align_regions(const orc_index *idx, const orc_opts *opt, const uint8_t *q_nt4, int len, int64_t lrand_id,
                      orc_region *out, int max_regs);

/* Collected SMEM intervals (mem_collect_intv), for stage tests: writes up to max entries of
 * (x0, x1, x2, info) quadruples; returns the count. */
int orc_collect_intv(const orc_index *idx, const orc_opts *opt, const uint8_t *q_nt4, int len, uint64_t *out, int max);
/* Seeding trace of one read for tools/seed_model.py (bwa_oracle.c tr_push); test infrastructure. */
int orc_seed_trace(const orc_index *idx, const orc_opts *o, const uint8_t *q, int len, int32_t *out, int cap);
int orc_ext_trace(const orc_index *idx, const orc_opts *o, const uint8_t *q, int len, int64_t id, int32_t *out, int cap);

/* Bench helper: aligns n reads (nt4 codes, concatenated, offsets[n+1]) with `threads` POSIX threads,
 * returning the number of regions and a 64-bit FNV checksum of (read, rb, re, qb, qe, score, flag,
 * cigar) in *checksum.  lrand ids: orc_lrand48_at(first_call + i). */
/* Seeding only over reads [0, n) (bench C2 cpu_baseline): returns the number of intervals; *checksum =
 * sum over reads of FNV(read, (x[0], x[2], info) of each interval). */
int64_t orc_seed_batch(const orc_index *idx, const orc_opts *opt, const uint8_t *codes, const int64_t *offsets, int n,
                       int threads, uint64_t *checksum);
int64_t orc_align_batch(const orc_index *idx, const orc_opts *opt, const uint8_t *codes, const int64_t *offsets,
                        int n, uint64_t first_call, int threads, uint64_t *checksum);

/* SURVEY.md 8(d) algorithmic bytes of the last orc_seed_batch / orc_align_batch, on libbwa's layout:
 * [0] occ blocks of bwt_extend x 64 B, [1] bwt_sa values x 8 B, [2] extension reference windows
 * ceil(bases/4) (bns_fetch_seq), [3] CIGAR / patch windows ceil(bases/4) (bns_get_seq). */
void orc_algo_bytes(uint64_t out[4]);

/* ksw restatements exposed for brute-force tests. */
/* r.score of ksw_align2(..., KSW_XSTART) (striped ksw_i16 emulated lane for lane; mem_seed_sw). */
int orc_ksw_align2_score(int qlen, const uint8_t *query, int tlen, const uint8_t *target, const int8_t *mat, int o_del,
                         int e_del, int o_ins, int e_ins);
int orc_ksw_extend2(int qlen, const uint8_t *query, int tlen, const uint8_t *target, const int8_t *mat,
                    int o_del, int e_del, int o_ins, int e_ins, int w, int end_bonus, int zdrop, int h0,
                    int *qle, int *tle, int *gtle, int *gscore, int *max_off);
int orc_ksw_global2(int qlen, const uint8_t *query, int tlen, const uint8_t *target, const int8_t *mat,
                    int o_del, int e_del, int o_ins, int e_ins, int w, int *n_cigar, uint32_t *cigar, int max_cigar);

#ifdef __cplusplus
}
#endif
#endif
