/*
 * bwa_oracle.c -- CPU oracle (TEST INFRASTRUCTURE ONLY) for the bioseqdb BWA alignment path.
 *
 * Clean-room restatement of
 *   bioseqdb:  bwa.cpp:20-181 (BwaIndex), sequence.{h,cpp} (nuclseq codec), extension.cpp:197-236
 *   libbwa [lh3/bwa branch Apache2, not vendored, restated from the published 0.7.x sources]:
 *     bwt.c        bwt_occ4/bwt_2occ4/bwt_occ/bwt_extend/bwt_smem1a/bwt_seed_strategy1/bwt_sa,
 *                  bwt_bwtupdate_core, bwt_cal_sa, bwt_gen_cnt_table
 *     bwamem.c     mem_collect_intv, mem_chain (+ kbtree), mem_chain_flt, mem_chain2aln,
 *                  mem_sort_dedup_patch (+ mem_patch_reg), mem_mark_primary_se, mem_reg2aln
 *     ksw.c        ksw_extend2, ksw_global2
 *     bwa.c        bwa_gen_cigar2, bwa_fill_scmat
 *     bntseq.c     bns_pos2rid, bns_intv2rid, bns_depos, bns_get_seq, bns_fetch_seq
 *     ksort.h      ks_introsort / ks_combsort / insertion sort (tie order is parity-relevant)
 *     kbtree.h     B-tree with t = 5 for mem_chain_t (duplicate-key placement is parity-relevant)
 * See SURVEY.md Appendix A for the behavioural spec this follows.  Never linked into the product.
 */
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ============================================================================================== */
/* small utilities                                                                                */
/* ============================================================================================== */
#define VEC(T) struct { size_t n, m; T *a; }
#define VPUSH(v, x) do { if ((v).n == (v).m) { (v).m = (v).m ? (v).m << 1 : 4; \
    (v).a = realloc((v).a, sizeof(*(v).a) * (v).m); } (v).a[(v).n++] = (x); } while (0)
#define VGROW(v) do { if ((v).n == (v).m) { (v).m = (v).m ? (v).m << 1 : 4; \
    (v).a = realloc((v).a, sizeof(*(v).a) * (v).m); } } while (0)

void orc_free(void *p) { free(p); }

/* libbwa nst_nt4_table: A/C/G/T (either case) -> 0..3, '-' -> 5, everything else -> 4 */
static inline int nt4_of(unsigned char c)
{
    switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    case '-': return 5;
    default: return 4;
    }
}

/* ============================================================================================== */
/* nuclseq varlena codec (sequence.h:18-38, sequence.cpp:59-81, 162-166, 209-245)                 */
/* layout: vl_len[4] | holes_num u32 | len u32 | holes_num x {i64 offset, i32 len, char amb, pad3} | pac */
/* ============================================================================================== */
static inline uint32_t ns_u32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint32_t ns_holes_num(const uint8_t *ns) { return ns_u32(ns + 4); }
static inline uint32_t ns_len(const uint8_t *ns) { return ns_u32(ns + 8); }
static inline const uint8_t *ns_pac(const uint8_t *ns) { return ns + 12 + 16 * (size_t)ns_holes_num(ns); }
static inline size_t pac_byte_size(size_t x) { return x / 4 + (x % 4 != 0 ? 1 : 0); }   /* sequence.h:49 */
static inline int pac_raw_get(const uint8_t *pac, uint64_t i) { return pac[i >> 2] >> ((~i & 3) << 1) & 3; }
static inline void pac_raw_set(uint8_t *pac, uint64_t i, int v) { pac[i >> 2] |= (uint8_t)(v << ((~i & 3) << 1)); }

typedef struct { int64_t offset; int32_t len; char amb; } hole_t; /* bntamb1_t */

static inline hole_t ns_hole(const uint8_t *ns, uint32_t i)
{
    hole_t h; const uint8_t *p = ns + 12 + 16 * (size_t)i;
    memcpy(&h.offset, p, 8); memcpy(&h.len, p + 8, 4); h.amb = (char)p[12];
    return h;
}

/* std::minstd_rand: x <- x * 48271 mod (2^31 - 1), seeded with s mod m (0 -> 1) */
typedef struct { uint64_t x; } minstd_t;
static void minstd_seed(minstd_t *r, uint64_t s) { uint64_t v = s % 2147483647ULL; r->x = v ? v : 1; }
static uint32_t minstd_next(minstd_t *r) { r->x = (r->x * 48271ULL) % 2147483647ULL; return (uint32_t)r->x; }

/* nuclseq_from_text, sequence.cpp:209-245 (hole count: calculate_num_of_holes, :46-57) */
uint8_t *orc_nuclseq_from_text(const char *str, size_t len, size_t *out_size)
{
    uint32_t holes_num = 0; char prev = 0; size_t i;
    for (i = 0; i < len; ++i) {
        if (prev != str[i] && nt4_of((unsigned char)str[i]) >= 4) ++holes_num;
        prev = str[i];
    }
    size_t size = 12 + 16 * (size_t)holes_num + pac_byte_size(len);
    uint8_t *ns = calloc(1, size);
    uint32_t vl = (uint32_t)(size << 2), l32 = (uint32_t)len;   /* SET_VARSIZE, little-endian 4B header */
    memcpy(ns, &vl, 4); memcpy(ns + 4, &holes_num, 4); memcpy(ns + 8, &l32, 4);
    uint8_t *pac = ns + 12 + 16 * (size_t)holes_num;
    minstd_t rng; minstd_seed(&rng, (uint64_t)holes_num ^ (uint64_t)len);
    uint8_t *hole = ns + 12 - 16; prev = 0;
    for (i = 0; i < len; ++i) {
        char c = str[i]; int code = nt4_of((unsigned char)c);
        if (code >= 4) {
            if (prev == c) {
                int32_t hl; memcpy(&hl, hole + 8, 4); ++hl; memcpy(hole + 8, &hl, 4);
            } else {
                hole += 16;
                int64_t off = (int64_t)i; int32_t hl = 1;
                memcpy(hole, &off, 8); memcpy(hole + 8, &hl, 4); hole[12] = (uint8_t)c;
            }
            pac_raw_set(pac, i, minstd_next(&rng) & 3);
        } else pac_raw_set(pac, i, code);
        prev = c;
    }
    for (i = len; i < pac_byte_size(len) * 4; ++i) pac_raw_set(pac, i, minstd_next(&rng) & 3);
    if (out_size) *out_size = size;
    return ns;
}

/* to_text_palloc / inplace_to_text, sequence.cpp:71-81 */
char *orc_nuclseq_to_text(const uint8_t *ns)
{
    uint32_t len = ns_len(ns), nh = ns_holes_num(ns), i;
    const uint8_t *pac = ns_pac(ns);
    char *t = malloc((size_t)len + 1);
    for (i = 0; i < len; ++i) t[i] = "ACGT"[pac_raw_get(pac, i)];
    for (i = 0; i < nh; ++i) {
        hole_t h = ns_hole(ns, i);
        for (int64_t j = h.offset; j < h.offset + h.len; ++j) t[j] = h.amb;
    }
    t[len] = 0;
    return t;
}

/* ============================================================================================== */
/* ksort.h restatement: ks_introsort with klib's exact pivot/partition/insertion-sort sequence     */
/* ============================================================================================== */
typedef int (*lt_fn)(const void *a, const void *b);

static inline void swap_bytes(char *a, char *b, size_t sz, char *tmp)
{ memcpy(tmp, a, sz); memcpy(a, b, sz); memcpy(b, tmp, sz); }

static void ks_insertsort(char *s, char *t, size_t sz, lt_fn lt, char *tmp)
{
    for (char *i = s + sz; i < t; i += sz)
        for (char *j = i; j > s && lt(j, j - sz); j -= sz) swap_bytes(j, j - sz, sz, tmp);
}

static void ks_combsort(size_t n, char *a, size_t sz, lt_fn lt, char *tmp)
{
    const double shrink_factor = 1.2473309501039786540366528676643;
    int do_swap; size_t gap = n;
    do {
        if (gap > 2) {
            gap = (size_t)(gap / shrink_factor);
            if (gap == 9 || gap == 10) gap = 11;
        }
        do_swap = 0;
        for (char *i = a; i < a + (n - gap) * sz; i += sz) {
            char *j = i + gap * sz;
            if (lt(j, i)) { swap_bytes(i, j, sz, tmp); do_swap = 1; }
        }
    } while (do_swap || gap > 2);
    if (gap != 1) ks_insertsort(a, a + n * sz, sz, lt, tmp);
}

typedef struct { char *left, *right; int depth; } ks_stack_t;

static void ks_introsort(size_t n, void *a_, size_t sz, lt_fn lt)
{
    char *a = a_, *s, *t, *i, *j, *k;
    char *rp = malloc(sz), *tmp = malloc(sz);
    int d;
    if (n < 1) goto done;
    if (n == 2) {
        if (lt(a + sz, a)) swap_bytes(a, a + sz, sz, tmp);
        goto done;
    }
    for (d = 2; (1ul << d) < n; ++d);
    ks_stack_t *stack = malloc(sizeof(ks_stack_t) * ((sizeof(size_t) * d) + 2)), *top = stack;
    s = a; t = a + (n - 1) * sz; d <<= 1;
    while (1) {
        if (s < t) {
            if (--d == 0) {
                ks_combsort((size_t)(t - s) / sz + 1, s, sz, lt, tmp);
                t = s;
                continue;
            }
            i = s; j = t; k = i + ((((size_t)(j - i) / sz) >> 1) + 1) * sz;
            if (lt(k, i)) {
                if (lt(k, j)) k = j;
            } else k = lt(j, i) ? i : j;
            memcpy(rp, k, sz);
            if (k != t) swap_bytes(k, t, sz, tmp);
            for (;;) {
                do i += sz; while (lt(i, rp));
                do j -= sz; while (i <= j && lt(rp, j));
                if (j <= i) break;
                swap_bytes(i, j, sz, tmp);
            }
            swap_bytes(i, t, sz, tmp);
            if (i - s > t - i) {
                if ((size_t)(i - s) > 16 * sz) { top->left = s; top->right = i - sz; top->depth = d; ++top; }
                s = (size_t)(t - i) > 16 * sz ? i + sz : t;
            } else {
                if ((size_t)(t - i) > 16 * sz) { top->left = i + sz; top->right = t; top->depth = d; ++top; }
                t = (size_t)(i - s) > 16 * sz ? i - sz : s;
            }
        } else {
            if (top == stack) {
                free(stack);
                ks_insertsort(a, a + n * sz, sz, lt, tmp);
                goto done;
            } else { --top; s = top->left; t = top->right; d = top->depth; }
        }
    }
done:
    free(rp); free(tmp);
}

/* ============================================================================================== */
/* index: BwaIndex (bwa.cpp:82-128) + libbwa bwt_t                                                 */
/* ============================================================================================== */
typedef struct { int64_t offset; int32_t len, n_ambs; int64_t id; } ann_t;   /* bntann1_t subset */

struct orc_index {
    VEC(uint8_t) pac;      /* pac_forward */
    VEC(hole_t) holes;     /* unshifted hole offsets (Q3) */
    VEC(ann_t) anns;
    int built;
    int64_t l_pac;
    /* bwt_t */
    uint64_t primary, L2[5], seq_len, bwt_size;
    uint32_t *bwt;         /* interleaved: per 128 bases 4 x u64 counts then 8 x u32 bases */
    uint32_t cnt_table[256];
    int sa_intv;
    uint64_t n_sa, *sa;
};

orc_index *orc_index_new(void) { return calloc(1, sizeof(orc_index)); }

void orc_index_free(orc_index *idx)
{
    if (!idx) return;
    free(idx->pac.a); free(idx->holes.a); free(idx->anns.a); free(idx->bwt); free(idx->sa); free(idx);
}

/* BwaIndex::add_ref_sequence, bwa.cpp:82-105 */
void orc_index_add_ref(orc_index *idx, int64_t id, const uint8_t *ns)
{
    uint32_t len = ns_len(ns), nh = ns_holes_num(ns);
    ann_t an = { (int64_t)idx->pac.n * 4, (int32_t)len, (int32_t)nh, id };
    VPUSH(idx->anns, an);
    size_t nb = pac_byte_size(len);
    const uint8_t *pac = ns_pac(ns);
    for (size_t i = 0; i < nb; ++i) VPUSH(idx->pac, pac[i]);
    for (uint32_t i = 0; i < nh; ++i) { hole_t h = ns_hole(ns, i); VPUSH(idx->holes, h); } /* Q3: unshifted */
}

int64_t orc_index_l_pac(const orc_index *idx) { return idx->l_pac; }
int64_t orc_index_seq_len(const orc_index *idx) { return (int64_t)idx->seq_len; }
int64_t orc_index_primary(const orc_index *idx) { return (int64_t)idx->primary; }
void orc_index_l2(const orc_index *idx, uint64_t l2[5]) { memcpy(l2, idx->L2, sizeof idx->L2); }
int orc_index_pac_base(const orc_index *idx, int64_t pos) { return pac_raw_get(idx->pac.a, (uint64_t)pos); }

/* pac2bwt text: T = forward (4 x bytes bases incl. padding) || reverse complement (bwa.cpp:20-53) */
static uint8_t *make_text(const orc_index *idx, uint64_t *n_out, uint64_t L2[5])
{
    uint64_t pac_len = (uint64_t)idx->pac.n * 4, n = pac_len * 2, i;
    uint8_t *buf = malloc(n + 1);
    memset(L2, 0, 5 * sizeof(uint64_t));
    for (i = 0; i < pac_len; ++i) {
        buf[i] = (uint8_t)pac_raw_get(idx->pac.a, i);
        L2[1 + buf[i]]++; L2[4 - buf[i]]++;
    }
    for (i = 0; i < pac_len; ++i) buf[2 * pac_len - 1 - i] = (uint8_t)(3 - pac_raw_get(idx->pac.a, i));
    for (i = 2; i <= 4; ++i) L2[i] += L2[i - 1];
    buf[n] = 0;
    *n_out = n;
    return buf;
}

/* Suffix array of T$ (n+1 suffixes, $ unique and smallest) by prefix doubling with two counting
 * sorts per round.  Any correct suffix sort gives the same array as libbwa is_sa (the SA of T$ is
 * unique), so this is an independent construction, not a restatement of is.c. */
static int64_t *suffix_sort(const uint8_t *T, uint64_t n)
{
    uint64_t N = n + 1, i, h;
    int64_t *sa = malloc(N * 8), *rk = malloc(N * 8), *tmp = malloc(N * 8), *cnt, *sa2 = malloc(N * 8);
    uint64_t K = (N > 6 ? N : 6) + 1;
    cnt = calloc(K + 1, 8);
    for (i = 0; i < n; ++i) rk[i] = T[i] + 1;
    rk[n] = 0;
    for (i = 0; i < N; ++i) cnt[rk[i]]++;
    for (i = 1; i <= K; ++i) cnt[i] += cnt[i - 1];
    for (i = N; i-- > 0;) sa[--cnt[rk[i]]] = (int64_t)i;
    /* initial ranks: class ids of first character */
    tmp[sa[0]] = 0;
    for (i = 1; i < N; ++i) tmp[sa[i]] = tmp[sa[i - 1]] + (rk[sa[i]] != rk[sa[i - 1]]);
    memcpy(rk, tmp, N * 8);
    for (h = 1; rk[sa[N - 1]] < (int64_t)N - 1; h <<= 1) {
        /* sort by second key rk[i+h] (0 -> shorter, use -1 shifted by +1) then stable by first key */
        memset(cnt, 0, (K + 1) * 8);
        for (i = 0; i < N; ++i) cnt[(i + h < N ? rk[i + h] + 1 : 0)]++;
        for (i = 1; i <= K; ++i) cnt[i] += cnt[i - 1];
        for (i = N; i-- > 0;) { uint64_t key = i + h < N ? (uint64_t)rk[i + h] + 1 : 0; sa2[--cnt[key]] = (int64_t)i; }
        memset(cnt, 0, (K + 1) * 8);
        for (i = 0; i < N; ++i) cnt[rk[i]]++;
        for (i = 1; i <= K; ++i) cnt[i] += cnt[i - 1];
        for (i = N; i-- > 0;) { int64_t s = sa2[i]; sa[--cnt[rk[s]]] = s; }
        tmp[sa[0]] = 0;
        for (i = 1; i < N; ++i) {
            int64_t a = sa[i], b = sa[i - 1];
            int64_t a2 = (uint64_t)a + h < N ? rk[a + h] : -1, b2 = (uint64_t)b + h < N ? rk[b + h] : -1;
            tmp[a] = tmp[b] + (rk[a] != rk[b] || a2 != b2);
        }
        memcpy(rk, tmp, N * 8);
    }
    free(rk); free(tmp); free(cnt); free(sa2);
    return sa;
}

/* bwt_gen_cnt_table */
static void gen_cnt_table(orc_index *b)
{
    for (int i = 0; i != 256; ++i) {
        uint32_t x = 0;
        for (int j = 0; j != 4; ++j)
            x |= (uint32_t)(((i & 3) == j) + ((i >> 2 & 3) == j) + ((i >> 4 & 3) == j) + (i >> 6 == j)) << (j << 3);
        b->cnt_table[i] = x;
    }
}

/* Fill bwt_t from T and its SA: is_bwt ($-removed BWT + primary), bwt packing (bwa.cpp:48-50),
 * bwt_bwtupdate_core (occ interleave every 128), bwt_cal_sa(32) (sampled true SA, sa[0] = -1). */
/* BWT of T$ from its suffix array and libbwa's interleaved occ layout (bwt_bwtupdate_core), on up to 16 POSIX
 * threads: a 3 Gbp text has 6e9 rows (bench.py --config c4 builds its CPU-baseline index this way). */
typedef struct {
    const uint8_t *T; const int64_t *sa64; const void *sa_ext; int sa_bytes;
    uint64_t n, lo, hi, primary, found, bad;   /* rows [lo, hi) / words [lo, hi) */
    uint32_t *raw, *buf; uint64_t cnt[4];
} bwt_job;

static uint64_t sa_at(const bwt_job *j, uint64_t r)
{
    return j->sa64 ? (uint64_t)j->sa64[r] : (j->sa_bytes == 4 ? (uint64_t)((const uint32_t *)j->sa_ext)[r]
                                                               : ((const uint64_t *)j->sa_ext)[r]);
}

static void *bwt_find_primary(void *a)
{
    bwt_job *j = a;
    j->found = (uint64_t)-1; j->bad = 0;
    for (uint64_t i = j->lo; i < j->hi; ++i) {
        const uint64_t s = sa_at(j, i);
        if (s > j->n) j->bad = 1;
        else if (s == 0) j->found = i;
    }
    return NULL;
}

static void *bwt_fill_words(void *a)   /* raw word w holds BWT characters 16w .. 16w+15 ($ row skipped) */
{
    bwt_job *j = a;
    for (uint64_t w = j->lo; w < j->hi; ++w) {
        uint32_t v = 0;
        for (uint64_t t = 0; t < 16; ++t) {
            const uint64_t pos = 16 * w + t;
            if (pos >= j->n) break;
            const uint64_t row = pos + (pos >= j->primary);
            v |= (uint32_t)j->T[sa_at(j, row) - 1] << ((15 - t) << 1);
        }
        j->raw[w] = v;
    }
    return NULL;
}

static void *bwt_count(void *a)   /* per-thread base counts over characters [lo, hi) (multiples of 128) */
{
    bwt_job *j = a;
    memset(j->cnt, 0, sizeof j->cnt);
    for (uint64_t i = j->lo; i < j->hi; ++i) ++j->cnt[j->raw[i >> 4] >> ((~i & 0xf) << 1) & 3];
    return NULL;
}

static void *bwt_interleave(void *a)   /* occ block b = counts before it (8 words) + its 8 BWT words */
{
    bwt_job *j = a;
    uint64_t c[4] = {j->cnt[0], j->cnt[1], j->cnt[2], j->cnt[3]};
    for (uint64_t i = j->lo; i < j->hi; ++i) {
        uint64_t k = (i >> 7) * 16 + ((i & 127) >> 4) + 8;
        if (i % 128 == 0) memcpy(j->buf + (i >> 7) * 16, c, 32);
        if (i % 16 == 0) j->buf[k] = j->raw[i / 16];
        ++c[j->raw[i >> 4] >> ((~i & 0xf) << 1) & 3];
    }
    return NULL;
}

static void run_jobs(bwt_job *jobs, int nt, void *(*fn)(void *))
{
    pthread_t th[16];
    for (int t = 1; t < nt; ++t) pthread_create(&th[t], NULL, fn, &jobs[t]);
    fn(&jobs[0]);
    for (int t = 1; t < nt; ++t) pthread_join(th[t], NULL);
}

/* Suffix a of T$ (T[n] = $, smaller than every base) strictly below suffix b?  Eight characters per step:
 * T holds one base 0..3 per byte, so a big-endian word compare is the lexicographic one. */
static int suffix_less(const uint8_t *T, uint64_t n, uint64_t a, uint64_t b)
{
    while (a + 8 <= n && b + 8 <= n) {
        uint64_t x, y;
        memcpy(&x, T + a, 8); memcpy(&y, T + b, 8);
        if (x != y) return __builtin_bswap64(x) < __builtin_bswap64(y);
        a += 8; b += 8;
    }
    for (;; ++a, ++b) {
        if (a == n || b == n) return a == n && b != n;   /* $ ends the shorter suffix; a == b is no order */
        if (T[a] != T[b]) return T[a] < T[b];
    }
}

/* The host certificate of an SA handed in from outside (orc_index_build_from_sa): rows [lo, hi) must hold
 * strictly increasing suffixes (row hi-1 against row hi too).  With every value already checked to lie in
 * [0, n] (bwt_find_primary), n+1 strictly increasing suffixes are n+1 distinct positions of n+1: the array
 * is a permutation, hence THE suffix array of T$, so the BWT and occ built from it are libbwa's. */
static void *sa_check_order(void *a)
{
    bwt_job *j = a;
    j->bad = 0;
    if (j->lo >= j->hi) return NULL;
    uint64_t prev = sa_at(j, j->lo);
    for (uint64_t i = j->lo + 1; i <= j->hi && i <= j->n; ++i) {
        if (i + 32 <= j->n) __builtin_prefetch(j->T + sa_at(j, i + 32));   /* one random line per row */
        const uint64_t s = sa_at(j, i);
        j->bad += !suffix_less(j->T, j->n, prev, s);
        prev = s;
    }
    return NULL;
}

static uint64_t orc_sa_violations_last;
uint64_t orc_sa_violations(void) { return orc_sa_violations_last; }

static int finish_bwt(orc_index *idx, const uint8_t *T, uint64_t n, const int64_t *sa64, const void *sa_ext, int sa_bytes)
{
    uint64_t i, c[4];
    const int nt = n < (1u << 20) ? 1 : 16;
    bwt_job jobs[16];
    for (int t = 0; t < nt; ++t) {
        memset(&jobs[t], 0, sizeof jobs[t]);
        jobs[t].T = T; jobs[t].sa64 = sa64; jobs[t].sa_ext = sa_ext; jobs[t].sa_bytes = sa_bytes; jobs[t].n = n;
    }
    idx->seq_len = n;
    idx->bwt_size = (n + 15) >> 4;
    /* the $ row (primary): SA[primary] == 0 */
    for (int t = 0; t < nt; ++t) { jobs[t].lo = (n + 1) * (uint64_t)t / nt; jobs[t].hi = (n + 1) * (uint64_t)(t + 1) / nt; }
    run_jobs(jobs, nt, bwt_find_primary);
    uint64_t primary = (uint64_t)-1, nfound = 0;
    for (int t = 0; t < nt; ++t) {
        if (jobs[t].bad) return -1;
        if (jobs[t].found != (uint64_t)-1) { primary = jobs[t].found; ++nfound; }
    }
    if (nfound != 1) return -1;
    if (!sa64) {   /* an SA from outside (the GPU build): certify order, which with the range implies permutation */
        for (int t = 0; t < nt; ++t) { jobs[t].lo = (n + 1) * (uint64_t)t / nt; jobs[t].hi = (n + 1) * (uint64_t)(t + 1) / nt; }
        run_jobs(jobs, nt, sa_check_order);
        uint64_t bad = 0;
        for (int t = 0; t < nt; ++t) bad += jobs[t].bad;
        orc_sa_violations_last = bad;
        if (bad) return -2;
    }
    idx->primary = primary;
    uint32_t *raw = calloc(idx->bwt_size + 1, 4);
    for (int t = 0; t < nt; ++t) {
        jobs[t].raw = raw; jobs[t].primary = primary;
        jobs[t].lo = idx->bwt_size * (uint64_t)t / nt; jobs[t].hi = idx->bwt_size * (uint64_t)(t + 1) / nt;
    }
    run_jobs(jobs, nt, bwt_fill_words);
    /* bwt_bwtupdate_core */
    uint64_t n_occ = (n + 127) / 128 + 1;
    idx->bwt_size += n_occ * 8;
    uint32_t *buf = calloc(idx->bwt_size, 4);
    const uint64_t nblk = (n + 127) / 128;
    for (int t = 0; t < nt; ++t) {
        jobs[t].buf = buf;
        jobs[t].lo = nblk * (uint64_t)t / nt * 128; jobs[t].hi = nblk * (uint64_t)(t + 1) / nt * 128;
        if (jobs[t].hi > n) jobs[t].hi = n;
        if (jobs[t].lo > n) jobs[t].lo = n;
    }
    run_jobs(jobs, nt, bwt_count);
    c[0] = c[1] = c[2] = c[3] = 0;
    for (int t = 0; t < nt; ++t) {   /* exclusive prefix of the per-thread counts */
        uint64_t x[4] = {jobs[t].cnt[0], jobs[t].cnt[1], jobs[t].cnt[2], jobs[t].cnt[3]};
        memcpy(jobs[t].cnt, c, 32);
        for (int b = 0; b < 4; ++b) c[b] += x[b];
    }
    run_jobs(jobs, nt, bwt_interleave);
    /* the counts after the last (possibly partial) block */
    const uint64_t fin = (n >> 7) * 16 + ((n & 127) ? 8 + (((n & 127) + 15) >> 4) : 0);
    if (fin + 8 != idx->bwt_size) { free(raw); free(buf); return -1; }
    memcpy(buf + fin, c, 32);
    free(raw);
    idx->bwt = buf;
    /* bwt_cal_sa(bwt, 32): samples of the true SA at rows multiple of 32; sa[0] = -1 */
    idx->sa_intv = 32;
    idx->n_sa = (n + 32) / 32;
    idx->sa = calloc(idx->n_sa, 8);
    for (i = 0; i <= n; i += 32) idx->sa[i / 32] = sa_at(&jobs[0], i);
    idx->sa[0] = (uint64_t)-1;
    gen_cnt_table(idx);
    idx->built = 1;
    return 0;
}

/* BwaIndex::build, bwa.cpp:107-128 */
int orc_index_build(orc_index *idx)
{
    if (idx->pac.n == 0) return 0;   /* reference returns with index == nullptr */
    uint64_t n;
    uint8_t *T = make_text(idx, &n, idx->L2);
    idx->l_pac = (int64_t)idx->pac.n * 4;
    int64_t *sa = suffix_sort(T, n);
    int r = finish_bwt(idx, T, n, sa, NULL, 0);
    free(sa); free(T);
    return r;
}

int orc_index_build_from_sa(orc_index *idx, const void *sa, int sa_bytes)
{
    if (idx->pac.n == 0) return 0;
    uint64_t n;
    uint8_t *T = make_text(idx, &n, idx->L2);
    idx->l_pac = (int64_t)idx->pac.n * 4;
    int r = finish_bwt(idx, T, n, NULL, sa, sa_bytes);
    free(T);
    return r;
}

/* ---- rank / SA (bwt.c) ---------------------------------------------------------------------- */
#define bwt_occ_intv(b, k) ((b)->bwt + ((k) >> 7 << 4))
#define bwt_bwt(b, k) ((b)->bwt[((k) >> 7 << 4) + 8 + (((k) & 0x7f) >> 4)])
#define bwt_B0(b, k) (bwt_bwt(b, k) >> ((~(k) & 0xf) << 1) & 3)
#define occ_aux4(b, w) ((b)->cnt_table[(w) & 0xff] + (b)->cnt_table[(w) >> 8 & 0xff] \
                        + (b)->cnt_table[(w) >> 16 & 0xff] + (b)->cnt_table[(w) >> 24])

static inline int occ_aux(uint64_t y, int c)
{
    y = ((c & 2) ? y : ~y) >> 1 & ((c & 1) ? y : ~y) & 0x5555555555555555ull;
    y = (y & 0x3333333333333333ull) + (y >> 2 & 0x3333333333333333ull);
    return (int)(((y + (y >> 4)) & 0xf0f0f0f0f0f0f0full) * 0x101010101010101ull >> 56);
}

static uint64_t bwt_occ(const orc_index *b, uint64_t k, int c)
{
    uint64_t n; const uint32_t *p, *end;
    if (k == b->seq_len) return b->L2[c + 1] - b->L2[c];
    if (k == (uint64_t)-1) return 0;
    k -= (k >= b->primary);
    p = bwt_occ_intv(b, k);
    memcpy(&n, (const uint64_t *)p + c, 8);
    p += 8;
    end = p + (((k >> 5) - ((k & ~(uint64_t)127) >> 5)) << 1);
    for (; p < end; p += 2) n += occ_aux((uint64_t)p[0] << 32 | p[1], c);
    n += occ_aux(((uint64_t)p[0] << 32 | p[1]) & ~((1ull << ((~k & 31) << 1)) - 1), c);
    if (c == 0) n -= ~k & 31;
    return n;
}

static void bwt_occ4(const orc_index *b, uint64_t k, uint64_t cnt[4])
{
    uint64_t x; const uint32_t *p, *end; uint32_t tmp;
    if (k == (uint64_t)-1) { memset(cnt, 0, 32); return; }
    k -= (k >= b->primary);
    p = bwt_occ_intv(b, k);
    memcpy(cnt, p, 32);
    p += 8;
    end = p + ((k >> 4) - ((k & ~(uint64_t)127) >> 4));
    for (x = 0; p < end; ++p) x += occ_aux4(b, *p);
    tmp = *p & ~((1U << ((~k & 15) << 1)) - 1);
    x += occ_aux4(b, tmp) - (~k & 15);
    cnt[0] += x & 0xff; cnt[1] += x >> 8 & 0xff; cnt[2] += x >> 16 & 0xff; cnt[3] += x >> 24;
}

void orc_index_occ4(const orc_index *idx, int64_t k, uint64_t cnt[4]) { bwt_occ4(idx, (uint64_t)k, cnt); }

typedef struct { uint64_t x[3], info; } bwtintv_t;

/* SURVEY.md section 8(d) algorithmic bytes, counted on libbwa's own layout (the figure behind the bench's
 * roofline `achieved`): [0] 64 B per occ block a bwt_extend touches (bwt_2occ4: one block when both
 * ranks share a 128-base interval, else two; a rank of -1 reads nothing), [1] 8 B per bwt_sa value,
 * [2] ceil(bases/4) per reference window of the extension (bns_fetch_seq), [3] the same for the windows
 * of CIGAR generation and patching (bns_get_seq).  Per thread, summed per batch (orc_algo_bytes). */
static __thread uint64_t orc_ab[4];
static uint64_t orc_ab_last[4];
void orc_algo_bytes(uint64_t out[4]) { memcpy(out, orc_ab_last, sizeof orc_ab_last); }

/* bwt_extend (bwt_2occ4 yields exactly two bwt_occ4 results) */
static void bwt_extend(const orc_index *b, const bwtintv_t *ik, bwtintv_t ok[4], int is_back)
{
    uint64_t tk[4], tl[4];
    {
        const uint64_t k = ik->x[!is_back] - 1, l = k + ik->x[2];
        const uint64_t kk = k - (k >= b->primary), ll = l - (l >= b->primary);
        orc_ab[0] += k == (uint64_t)-1 || (kk >> 7) == (ll >> 7) ? 64 : 128;
    }
    bwt_occ4(b, ik->x[!is_back] - 1, tk);
    bwt_occ4(b, ik->x[!is_back] - 1 + ik->x[2], tl);
    for (int i = 0; i != 4; ++i) {
        ok[i].x[!is_back] = b->L2[i] + 1 + tk[i];
        ok[i].x[2] = tl[i] - tk[i];
    }
    ok[3].x[is_back] = ik->x[is_back] + (ik->x[!is_back] <= b->primary && ik->x[!is_back] + ik->x[2] - 1 >= b->primary);
    ok[2].x[is_back] = ok[3].x[is_back] + ok[3].x[2];
    ok[1].x[is_back] = ok[2].x[is_back] + ok[2].x[2];
    ok[0].x[is_back] = ok[1].x[is_back] + ok[1].x[2];
}

static inline uint64_t bwt_invPsi(const orc_index *b, uint64_t k)
{
    uint64_t x = k - (k > b->primary);
    x = bwt_B0(b, x);
    x = b->L2[x] + bwt_occ(b, k, (int)x);
    return k == b->primary ? 0 : x;
}

static uint64_t bwt_sa(const orc_index *b, uint64_t k)
{
    orc_ab[1] += 8;
    uint64_t sa = 0, mask = (uint64_t)b->sa_intv - 1;
    while (k & mask) { ++sa; k = bwt_invPsi(b, k); }
    return sa + b->sa[k / b->sa_intv];
}

int64_t orc_index_sa(const orc_index *idx, int64_t k) { return (int64_t)bwt_sa(idx, (uint64_t)k); }

#define bwt_set_intv(b, c, ik) ((ik).x[0] = (b)->L2[(int)(c)] + 1, (ik).x[2] = (b)->L2[(int)(c) + 1] - (b)->L2[(int)(c)], \
                                (ik).x[1] = (b)->L2[3 - (c)] + 1, (ik).info = 0)

typedef VEC(bwtintv_t) intv_v;

static void reverse_intvs(intv_v *p)
{
    if (p->n > 1)
        for (size_t j = 0; j < p->n >> 1; ++j) {
            bwtintv_t t = p->a[p->n - 1 - j]; p->a[p->n - 1 - j] = p->a[j]; p->a[j] = t;
        }
}

#ifdef ORC_PROFILE
/* seeding work profile (tools/seed_profile.py): bwt_extend calls by phase and by what the interval is
 * (the string fits the GPU k-mer table / the interval has one occurrence / other) */
uint64_t orc_prof[20];   /* [12..15]: backward extensions of strings of 12..15 bases; [16..19] ksw_extend2 rows, cells,
                             rows and cells after the one-column tail condition (tools/ext_profile.py) */
void orc_profile_get(uint64_t *out) { memcpy(out, orc_prof, sizeof orc_prof); }
#define PROF(k) (++orc_prof[k])
#else
#define PROF(k) ((void)0)
#endif

/* Seeding trace (tools/seed_model.py: a model of the seeding kernels' schedules): per bwt_smem1 call its forward
 * and backward trips counted the way smem.hip's kernels take them (the k-mer prefix as one trip, one trip per
 * extension past it, the unique-interval text walk as one trip per 8 bases; backward: one trip per pair of list
 * entries per position), per bwt_seed_strategy1 call its trips (one k-mer prefix trip, one per extension past it).
 * Test infrastructure; off unless orc_seed_trace is used. */
static __thread int32_t *orc_tr = NULL;
static __thread int orc_tr_n = 0, orc_tr_cap = 0, orc_tr_pass = 0, orc_tr_k = 0;
static void tr_push(int kind, int a, int b, int k)
{
    if (!orc_tr || orc_tr_n + 4 > orc_tr_cap) return;
    orc_tr[orc_tr_n++] = kind; orc_tr[orc_tr_n++] = a; orc_tr[orc_tr_n++] = b; orc_tr[orc_tr_n++] = k;
}

/* bwt_smem1a with max_intv = 0 (as called through bwt_smem1) */
static int bwt_smem1(const orc_index *b, int len, const uint8_t *q, int x, int min_intv, intv_v *mem, intv_v *tmpv)
{
    int i, j, c, ret;
    bwtintv_t ik, ok[4];
    intv_v *prev, *curr, *swap;
    const uint64_t max_intv = 0;
    mem->n = 0;
    if (q[x] > 3) return x + 1;
    if (min_intv < 1) min_intv = 1;
    prev = &tmpv[0]; curr = &tmpv[1];
    bwt_set_intv(b, q[x], ik);
    ik.info = (uint64_t)(x + 1);
    int t_pre = 0, t_ext = 0, t_walk = 0, t_bwd = 0, t_pos = 0, t_pos12 = 0, t_pos1u = 0;
    for (i = x + 1, curr->n = 0; i < len; ++i) {
        if (ik.x[2] < max_intv) { VPUSH(*curr, ik); break; }
        else if (q[i] < 4) {
            c = 3 - q[i];
            PROF(i - x + 1 <= 11 ? 0 : ik.x[2] == 1 ? 1 : 2);
            if (i - x + 1 <= 11) t_pre = 1;
            else if (ik.x[2] == 1 && min_intv <= 1) ++t_walk;
            else ++t_ext;
            bwt_extend(b, &ik, ok, 0);
            if (ok[c].x[2] != ik.x[2]) {
                VPUSH(*curr, ik);
                if (ok[c].x[2] < (uint64_t)min_intv) break;
            }
            ik = ok[c]; ik.info = (uint64_t)(i + 1);
        } else { VPUSH(*curr, ik); break; }
    }
    if (i == len) VPUSH(*curr, ik);
    reverse_intvs(curr);
    ret = (int)curr->a[0].info;
    swap = curr; curr = prev; prev = swap;
    for (i = x - 1; i >= -1; --i) {
        c = i < 0 ? -1 : q[i] < 4 ? q[i] : -1;
#ifdef ORC_PROFILE
        if (prev->n == 1 && prev->a[0].x[2] == 1) PROF(9);
#endif
        t_bwd += ((int)prev->n + 1) / 2;
        ++t_pos; t_pos12 += prev->n <= 2; t_pos1u += prev->n == 1 && prev->a[0].x[2] == 1;
        for (j = 0, curr->n = 0; j < (int)prev->n; ++j) {
            bwtintv_t *p = &prev->a[j];
            if (c >= 0 && ik.x[2] >= max_intv) {
                PROF((int)(uint32_t)p->info - i <= 11 ? 3 : p->x[2] == 1 ? 4 : 5);
#ifdef ORC_PROFILE
                { const int sl = (int)(uint32_t)p->info - i; if (sl >= 12 && sl <= 15) PROF(sl); }
#endif
                bwt_extend(b, p, ok, 1);
            }
            if (c < 0 || ik.x[2] < max_intv || ok[c].x[2] < (uint64_t)min_intv) {
                if (curr->n == 0) {
                    if (mem->n == 0 || (uint64_t)(i + 1) < mem->a[mem->n - 1].info >> 32) {
                        ik = *p; ik.info |= (uint64_t)(i + 1) << 32;
                        VPUSH(*mem, ik);
                    }
                }
            } else if (curr->n == 0 || ok[c].x[2] != curr->a[curr->n - 1].x[2]) {
                ok[c].info = p->info;
                VPUSH(*curr, ok[c]);
            }
        }
        if (curr->n == 0) break;
        swap = curr; curr = prev; prev = swap;
    }
    reverse_intvs(mem);
    tr_push(orc_tr_pass, t_pre + t_ext + (t_walk ? t_walk / 8 + 1 : 0), t_bwd, orc_tr_k);
    tr_push(4, t_pos, t_pos12, t_pos1u);
    return ret;
}

static int bwt_seed_strategy1(const orc_index *b, int len, const uint8_t *q, int x, int min_len, int max_intv, bwtintv_t *mem)
{
    int i, c; bwtintv_t ik, ok[4];
    memset(mem, 0, sizeof(bwtintv_t));
    if (q[x] > 3) return x + 1;
    bwt_set_intv(b, q[x], ik);
    int t_pre = 0, t_ext = 0, t_uni = 0;
    for (i = x + 1; i < len; ++i) {
        if (q[i] < 4) {
            c = 3 - q[i];
            PROF(i - x + 1 <= 11 ? 6 : ik.x[2] == 1 ? 7 : 8);
            if (i - x + 1 <= 11) t_pre = 1;
            else if (ik.x[2] == 1) ++t_uni;
            else ++t_ext;
            bwt_extend(b, &ik, ok, 0);
            if (ok[c].x[2] < (uint64_t)max_intv && i - x >= min_len) {
                *mem = ok[c];
                mem->info = (uint64_t)x << 32 | (uint64_t)(i + 1);
                tr_push(3, t_pre + t_ext, t_uni, orc_tr_k);
                return i + 1;
            }
            ik = ok[c];
        } else { tr_push(3, t_pre + t_ext, t_uni, orc_tr_k); return i + 1; }
    }
    tr_push(3, t_pre + t_ext, t_uni, orc_tr_k);
    return len;
}

/* ============================================================================================== */
/* mem_opt_t (mem_opt_init + the bioseqdb overrides; Q2: mat is NOT refilled after a/b override)  */
/* ============================================================================================== */
typedef struct {
    int a, b, o_del, e_del, o_ins, e_ins, pen_clip5, pen_clip3, w, zdrop;
    int min_seed_len, max_occ, split_width, max_chain_gap, min_chain_weight, max_chain_extend, max_mem_intv;
    float split_factor, mask_level, drop_ratio, mask_level_redun;
    int8_t mat[25];
} mopt_t;

static void fill_scmat(int a, int b, int8_t mat[25])
{
    int i, j, k;
    for (i = k = 0; i < 4; ++i) {
        for (j = 0; j < 4; ++j) mat[k++] = (int8_t)(i == j ? a : -b);
        mat[k++] = -1;
    }
    for (j = 0; j < 5; ++j) mat[k++] = -1;
}

static void make_opt(const orc_opts *o, mopt_t *m)
{
    memset(m, 0, sizeof *m);
    m->split_width = 10; m->max_chain_gap = 10000; m->min_chain_weight = 0; m->max_chain_extend = 1 << 30;
    m->max_mem_intv = 20; m->split_factor = 1.5f; m->mask_level = 0.50f; m->drop_ratio = 0.50f;
    m->mask_level_redun = 0.95f;
    fill_scmat(1, 4, m->mat);                       /* mem_opt_init: a=1, b=4 */
    m->max_occ = o->max_occ; m->min_seed_len = o->min_seed_len; m->a = o->a; m->b = o->b;
    m->pen_clip3 = o->pen_clip3; m->pen_clip5 = o->pen_clip5; m->zdrop = o->zdrop; m->w = o->w;
    m->o_del = o->o_del; m->o_ins = o->o_ins; m->e_del = o->e_del; m->e_ins = o->e_ins;
}

/* ============================================================================================== */
/* bntseq helpers                                                                                  */
/* ============================================================================================== */
static inline int64_t bns_depos(const orc_index *x, int64_t pos, int *is_rev)
{
    return (*is_rev = (pos >= x->l_pac)) ? (x->l_pac << 1) - 1 - pos : pos;
}

static int bns_pos2rid(const orc_index *x, int64_t pos_f)
{
    int left, mid, right, n = (int)x->anns.n;
    if (pos_f >= x->l_pac) return -1;
    left = 0; mid = 0; right = n;
    while (left < right) {
        mid = (left + right) >> 1;
        if (pos_f >= x->anns.a[mid].offset) {
            if (mid == n - 1) break;
            if (pos_f < x->anns.a[mid + 1].offset) break;
            left = mid + 1;
        } else right = mid;
    }
    return mid;
}

static int bns_intv2rid(const orc_index *x, int64_t rb, int64_t re)
{
    int is_rev, rid_b, rid_e;
    if (rb < x->l_pac && re > x->l_pac) return -2;
    rid_b = bns_pos2rid(x, bns_depos(x, rb, &is_rev));
    rid_e = rb < re ? bns_pos2rid(x, bns_depos(x, re - 1, &is_rev)) : rid_b;
    return rid_b == rid_e ? rid_b : -1;
}

static uint8_t *bns_get_seq(int64_t l_pac, const uint8_t *pac, int64_t beg, int64_t end, int64_t *len)
{
    uint8_t *seq = 0;
    if (end < beg) { int64_t t = end; end = beg; beg = t; }
    if (end > l_pac << 1) end = l_pac << 1;
    if (beg < 0) beg = 0;
    if (beg >= l_pac || end <= l_pac) {
        int64_t k, l = 0;
        *len = end - beg;
        orc_ab[3] += (uint64_t)((end - beg + 3) >> 2);
        seq = malloc(end - beg > 0 ? (size_t)(end - beg) : 1);
        if (beg >= l_pac) {
            int64_t beg_f = (l_pac << 1) - 1 - end, end_f = (l_pac << 1) - 1 - beg;
            for (k = end_f; k > beg_f; --k) seq[l++] = (uint8_t)(3 - pac_raw_get(pac, (uint64_t)k));
        } else {
            for (k = beg; k < end; ++k) seq[l++] = (uint8_t)pac_raw_get(pac, (uint64_t)k);
        }
    } else *len = 0;
    return seq;
}

static uint8_t *bns_fetch_seq(const orc_index *x, int64_t *beg, int64_t mid, int64_t *end, int *rid)
{
    int64_t far_beg, far_end, len; int is_rev;
    if (*end < *beg) { int64_t t = *end; *end = *beg; *beg = t; }
    *rid = bns_pos2rid(x, bns_depos(x, mid, &is_rev));
    far_beg = x->anns.a[*rid].offset;
    far_end = far_beg + x->anns.a[*rid].len;
    if (is_rev) { int64_t t = far_beg; far_beg = (x->l_pac << 1) - far_end; far_end = (x->l_pac << 1) - t; }
    *beg = *beg > far_beg ? *beg : far_beg;
    *end = *end < far_end ? *end : far_end;
    const uint64_t before = orc_ab[3];
    uint8_t *seq = bns_get_seq(x->l_pac, x->pac.a, *beg, *end, &len);
    orc_ab[2] += orc_ab[3] - before;   /* an extension window, not a CIGAR one */
    orc_ab[3] = before;
    return seq;
}

/* ============================================================================================== */
/* ksw.c: ksw_extend2 and ksw_global2                                                              */
/* ============================================================================================== */
typedef struct { int32_t h, e; } eh_t;

static int ksw_extend2(int qlen, const uint8_t *query, int tlen, const uint8_t *target, int m, const int8_t *mat,
                       int o_del, int e_del, int o_ins, int e_ins, int w, int end_bonus, int zdrop, int h0,
                       int *_qle, int *_tle, int *_gtle, int *_gscore, int *_max_off)
{
    eh_t *eh; int8_t *qp;
    int i, j, k, oe_del = o_del + e_del, oe_ins = o_ins + e_ins, beg, end, max, max_i, max_j, max_ins, max_del,
        max_ie, gscore, max_off;
    if (qlen < 0) qlen = 0;
    qp = malloc((size_t)qlen * m + 1);
    eh = calloc((size_t)qlen + 1, 8);
    for (k = i = 0; k < m; ++k) {
        const int8_t *p = &mat[k * m];
        for (j = 0; j < qlen; ++j) qp[i++] = p[query[j]];
    }
    eh[0].h = h0; if (qlen >= 1) eh[1].h = h0 > oe_ins ? h0 - oe_ins : 0;
    for (j = 2; j <= qlen && eh[j - 1].h > e_ins; ++j) eh[j].h = eh[j - 1].h - e_ins;
    k = m * m;
    for (i = 0, max = 0; i < k; ++i) max = max > mat[i] ? max : mat[i];
    max_ins = (int)((double)(qlen * max + end_bonus - o_ins) / e_ins + 1.);
    max_ins = max_ins > 1 ? max_ins : 1;
    w = w < max_ins ? w : max_ins;
    max_del = (int)((double)(qlen * max + end_bonus - o_del) / e_del + 1.);
    max_del = max_del > 1 ? max_del : 1;
    w = w < max_del ? w : max_del;
    max = h0, max_i = max_j = -1; max_ie = -1, gscore = -1;
    max_off = 0;
    beg = 0, end = qlen;
#ifdef ORC_PROFILE
    int tail = 0, row_reached_qlen = 0;
#endif
#ifdef ORC_PROFILE
    tr_push(10, qlen, tlen, w);
#endif
    for (i = 0; i < tlen; ++i) {
        int t, f = 0, h1, mm = 0, mj = -1;
        int8_t *q = &qp[target[i] * qlen];
        if (beg < i - w) beg = i - w;
        if (end > i + w + 1) end = i + w + 1;
        if (end > qlen) end = qlen;
        if (beg == 0) {
            h1 = h0 - (o_del + e_del * (i + 1));
            if (h1 < 0) h1 = 0;
        } else h1 = 0;
        for (j = beg; j < end; ++j) {
            eh_t *p = &eh[j];
            int h, M = p->h, e = p->e;
            p->h = h1;
            M = M ? M + q[j] : 0;
            h = M > e ? M : e;
            h = h > f ? h : f;
            h1 = h;
            mj = mm > h ? mj : j;
            mm = mm > h ? mm : h;
            t = M - oe_del; t = t > 0 ? t : 0;
            e -= e_del; e = e > t ? e : t;
            p->e = e;
            t = M - oe_ins; t = t > 0 ? t : 0;
            f -= e_ins; f = f > t ? f : t;
        }
        eh[end].h = h1; eh[end].e = 0;
#ifdef ORC_PROFILE
        row_reached_qlen = j == qlen;
        PROF(16); orc_prof[17] += (uint64_t)(end > beg ? end - beg : 0);
        tr_push(11, end > beg ? end - beg : 0, beg, end);
        if (tail) { PROF(18); orc_prof[19] += (uint64_t)(end > beg ? end - beg : 0); }
#endif
        if (j == qlen) {
            max_ie = gscore > h1 ? max_ie : i;
            gscore = gscore > h1 ? gscore : h1;
        }
        if (mm == 0) break;
        if (mm > max) {
            max = mm, max_i = i, max_j = mj;
            max_off = max_off > abs(mj - i) ? max_off : abs(mj - i);
        } else if (zdrop > 0) {
            if (i - max_i > mj - max_j) {
                if (max - mm - ((i - max_i) - (mj - max_j)) * e_del > zdrop) break;
            } else {
                if (max - mm - ((mj - max_j) - (i - max_i)) * e_ins > zdrop) break;
            }
        }
        for (j = beg; j < end && eh[j].h == 0 && eh[j].e == 0; ++j);
        beg = j;
        for (j = end; j >= beg && eh[j].h == 0 && eh[j].e == 0; --j);
        end = j + 2 < qlen ? j + 2 : qlen;
#ifdef ORC_PROFILE
        if (!tail && qlen >= 2 && beg == qlen - 1 && end == qlen && eh[qlen - 1].h == 0 && row_reached_qlen) tail = 1;
#endif
    }
    free(eh); free(qp);
    if (_qle) *_qle = max_j + 1;
    if (_tle) *_tle = max_i + 1;
    if (_gtle) *_gtle = max_ie + 1;
    if (_gscore) *_gscore = gscore;
    if (_max_off) *_max_off = max_off;
    return max;
}

#define MINUS_INF -0x40000000

static uint32_t *push_cigar(int *n_cigar, int *m_cigar, uint32_t *cigar, int op, int len)
{
    if (*n_cigar == 0 || op != (int)(cigar[(*n_cigar) - 1] & 0xf)) {
        if (*n_cigar == *m_cigar) {
            *m_cigar = *m_cigar ? (*m_cigar) << 1 : 4;
            cigar = realloc(cigar, (size_t)(*m_cigar) << 2);
        }
        cigar[(*n_cigar)++] = (uint32_t)len << 4 | (uint32_t)op;
    } else cigar[(*n_cigar) - 1] += (uint32_t)len << 4;
    return cigar;
}

static int ksw_global2(int qlen, const uint8_t *query, int tlen, const uint8_t *target, int m, const int8_t *mat,
                       int o_del, int e_del, int o_ins, int e_ins, int w, int *n_cigar_, uint32_t **cigar_)
{
    eh_t *eh; int8_t *qp;
    int i, j, k, oe_del = o_del + e_del, oe_ins = o_ins + e_ins, score, n_col;
    uint8_t *z;
    if (n_cigar_) *n_cigar_ = 0;
    n_col = qlen < 2 * w + 1 ? qlen : 2 * w + 1;
    z = n_cigar_ && cigar_ ? calloc((size_t)n_col * tlen + 1, 1) : 0;
    qp = malloc((size_t)qlen * m + 1);
    eh = calloc((size_t)qlen + 1, 8);
    for (k = i = 0; k < m; ++k) {
        const int8_t *p = &mat[k * m];
        for (j = 0; j < qlen; ++j) qp[i++] = p[query[j]];
    }
    eh[0].h = 0; eh[0].e = MINUS_INF;
    for (j = 1; j <= qlen && j <= w; ++j) eh[j].h = -(o_ins + e_ins * j), eh[j].e = MINUS_INF;
    for (; j <= qlen; ++j) eh[j].h = eh[j].e = MINUS_INF;
    for (i = 0; i < tlen; ++i) {
        int32_t f = MINUS_INF, h1, beg, end, t;
        int8_t *q = &qp[target[i] * qlen];
        beg = i > w ? i - w : 0;
        end = i + w + 1 < qlen ? i + w + 1 : qlen;
        h1 = beg == 0 ? -(o_del + e_del * (i + 1)) : MINUS_INF;
        uint8_t *zi = z ? &z[(long)i * n_col] : 0;
        for (j = beg; j < end; ++j) {
            eh_t *p = &eh[j];
            int32_t h, mm = p->h, e = p->e;
            uint8_t d;
            p->h = h1;
            mm += q[j];
            d = mm >= e ? 0 : 1;
            h = mm >= e ? mm : e;
            d = h >= f ? d : 2;
            h = h >= f ? h : f;
            h1 = h;
            t = mm - oe_del;
            e -= e_del;
            d |= e > t ? 1 << 2 : 0;
            e = e > t ? e : t;
            p->e = e;
            t = mm - oe_ins;
            f -= e_ins;
            d |= f > t ? 2 << 4 : 0;
            f = f > t ? f : t;
            if (zi) zi[j - beg] = d;
        }
        eh[end].h = h1; eh[end].e = MINUS_INF;
    }
    score = eh[qlen].h;
    if (n_cigar_ && cigar_) {
        int n_cigar = 0, m_cigar = 0, which = 0;
        uint32_t *cigar = 0, tmp;
        i = tlen - 1; k = (i + w + 1 < qlen ? i + w + 1 : qlen) - 1;
        while (i >= 0 && k >= 0) {
            which = z[(long)i * n_col + (k - (i > w ? i - w : 0))] >> (which << 1) & 3;
            if (which == 0) cigar = push_cigar(&n_cigar, &m_cigar, cigar, 0, 1), --i, --k;
            else if (which == 1) cigar = push_cigar(&n_cigar, &m_cigar, cigar, 2, 1), --i;
            else cigar = push_cigar(&n_cigar, &m_cigar, cigar, 1, 1), --k;
        }
        if (i >= 0) cigar = push_cigar(&n_cigar, &m_cigar, cigar, 2, i + 1);
        if (k >= 0) cigar = push_cigar(&n_cigar, &m_cigar, cigar, 1, k + 1);
        for (i = 0; i < n_cigar >> 1; ++i)
            tmp = cigar[i], cigar[i] = cigar[n_cigar - 1 - i], cigar[n_cigar - 1 - i] = tmp;
        *n_cigar_ = n_cigar, *cigar_ = cigar;
    }
    free(eh); free(qp); free(z);
    return score;
}

int orc_ksw_extend2(int qlen, const uint8_t *query, int tlen, const uint8_t *target, const int8_t *mat,
                    int o_del, int e_del, int o_ins, int e_ins, int w, int end_bonus, int zdrop, int h0,
                    int *qle, int *tle, int *gtle, int *gscore, int *max_off)
{
    return ksw_extend2(qlen, query, tlen, target, 5, mat, o_del, e_del, o_ins, e_ins, w, end_bonus, zdrop, h0,
                       qle, tle, gtle, gscore, max_off);
}

int orc_ksw_global2(int qlen, const uint8_t *query, int tlen, const uint8_t *target, const int8_t *mat,
                    int o_del, int e_del, int o_ins, int e_ins, int w, int *n_cigar, uint32_t *cigar, int max_cigar)
{
    uint32_t *c = 0; int n = 0;
    int sc = ksw_global2(qlen, query, tlen, target, 5, mat, o_del, e_del, o_ins, e_ins, w, &n, &c);
    for (int i = 0; i < n && i < max_cigar; ++i) cigar[i] = c[i];
    *n_cigar = n;
    free(c);
    return sc;
}

/* bwa.c bwa_gen_cigar2 (MD/NM are not part of bioseqdb's output and are not computed) */
static uint32_t *bwa_gen_cigar2(const int8_t mat[25], int o_del, int e_del, int o_ins, int e_ins, int w_, int64_t l_pac,
                                const uint8_t *pac, int l_query, const uint8_t *query_in, int64_t rb, int64_t re,
                                int *score, int *n_cigar)
{
    uint32_t *cigar = 0; uint8_t *rseq, *query; int i; int64_t rlen;
    if (n_cigar) *n_cigar = 0;
    if (l_query <= 0 || rb >= re || (rb < l_pac && re > l_pac)) return 0;
    rseq = bns_get_seq(l_pac, pac, rb, re, &rlen);
    if (re - rb != rlen) { free(rseq); return 0; }
    query = malloc((size_t)l_query);
    memcpy(query, query_in, (size_t)l_query);
    if (rb >= l_pac) {   /* reverse both (bwa reverses the caller's buffer and restores it afterwards) */
        uint8_t t;
        for (i = 0; i < l_query >> 1; ++i) t = query[i], query[i] = query[l_query - 1 - i], query[l_query - 1 - i] = t;
        for (i = 0; i < rlen >> 1; ++i) t = rseq[i], rseq[i] = rseq[rlen - 1 - i], rseq[rlen - 1 - i] = t;
    }
    if (l_query == re - rb && w_ == 0) {
        cigar = malloc(4);
        cigar[0] = (uint32_t)l_query << 4 | 0;
        if (n_cigar) *n_cigar = 1;
        for (i = 0, *score = 0; i < l_query; ++i) *score += mat[rseq[i] * 5 + query[i]];
    } else {
        int w, max_gap, max_ins, max_del, min_w;
        max_ins = (int)((double)(((l_query + 1) >> 1) * mat[0] - o_ins) / e_ins + 1.);
        max_del = (int)((double)(((l_query + 1) >> 1) * mat[0] - o_del) / e_del + 1.);
        max_gap = max_ins > max_del ? max_ins : max_del;
        max_gap = max_gap > 1 ? max_gap : 1;
        w = (max_gap + abs((int)rlen - l_query) + 1) >> 1;
        w = w < w_ ? w : w_;
        min_w = abs((int)rlen - l_query) + 3;
        w = w > min_w ? w : min_w;
        *score = ksw_global2(l_query, query, (int)rlen, rseq, 5, mat, o_del, e_del, o_ins, e_ins, w,
                             n_cigar, n_cigar ? &cigar : 0);
    }
    free(query); free(rseq);
    return cigar;
}

/* ============================================================================================== */
/* bwamem.c                                                                                        */
/* ============================================================================================== */
static int intv_lt(const void *a, const void *b) { return ((const bwtintv_t *)a)->info < ((const bwtintv_t *)b)->info; }

static void mem_collect_intv(const mopt_t *opt, const orc_index *bwt, int len, const uint8_t *seq, intv_v *mem,
                             intv_v *mem1, intv_v tmpv[2])
{
    int i, k, x = 0, old_n;
    int start_width = 1;
    int split_len = (int)(opt->min_seed_len * opt->split_factor + .499);
    mem->n = 0;
    orc_tr_pass = 1; orc_tr_k = 0;
    while (x < len) {
        if (seq[x] < 4) {
            x = bwt_smem1(bwt, len, seq, x, start_width, mem1, tmpv);
            ++orc_tr_k;
            for (i = 0; i < (int)mem1->n; ++i) {
                bwtintv_t *p = &mem1->a[i];
                int slen = (int)((uint32_t)p->info - (p->info >> 32));
                if (slen >= opt->min_seed_len) VPUSH(*mem, *p);
            }
        } else ++x;
    }
    old_n = (int)mem->n;
    orc_tr_pass = 2;
    for (k = 0; k < old_n; ++k) {
        bwtintv_t p = mem->a[k];
        int start = (int)(p.info >> 32), end = (int32_t)p.info;
        if (end - start < split_len || p.x[2] > (uint64_t)opt->split_width) continue;
        orc_tr_k = k;
        bwt_smem1(bwt, len, seq, (start + end) >> 1, (int)p.x[2] + 1, mem1, tmpv);
        for (i = 0; i < (int)mem1->n; ++i)
            if ((uint32_t)mem1->a[i].info - (mem1->a[i].info >> 32) >= (uint64_t)opt->min_seed_len)
                VPUSH(*mem, mem1->a[i]);
    }
    if (opt->max_mem_intv > 0) {
        x = 0;
        orc_tr_k = 0;
        while (x < len) {
            if (seq[x] < 4) {
                bwtintv_t m;
                x = bwt_seed_strategy1(bwt, len, seq, x, opt->min_seed_len, opt->max_mem_intv, &m);
                ++orc_tr_k;
                if (m.x[2] > 0) VPUSH(*mem, m);
            } else ++x;
        }
    }
    ks_introsort(mem->n, mem->a, sizeof(bwtintv_t), intv_lt);
}

typedef struct { int64_t rbeg; int32_t qbeg, len; int score; } mem_seed_t;
typedef struct {
    int n, m, first, rid;
    uint32_t w, kept, is_alt;
    float frac_rep;
    int64_t pos;
    mem_seed_t *seeds;
} mem_chain_t;
typedef VEC(mem_chain_t) chain_v;

/* ---- kbtree.h restatement: KBTREE_INIT(chn, mem_chain_t, chain_cmp), KB_DEFAULT_SIZE = 512 ----- */
/* t = ((512 - 4 - sizeof(void*)) / (sizeof(void*) + sizeof(mem_chain_t) = 40) + 1) >> 1 = 5 on LP64 */
#define KB_T 5
#define KB_N (2 * KB_T - 1)
typedef struct kbnode { int is_internal, n; mem_chain_t key[KB_N]; struct kbnode *ptr[KB_N + 1]; } kbnode_t;
typedef struct { kbnode_t *root; int n_keys; } kbtree_t;

static inline int chain_cmp(const mem_chain_t *a, const mem_chain_t *b) { return (b->pos < a->pos) - (a->pos < b->pos); }

static int kb_getp_aux(const kbnode_t *x, const mem_chain_t *k, int *r)
{
    int tr, *rr, begin = 0, end = x->n;
    if (x->n == 0) return -1;
    rr = r ? r : &tr;
    while (begin < end) {
        int mid = (begin + end) >> 1;
        if (chain_cmp(&x->key[mid], k) < 0) begin = mid + 1;
        else end = mid;
    }
    if (begin == x->n) { *rr = 1; return x->n - 1; }
    if ((*rr = chain_cmp(k, &x->key[begin])) < 0) --begin;
    return begin;
}

static void kb_intervalp(kbtree_t *b, const mem_chain_t *k, mem_chain_t **lower, mem_chain_t **upper)
{
    int i, r = 0;
    kbnode_t *x = b->root;
    *lower = *upper = 0;
    while (x) {
        i = kb_getp_aux(x, k, &r);
        if (i >= 0 && r == 0) { *lower = *upper = &x->key[i]; return; }
        if (i >= 0) *lower = &x->key[i];
        if (i < x->n - 1) *upper = &x->key[i + 1];
        if (x->is_internal == 0) return;
        x = x->ptr[i + 1];
    }
}

static void kb_split(kbnode_t *x, int i, kbnode_t *y)
{
    kbnode_t *z = calloc(1, sizeof(kbnode_t));
    z->is_internal = y->is_internal;
    z->n = KB_T - 1;
    memcpy(z->key, y->key + KB_T, sizeof(mem_chain_t) * (KB_T - 1));
    if (y->is_internal) memcpy(z->ptr, y->ptr + KB_T, sizeof(void *) * KB_T);
    y->n = KB_T - 1;
    memmove(x->ptr + i + 2, x->ptr + i + 1, sizeof(void *) * (x->n - i));
    x->ptr[i + 1] = z;
    memmove(x->key + i + 1, x->key + i, sizeof(mem_chain_t) * (x->n - i));
    x->key[i] = y->key[KB_T - 1];
    ++x->n;
}

static void kb_putp_aux(kbnode_t *x, const mem_chain_t *k)
{
    int i = x->n - 1;
    if (x->is_internal == 0) {
        i = kb_getp_aux(x, k, 0);
        if (i != x->n - 1) memmove(x->key + i + 2, x->key + i + 1, (size_t)(x->n - i - 1) * sizeof(mem_chain_t));
        x->key[i + 1] = *k;
        ++x->n;
    } else {
        i = kb_getp_aux(x, k, 0) + 1;
        if (x->ptr[i]->n == 2 * KB_T - 1) {
            kb_split(x, i, x->ptr[i]);
            if (chain_cmp(k, &x->key[i]) > 0) ++i;
        }
        kb_putp_aux(x->ptr[i], k);
    }
}

static void kb_putp(kbtree_t *b, const mem_chain_t *k)
{
    kbnode_t *r = b->root;
    ++b->n_keys;
    if (r->n == 2 * KB_T - 1) {
        kbnode_t *s = calloc(1, sizeof(kbnode_t));
        b->root = s; s->is_internal = 1; s->n = 0;
        s->ptr[0] = r;
        kb_split(s, 0, r);
        r = s;
    }
    kb_putp_aux(r, k);
}

static void kb_traverse(const kbnode_t *x, chain_v *out)
{
    for (int i = 0; i <= x->n; ++i) {
        if (x->is_internal) kb_traverse(x->ptr[i], out);
        if (i < x->n) VPUSH(*out, x->key[i]);
    }
}

static void kb_destroy(kbnode_t *x)
{
    if (!x) return;
    if (x->is_internal) for (int i = 0; i <= x->n; ++i) kb_destroy(x->ptr[i]);
    free(x);
}

static int test_and_merge(const mopt_t *opt, int64_t l_pac, mem_chain_t *c, const mem_seed_t *p, int seed_rid)
{
    int64_t qend, rend, x, y;
    const mem_seed_t *last = &c->seeds[c->n - 1];
    qend = last->qbeg + last->len;
    rend = last->rbeg + last->len;
    if (seed_rid != c->rid) return 0;
    if (p->qbeg >= c->seeds[0].qbeg && p->qbeg + p->len <= qend && p->rbeg >= c->seeds[0].rbeg && p->rbeg + p->len <= rend)
        return 1;
    if ((last->rbeg < l_pac || c->seeds[0].rbeg < l_pac) && p->rbeg >= l_pac) return 0;
    x = p->qbeg - last->qbeg;
    y = p->rbeg - last->rbeg;
    if (y >= 0 && x - y <= opt->w && y - x <= opt->w && x - last->len < opt->max_chain_gap && y - last->len < opt->max_chain_gap) {
        if (c->n == c->m) { c->m <<= 1; c->seeds = realloc(c->seeds, (size_t)c->m * sizeof(mem_seed_t)); }
        c->seeds[c->n++] = *p;
        return 1;
    }
    return 0;
}

static int mem_chain_weight(const mem_chain_t *c)
{
    int64_t end; int j, w = 0, tmp;
    for (j = 0, end = 0; j < c->n; ++j) {
        const mem_seed_t *s = &c->seeds[j];
        if (s->qbeg >= end) w += s->len;
        else if (s->qbeg + s->len > end) w += (int)(s->qbeg + s->len - end);
        end = end > s->qbeg + s->len ? end : s->qbeg + s->len;
    }
    tmp = w; w = 0;
    for (j = 0, end = 0; j < c->n; ++j) {
        const mem_seed_t *s = &c->seeds[j];
        if (s->rbeg >= end) w += s->len;
        else if (s->rbeg + s->len > end) w += (int)(s->rbeg + s->len - end);
        end = end > s->rbeg + s->len ? end : s->rbeg + s->len;
    }
    w = w < tmp ? w : tmp;
    return w < 1 << 30 ? w : (1 << 30) - 1;
}

static void mem_chain(const mopt_t *opt, const orc_index *bwt, int len, const uint8_t *seq, chain_v *chain)
{
    int i, b, e, l_rep;
    int64_t l_pac = bwt->l_pac;
    intv_v mem = {0, 0, 0}, mem1 = {0, 0, 0}, tmpv[2] = {{0, 0, 0}, {0, 0, 0}};
    chain->n = 0;
    if (len < opt->min_seed_len) return;
    kbtree_t tree = { calloc(1, sizeof(kbnode_t)), 0 };
    mem_collect_intv(opt, bwt, len, seq, &mem, &mem1, tmpv);
    for (i = 0, b = e = l_rep = 0; i < (int)mem.n; ++i) {
        bwtintv_t *p = &mem.a[i];
        int sb = (int)(p->info >> 32), se = (int)(uint32_t)p->info;
        if (p->x[2] <= (uint64_t)opt->max_occ) continue;
        if (sb > e) l_rep += e - b, b = sb, e = se;
        else e = e > se ? e : se;
    }
    l_rep += e - b;
    for (i = 0; i < (int)mem.n; ++i) {
        bwtintv_t *p = &mem.a[i];
        int step, count, slen = (int)((uint32_t)p->info - (p->info >> 32));
        int64_t k;
        step = p->x[2] > (uint64_t)opt->max_occ ? (int)(p->x[2] / (uint64_t)opt->max_occ) : 1;
        for (k = count = 0; (uint64_t)k < p->x[2] && count < opt->max_occ; k += step, ++count) {
            mem_chain_t tmp, *lower, *upper;
            mem_seed_t s;
            int rid, to_add = 0;
            s.rbeg = tmp.pos = (int64_t)bwt_sa(bwt, p->x[0] + (uint64_t)k);
            s.qbeg = (int32_t)(p->info >> 32);
            s.score = s.len = slen;
            rid = bns_intv2rid(bwt, s.rbeg, s.rbeg + s.len);
            if (rid < 0) continue;
            if (tree.n_keys) {
                kb_intervalp(&tree, &tmp, &lower, &upper);
                if (!lower || !test_and_merge(opt, l_pac, lower, &s, rid)) to_add = 1;
            } else to_add = 1;
            if (to_add) {
                tmp.n = 1; tmp.m = 4;
                tmp.seeds = calloc((size_t)tmp.m, sizeof(mem_seed_t));
                tmp.seeds[0] = s;
                tmp.rid = rid;
                tmp.is_alt = 0;
                tmp.first = 0; tmp.w = 0; tmp.kept = 0; tmp.frac_rep = 0;
                kb_putp(&tree, &tmp);
            }
        }
    }
    kb_traverse(tree.root, chain);
    for (i = 0; i < (int)chain->n; ++i) chain->a[i].frac_rep = (float)l_rep / len;
    kb_destroy(tree.root);
    free(mem.a); free(mem1.a); free(tmpv[0].a); free(tmpv[1].a);
}

static int flt_lt(const void *a, const void *b) { return ((const mem_chain_t *)a)->w > ((const mem_chain_t *)b)->w; }

#define chn_beg(ch) ((ch).seeds->qbeg)
#define chn_end(ch) ((ch).seeds[(ch).n - 1].qbeg + (ch).seeds[(ch).n - 1].len)

static int mem_chain_flt(const mopt_t *opt, int n_chn, mem_chain_t *a)
{
    int i, k;
    VEC(int) chains = {0, 0, 0};
    if (n_chn == 0) return 0;
    for (i = k = 0; i < n_chn; ++i) {
        mem_chain_t *c = &a[i];
        c->first = -1; c->kept = 0;
        c->w = (uint32_t)mem_chain_weight(c);
        if ((int)c->w < opt->min_chain_weight) free(c->seeds);
        else a[k++] = *c;
    }
    n_chn = k;
    ks_introsort((size_t)n_chn, a, sizeof(mem_chain_t), flt_lt);
    a[0].kept = 3;
    VPUSH(chains, 0);
    for (i = 1; i < n_chn; ++i) {
        int large_ovlp = 0;
        for (k = 0; k < (int)chains.n; ++k) {
            int j = chains.a[k];
            int b_max = chn_beg(a[j]) > chn_beg(a[i]) ? chn_beg(a[j]) : chn_beg(a[i]);
            int e_min = chn_end(a[j]) < chn_end(a[i]) ? chn_end(a[j]) : chn_end(a[i]);
            if (e_min > b_max && (!a[j].is_alt || a[i].is_alt)) {
                int li = chn_end(a[i]) - chn_beg(a[i]);
                int lj = chn_end(a[j]) - chn_beg(a[j]);
                int min_l = li < lj ? li : lj;
                if (e_min - b_max >= min_l * opt->mask_level && min_l < opt->max_chain_gap) {
                    large_ovlp = 1;
                    if (a[j].first < 0) a[j].first = i;
                    if ((int)a[i].w < (int)a[j].w * opt->drop_ratio && (int)a[j].w - (int)a[i].w >= opt->min_seed_len << 1)
                        break;
                }
            }
        }
        if (k == (int)chains.n) {
            VPUSH(chains, i);
            a[i].kept = large_ovlp ? 2 : 3;
        }
    }
    for (i = 0; i < (int)chains.n; ++i) {
        mem_chain_t *c = &a[chains.a[i]];
        if (c->first >= 0) a[c->first].kept = 1;
    }
    free(chains.a);
    for (i = k = 0; i < n_chn; ++i) {
        if (a[i].kept == 0 || a[i].kept == 3) continue;
        if (++k >= opt->max_chain_extend) break;
    }
    for (; i < n_chn; ++i)
        if (a[i].kept < 3) a[i].kept = 0;
    for (i = k = 0; i < n_chn; ++i) {
        mem_chain_t *c = &a[i];
        if (c->kept == 0) free(c->seeds);
        else a[k++] = a[i];
    }
    return k;
}

typedef struct {
    int64_t rb, re;
    int qb, qe, rid, score, truesc, sub, alt_sc, csub, sub_n, w, seedcov, secondary, secondary_all, seedlen0;
    int n_comp, is_alt;
    float frac_rep;
    uint64_t hash;
} mem_alnreg_t;
typedef VEC(mem_alnreg_t) alnreg_v;

static inline int cal_max_gap(const mopt_t *opt, int qlen)
{
    int l_del = (int)((double)(qlen * opt->a - opt->o_del) / opt->e_del + 1.);
    int l_ins = (int)((double)(qlen * opt->a - opt->o_ins) / opt->e_ins + 1.);
    int l = l_del > l_ins ? l_del : l_ins;
    l = l > 1 ? l : 1;
    return l < opt->w << 1 ? l : opt->w << 1;
}

static int u64_lt(const void *a, const void *b) { return *(const uint64_t *)a < *(const uint64_t *)b; }

#define MAX_BAND_TRY 2

static void mem_chain2aln(const mopt_t *opt, const orc_index *bns, int l_query, const uint8_t *query,
                          const mem_chain_t *c, alnreg_v *av)
{
    int i, k, rid, max_off[2], aw[2];
    int64_t l_pac = bns->l_pac, rmax[2], tmp, max = 0;
    const mem_seed_t *s;
    uint8_t *rseq = 0;
    uint64_t *srt;
    if (c->n == 0) return;
    rmax[0] = l_pac << 1; rmax[1] = 0;
    for (i = 0; i < c->n; ++i) {
        int64_t b, e;
        const mem_seed_t *t = &c->seeds[i];
        b = t->rbeg - (t->qbeg + cal_max_gap(opt, t->qbeg));
        e = t->rbeg + t->len + ((l_query - t->qbeg - t->len) + cal_max_gap(opt, l_query - t->qbeg - t->len));
        rmax[0] = rmax[0] < b ? rmax[0] : b;
        rmax[1] = rmax[1] > e ? rmax[1] : e;
        if (t->len > max) max = t->len;
    }
    rmax[0] = rmax[0] > 0 ? rmax[0] : 0;
    rmax[1] = rmax[1] < l_pac << 1 ? rmax[1] : l_pac << 1;
    if (rmax[0] < l_pac && l_pac < rmax[1]) {
        if (c->seeds[0].rbeg < l_pac) rmax[1] = l_pac;
        else rmax[0] = l_pac;
    }
    rseq = bns_fetch_seq(bns, &rmax[0], c->seeds[0].rbeg, &rmax[1], &rid);
    srt = malloc((size_t)c->n * 8);
#ifdef ORC_PROFILE
    tr_push(20, c->n, (int)max, 0);
#endif
    for (i = 0; i < c->n; ++i) srt[i] = (uint64_t)c->seeds[i].score << 32 | (uint64_t)i;
    ks_introsort((size_t)c->n, srt, 8, u64_lt);
    for (k = c->n - 1; k >= 0; --k) {
        mem_alnreg_t *a;
        s = &c->seeds[(uint32_t)srt[k]];
        for (i = 0; i < (int)av->n; ++i) {
            mem_alnreg_t *p = &av->a[i];
            int64_t rd; int qd, w, max_gap;
            if (s->rbeg < p->rb || s->rbeg + s->len > p->re || s->qbeg < p->qb || s->qbeg + s->len > p->qe) continue;
            if (s->len - p->seedlen0 > .1 * l_query) continue;
            qd = s->qbeg - p->qb; rd = s->rbeg - p->rb;
            max_gap = cal_max_gap(opt, qd < rd ? qd : (int)rd);
            w = max_gap < p->w ? max_gap : p->w;
            if (qd - rd < w && rd - qd < w) break;
            qd = p->qe - (s->qbeg + s->len); rd = p->re - (s->rbeg + s->len);
            max_gap = cal_max_gap(opt, qd < rd ? qd : (int)rd);
            w = max_gap < p->w ? max_gap : p->w;
            if (qd - rd < w && rd - qd < w) break;
        }
        if (i < (int)av->n) {
            for (i = k + 1; i < c->n; ++i) {
                const mem_seed_t *t;
                if (srt[i] == 0) continue;
                t = &c->seeds[(uint32_t)srt[i]];
                if (t->len < s->len * .95) continue;
                if (s->qbeg <= t->qbeg && s->qbeg + s->len - t->qbeg >= s->len >> 2 && t->qbeg - s->qbeg != t->rbeg - s->rbeg) break;
                if (t->qbeg <= s->qbeg && t->qbeg + t->len - s->qbeg >= s->len >> 2 && s->qbeg - t->qbeg != s->rbeg - t->rbeg) break;
            }
            if (i == c->n) {
#ifdef ORC_PROFILE
                tr_push(21, 1, 0, 0);
#endif
                srt[k] = 0; continue;
            }
        }
#ifdef ORC_PROFILE
        tr_push(21, 0, s->qbeg, s->len);
#endif
        VGROW(*av);
        a = &av->a[av->n++];
        memset(a, 0, sizeof(mem_alnreg_t));
        a->w = aw[0] = aw[1] = opt->w;
        a->score = a->truesc = -1;
        a->rid = c->rid;
        if (s->qbeg) {
            uint8_t *rs, *qs;
            int qle, tle, gtle, gscore;
            qs = malloc((size_t)s->qbeg);
            for (i = 0; i < s->qbeg; ++i) qs[i] = query[s->qbeg - 1 - i];
            tmp = s->rbeg - rmax[0];
#ifdef ORC_PROFILE
            tr_push(22, 0, 0, 0);
#endif
            rs = malloc(tmp > 0 ? (size_t)tmp : 1);
            for (i = 0; i < tmp; ++i) rs[i] = rseq[tmp - 1 - i];
            for (i = 0; i < MAX_BAND_TRY; ++i) {
                int prev = a->score;
                aw[0] = opt->w << i;
                a->score = ksw_extend2(s->qbeg, qs, (int)tmp, rs, 5, opt->mat, opt->o_del, opt->e_del, opt->o_ins, opt->e_ins,
                                       aw[0], opt->pen_clip5, opt->zdrop, s->len * opt->a, &qle, &tle, &gtle, &gscore, &max_off[0]);
                if (a->score == prev || max_off[0] < (aw[0] >> 1) + (aw[0] >> 2)) break;
            }
            if (gscore <= 0 || gscore <= a->score - opt->pen_clip5) {
                a->qb = s->qbeg - qle, a->rb = s->rbeg - tle;
                a->truesc = a->score;
            } else {
                a->qb = 0, a->rb = s->rbeg - gtle;
                a->truesc = gscore;
            }
            free(qs); free(rs);
        } else a->score = a->truesc = s->len * opt->a, a->qb = 0, a->rb = s->rbeg;
        if (s->qbeg + s->len != l_query) {
            int qle, tle, qe, re, gtle, gscore, sc0 = a->score;
            qe = s->qbeg + s->len;
            re = (int)(s->rbeg + s->len - rmax[0]);
#ifdef ORC_PROFILE
            tr_push(22, 1, 0, 0);
#endif
            for (i = 0; i < MAX_BAND_TRY; ++i) {
                int prev = a->score;
                aw[1] = opt->w << i;
                a->score = ksw_extend2(l_query - qe, query + qe, (int)(rmax[1] - rmax[0] - re), rseq + re, 5, opt->mat,
                                       opt->o_del, opt->e_del, opt->o_ins, opt->e_ins, aw[1], opt->pen_clip3, opt->zdrop,
                                       sc0, &qle, &tle, &gtle, &gscore, &max_off[1]);
                if (a->score == prev || max_off[1] < (aw[1] >> 1) + (aw[1] >> 2)) break;
            }
            if (gscore <= 0 || gscore <= a->score - opt->pen_clip3) {
                a->qe = qe + qle, a->re = rmax[0] + re + tle;
                a->truesc += a->score - sc0;
            } else {
                a->qe = l_query, a->re = rmax[0] + re + gtle;
                a->truesc += gscore - sc0;
            }
        } else a->qe = l_query, a->re = s->rbeg + s->len;
        for (i = 0, a->seedcov = 0; i < c->n; ++i) {
            const mem_seed_t *t = &c->seeds[i];
            if (t->qbeg >= a->qb && t->qbeg + t->len <= a->qe && t->rbeg >= a->rb && t->rbeg + t->len <= a->re)
                a->seedcov += t->len;
        }
        a->w = aw[0] > aw[1] ? aw[0] : aw[1];
        a->seedlen0 = s->len;
        a->frac_rep = c->frac_rep;
    }
    free(srt); free(rseq);
}

#define PATCH_MAX_R_BW 0.05f
#define PATCH_MIN_SC_RATIO 0.90f

static int mem_patch_reg(const mopt_t *opt, const orc_index *bns, const uint8_t *query, const mem_alnreg_t *a,
                         const mem_alnreg_t *b, int *_w)
{
    int w, score, q_s, r_s; double r;
    if (a->rb < bns->l_pac && b->rb >= bns->l_pac) return 0;
    if (a->qb >= b->qb || a->qe >= b->qe || a->re >= b->re) return 0;
    w = (int)((a->re - b->rb) - (a->qe - b->qb));
    w = w > 0 ? w : -w;
    r = (double)(a->re - b->rb) / (b->re - a->rb) - (double)(a->qe - b->qb) / (b->qe - a->qb);
    r = r > 0. ? r : -r;
    if (a->re < b->rb || a->qe < b->qb) {
        if (w > opt->w << 1 || r >= PATCH_MAX_R_BW) return 0;
    } else if (w > opt->w << 2 || r >= PATCH_MAX_R_BW * 2) return 0;
    w += a->w + b->w;
    w = w < opt->w << 2 ? w : opt->w << 2;
    score = 0;
    uint32_t *cg = bwa_gen_cigar2(opt->mat, opt->o_del, opt->e_del, opt->o_ins, opt->e_ins, w, bns->l_pac, bns->pac.a,
                                  b->qe - a->qb, query + a->qb, a->rb, b->re, &score, 0);
    free(cg);
    q_s = (int)((double)(b->qe - a->qb) / ((b->qe - b->qb) + (a->qe - a->qb)) * (b->score + a->score) + .499);
    r_s = (int)((double)(b->re - a->rb) / ((b->re - b->rb) + (a->re - a->rb)) * (b->score + a->score) + .499);
    if ((double)score / (q_s > r_s ? q_s : r_s) < PATCH_MIN_SC_RATIO) return 0;
    *_w = w;
    return score;
}

static int alnreg_slt2(const void *a_, const void *b_)
{ const mem_alnreg_t *a = a_, *b = b_; return a->re < b->re; }
static int alnreg_slt(const void *a_, const void *b_)
{
    const mem_alnreg_t *a = a_, *b = b_;
    return a->score > b->score || (a->score == b->score && (a->rb < b->rb || (a->rb == b->rb && a->qb < b->qb)));
}
static int alnreg_hlt(const void *a_, const void *b_)
{
    const mem_alnreg_t *a = a_, *b = b_;
    return a->score > b->score || (a->score == b->score && a->hash < b->hash);
}

static int mem_sort_dedup_patch(const mopt_t *opt, const orc_index *bns, const uint8_t *query, int n, mem_alnreg_t *a)
{
    int m, i, j;
    if (n <= 1) return n;
    ks_introsort((size_t)n, a, sizeof(mem_alnreg_t), alnreg_slt2);
    for (i = 0; i < n; ++i) a[i].n_comp = 1;
    for (i = 1; i < n; ++i) {
        mem_alnreg_t *p = &a[i];
        if (p->rid != a[i - 1].rid || p->rb >= a[i - 1].re + opt->max_chain_gap) continue;
        for (j = i - 1; j >= 0 && p->rid == a[j].rid && p->rb < a[j].re + opt->max_chain_gap; --j) {
            mem_alnreg_t *q = &a[j];
            int64_t or_, oq, mr, mq;
            int score, w;
            if (q->qe == q->qb) continue;
            or_ = q->re - p->rb;
            oq = q->qb < p->qb ? q->qe - p->qb : p->qe - q->qb;
            mr = q->re - q->rb < p->re - p->rb ? q->re - q->rb : p->re - p->rb;
            mq = q->qe - q->qb < p->qe - p->qb ? q->qe - q->qb : p->qe - p->qb;
            if (or_ > opt->mask_level_redun * mr && oq > opt->mask_level_redun * mq) {
                if (p->score < q->score) { p->qe = p->qb; break; }
                else q->qe = q->qb;
            } else if (q->rb < p->rb && (score = mem_patch_reg(opt, bns, query, q, p, &w)) > 0) {
                p->n_comp += q->n_comp + 1;
                p->seedcov = p->seedcov > q->seedcov ? p->seedcov : q->seedcov;
                p->sub = p->sub > q->sub ? p->sub : q->sub;
                p->csub = p->csub > q->csub ? p->csub : q->csub;
                p->qb = q->qb, p->rb = q->rb;
                p->truesc = p->score = score;
                p->w = w;
                q->qb = q->qe;
            }
        }
    }
    for (i = 0, m = 0; i < n; ++i)
        if (a[i].qe > a[i].qb) { if (m != i) a[m++] = a[i]; else ++m; }
    n = m;
    ks_introsort((size_t)n, a, sizeof(mem_alnreg_t), alnreg_slt);
    for (i = 1; i < n; ++i)
        if (a[i].score == a[i - 1].score && a[i].rb == a[i - 1].rb && a[i].qb == a[i - 1].qb) a[i].qe = a[i].qb;
    for (i = 1, m = 1; i < n; ++i)
        if (a[i].qe > a[i].qb) { if (m != i) a[m++] = a[i]; else ++m; }
    return m;
}

static inline uint64_t hash_64(uint64_t key)
{
    key += ~(key << 32);
    key ^= (key >> 22);
    key += ~(key << 13);
    key ^= (key >> 8);
    key += (key << 3);
    key ^= (key >> 15);
    key += ~(key << 27);
    key ^= (key >> 31);
    return key;
}

static void mem_mark_primary_se(const mopt_t *opt, int n, mem_alnreg_t *a, int64_t id)
{
    int i, k, tmp;
    VEC(int) z = {0, 0, 0};
    if (n == 0) return;
    for (i = 0; i < n; ++i) {
        a[i].sub = a[i].alt_sc = 0, a[i].secondary = a[i].secondary_all = -1, a[i].hash = hash_64((uint64_t)(id + i));
    }
    ks_introsort((size_t)n, a, sizeof(mem_alnreg_t), alnreg_hlt);
    /* mem_mark_primary_se_core */
    tmp = opt->a + opt->b;
    tmp = opt->o_del + opt->e_del > tmp ? opt->o_del + opt->e_del : tmp;
    tmp = opt->o_ins + opt->e_ins > tmp ? opt->o_ins + opt->e_ins : tmp;
    VPUSH(z, 0);
    for (i = 1; i < n; ++i) {
        for (k = 0; k < (int)z.n; ++k) {
            int j = z.a[k];
            int b_max = a[j].qb > a[i].qb ? a[j].qb : a[i].qb;
            int e_min = a[j].qe < a[i].qe ? a[j].qe : a[i].qe;
            if (e_min > b_max) {
                int min_l = a[i].qe - a[i].qb < a[j].qe - a[j].qb ? a[i].qe - a[i].qb : a[j].qe - a[j].qb;
                if (e_min - b_max >= min_l * opt->mask_level) {
                    if (a[j].sub == 0) a[j].sub = a[i].score;
                    if (a[j].score - a[i].score <= tmp && (a[j].is_alt || !a[i].is_alt)) ++a[j].sub_n;
                    break;
                }
            }
        }
        if (k == (int)z.n) VPUSH(z, i);
        else a[i].secondary = z.a[k];
    }
    for (i = 0; i < n; ++i) a[i].secondary_all = i;
    free(z.a);
}

/* ksw_align2(..., KSW_XSTART, 0) as mem_seed_sw uses it (ksw.c: ksw_qinit with size 2 -> ksw_i16); only
 * r.score is read.  Restated as a scalar emulation of the striped SSE2 kernel, lane for lane, because its
 * result is not the plain Gotoh optimum: p = 8 int16 lanes, query position j + k*slen in lane k of vector
 * j (slen = ceil(qlen/8), padding scores 0).  Per target row: the main loop computes H = max(diag + s, E,
 * F) with F carried only within a lane's segment, records the row maximum and updates E from that H; the
 * "lazy F" loop (at most 16 sweeps, leaving as soon as no lane has f > H - oe_ins) then carries F across
 * segment boundaries into H only -- neither E nor the maximum see those corrections.  Gap terms saturate
 * at 0 (_mm_subs_epu16); the score is the best row maximum (KSW_XSTOP unset: no early stop). */
#define KSW_P 8
static inline int sub0(int a, int b) { return a > b ? a - b : 0; }   /* _mm_subs_epu16 on values >= 0 */
static int ksw_align2_score(int qlen, const uint8_t *query, int tlen, const uint8_t *target, const int8_t *mat,
                            int o_del, int e_del, int o_ins, int e_ins)
{
    const int slen = (qlen + KSW_P - 1) / KSW_P, oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
    int16_t *H0 = calloc((size_t)slen * KSW_P, 2), *H1 = calloc((size_t)slen * KSW_P, 2), *E = calloc((size_t)slen * KSW_P, 2);
    int gmax = 0;
    for (int i = 0; i < tlen; ++i) {
        int f[KSW_P] = {0}, mx[KSW_P] = {0}, h[KSW_P];
        const int8_t *ma = mat + target[i] * 5;
        h[0] = 0;
        for (int k = 1; k < KSW_P; ++k) h[k] = H0[(slen - 1) * KSW_P + k - 1];
        for (int j = 0; j < slen; ++j) {
            for (int k = 0; k < KSW_P; ++k) {
                const int pos = j + k * slen;
                int v = h[k] + (pos < qlen ? ma[query[pos]] : 0);
                const int e = E[j * KSW_P + k];
                v = v > e ? v : e;
                v = v > f[k] ? v : f[k];
                mx[k] = mx[k] > v ? mx[k] : v;
                H1[j * KSW_P + k] = (int16_t)v;
                const int en = sub0(e, e_del), t = sub0(v, oe_del);
                E[j * KSW_P + k] = (int16_t)(en > t ? en : t);
                const int fn = sub0(f[k], e_ins), t2 = sub0(v, oe_ins);
                f[k] = fn > t2 ? fn : t2;
                h[k] = H0[j * KSW_P + k];
            }
        }
        for (int kk = 0; kk < 16; ++kk) {
            for (int k = KSW_P - 1; k > 0; --k) f[k] = f[k - 1];
            f[0] = 0;
            int more = 1;
            for (int j = 0; j < slen && more; ++j) {
                more = 0;
                for (int k = 0; k < KSW_P; ++k) {
                    int v = H1[j * KSW_P + k];
                    v = v > f[k] ? v : f[k];
                    H1[j * KSW_P + k] = (int16_t)v;
                    const int hv = sub0(v, oe_ins);
                    f[k] = sub0(f[k], e_ins);
                    if (f[k] > hv) more = 1;
                }
            }
            if (!more) break;
        }
        int imax = 0;
        for (int k = 0; k < KSW_P; ++k) imax = imax > mx[k] ? imax : mx[k];
        if (imax > gmax) gmax = imax;
        int16_t *sw = H0; H0 = H1; H1 = sw;
    }
    free(H0); free(H1); free(E);
    return gmax;
}

#define MEM_SHORT_EXT 50
#define MEM_SHORT_LEN 200
#define MEM_HSP_COEF 1.1f
#define MEM_MINSC_COEF 5.5f
#define MEM_SEEDSW_COEF 0.05f

/* mem_seed_sw (bwamem.c): SW score of a short seed's neighbourhood, -1 when no SW is needed */
static int mem_seed_sw(const mopt_t *opt, const orc_index *bns, int l_query, const uint8_t *query, const mem_seed_t *s)
{
    int qb, qe, rid;
    int64_t rb, re, mid, l_pac = bns->l_pac;
    if (s->len >= MEM_SHORT_LEN) return -1;
    qb = s->qbeg, qe = s->qbeg + s->len;
    rb = s->rbeg, re = s->rbeg + s->len;
    mid = (rb + re) >> 1;
    qb -= MEM_SHORT_EXT; qb = qb > 0 ? qb : 0;
    qe += MEM_SHORT_EXT; qe = qe < l_query ? qe : l_query;
    rb -= MEM_SHORT_EXT; rb = rb > 0 ? rb : 0;
    re += MEM_SHORT_EXT; re = re < l_pac << 1 ? re : l_pac << 1;
    if (rb < l_pac && l_pac < re) {
        if (mid < l_pac) re = l_pac;
        else rb = l_pac;
    }
    if (qe - qb >= MEM_SHORT_LEN || re - rb >= MEM_SHORT_LEN) return -1;
    uint8_t *rseq = bns_fetch_seq(bns, &rb, mid, &re, &rid);
    const int sc = ksw_align2_score(qe - qb, query + qb, (int)(re - rb), rseq, opt->mat, opt->o_del, opt->e_del,
                                    opt->o_ins, opt->e_ins);
    free(rseq);
    return sc;
}

/* mem_flt_chained_seeds (bwamem.c): for reads long enough, seeds whose neighbourhood scores below the
 * HSP threshold are dropped and the kept ones take the SW score (or len*a when no SW was run) */
static void mem_flt_chained_seeds(const mopt_t *opt, const orc_index *bns, int l_query, const uint8_t *query, int n_chn,
                                  mem_chain_t *a)
{
    double min_l = opt->min_chain_weight ? MEM_HSP_COEF * opt->min_chain_weight : MEM_MINSC_COEF * log(l_query);
    int i, j, k, min_HSP_score = (int)(opt->a * min_l + .499);
    if (min_l > MEM_SEEDSW_COEF * l_query) return;
    for (i = 0; i < n_chn; ++i) {
        mem_chain_t *c = &a[i];
        for (j = k = 0; j < c->n; ++j) {
            mem_seed_t *s = &c->seeds[j];
            s->score = mem_seed_sw(opt, bns, l_query, query, s);
            if (s->score < 0 || s->score >= min_HSP_score) {
                s->score = s->score < 0 ? s->len * opt->a : s->score;
                c->seeds[k++] = *s;
            }
        }
        c->n = k;
    }
}

int orc_ksw_align2_score(int qlen, const uint8_t *query, int tlen, const uint8_t *target, const int8_t *mat, int o_del,
                         int e_del, int o_ins, int e_ins)
{
    return ksw_align2_score(qlen, query, tlen, target, mat, o_del, e_del, o_ins, e_ins);
}

/* mem_align1 = mem_align1_core + mem_mark_primary_se (bwamem.c) */
static int mem_align1(const mopt_t *opt, const orc_index *idx, int l_seq, const uint8_t *seq, int64_t id, alnreg_v *regs)
{
    chain_v chn = {0, 0, 0};
    regs->n = 0;
    mem_chain(opt, idx, l_seq, seq, &chn);
    chn.n = (size_t)mem_chain_flt(opt, (int)chn.n, chn.a);
    mem_flt_chained_seeds(opt, idx, l_seq, seq, (int)chn.n, chn.a);
    for (size_t i = 0; i < chn.n; ++i) {
        mem_chain2aln(opt, idx, l_seq, seq, &chn.a[i], regs);
        free(chn.a[i].seeds);
    }
    free(chn.a);
    regs->n = (size_t)mem_sort_dedup_patch(opt, idx, seq, (int)regs->n, regs->a);
    mem_mark_primary_se(opt, (int)regs->n, regs->a, id);
    return 0;
}

static inline int infer_bw(int l1, int l2, int score, int a, int q, int r)
{
    int w;
    if (l1 == l2 && l1 * a - score < (q + r - a) << 1) return 0;
    w = (int)((double)((l1 < l2 ? l1 : l2) * a - score - q) / r + 2.);
    if (w < abs(l1 - l2)) w = abs(l1 - l2);
    return w;
}

typedef struct { int flag, is_rev, n_cigar, score; uint32_t *cigar; int64_t pos; int rid; } mem_aln_t;

static mem_aln_t mem_reg2aln(const mopt_t *opt, const orc_index *bns, int l_query, const uint8_t *query, const mem_alnreg_t *ar)
{
    mem_aln_t a; int i, w2, tmp, qb, qe, score = 0, is_rev, last_sc = -(1 << 30);
    int64_t pos, rb, re;
    memset(&a, 0, sizeof a);
    qb = ar->qb, qe = ar->qe; rb = ar->rb, re = ar->re;
    if (ar->secondary >= 0) a.flag |= 0x100;
    tmp = infer_bw(qe - qb, (int)(re - rb), ar->truesc, opt->a, opt->o_del, opt->e_del);
    w2 = infer_bw(qe - qb, (int)(re - rb), ar->truesc, opt->a, opt->o_ins, opt->e_ins);
    w2 = w2 > tmp ? w2 : tmp;
    if (w2 > opt->w) w2 = w2 < ar->w ? w2 : ar->w;
    i = 0; a.cigar = 0;
    do {
        free(a.cigar);
        w2 = w2 < opt->w << 2 ? w2 : opt->w << 2;
        a.cigar = bwa_gen_cigar2(opt->mat, opt->o_del, opt->e_del, opt->o_ins, opt->e_ins, w2, bns->l_pac, bns->pac.a,
                                 qe - qb, &query[qb], rb, re, &score, &a.n_cigar);
        if (score == last_sc || w2 == opt->w << 2) break;
        last_sc = score;
        w2 <<= 1;
    } while (++i < 3 && score < ar->truesc - opt->a);
    pos = bns_depos(bns, rb < bns->l_pac ? rb : re - 1, &is_rev);
    a.is_rev = is_rev;
    if (a.n_cigar > 0) {
        if ((a.cigar[0] & 0xf) == 2) {
            pos += a.cigar[0] >> 4;
            --a.n_cigar;
            memmove(a.cigar, a.cigar + 1, (size_t)a.n_cigar * 4);
        } else if ((a.cigar[a.n_cigar - 1] & 0xf) == 2) {
            --a.n_cigar;
        }
    }
    if (qb != 0 || qe != l_query) {
        int clip5 = is_rev ? l_query - qe : qb, clip3 = is_rev ? qb : l_query - qe;
        a.cigar = realloc(a.cigar, 4 * (size_t)(a.n_cigar + 2));
        if (clip5) {
            memmove(a.cigar + 1, a.cigar, (size_t)a.n_cigar * 4);
            a.cigar[0] = (uint32_t)clip5 << 4 | 3;
            ++a.n_cigar;
        }
        if (clip3) a.cigar[a.n_cigar++] = (uint32_t)clip3 << 4 | 3;
    }
    a.rid = bns_pos2rid(bns, pos);
    a.pos = pos - bns->anns.a[a.rid].offset;
    a.score = ar->score;
    return a;
}

/* ============================================================================================== */
/* public entry points                                                                             */
/* ============================================================================================== */
/* The seeding trace of one read (see tr_push): 4 int32 per call {kind (1 pass-1 smem, 2 pass-2 smem, 3 seed strategy),
 * forward trips (or SS trips before its interval is unique), backward trips (or SS steps on a unique interval), call index (pass 1 / SS: ordinal; pass 2:
 * the mem index k)}; returns the number of int32 written (at most cap). */
int orc_seed_trace(const orc_index *idx, const orc_opts *o, const uint8_t *q, int len, int32_t *out, int cap)
{
    orc_tr = out; orc_tr_n = 0; orc_tr_cap = cap;
    uint64_t tmp[4 * 512];
    orc_collect_intv(idx, o, q, len, tmp, 512);
    const int n = orc_tr_n;
    orc_tr = NULL; orc_tr_n = 0; orc_tr_cap = 0;
    return n;
}

/* The extension trace of one read (ORC_PROFILE builds only; tools/ext_model.py): 4 int32 per record {20, seeds, longest
 * seed} per mem_chain2aln call, {21, skipped, qbeg, len} per seed it
 * visits (qbeg and len for extended seeds), {22, side} per extension side (0 left, 1 right), {10, qlen,
 * tlen, w} per ksw_extend2 call and {11, cells, beg, end} per row of it; returns the number of int32 written. */
int orc_ext_trace(const orc_index *idx, const orc_opts *o, const uint8_t *q, int len, int64_t id, int32_t *out, int cap)
{
    orc_tr = out; orc_tr_n = 0; orc_tr_cap = cap;
    mopt_t opt; make_opt(o, &opt);
    alnreg_v regs = {0, 0, 0};
    if (idx->built) mem_align1(&opt, idx, len, q, id, &regs);
    free(regs.a);
    const int n = orc_tr_n;
    orc_tr = NULL; orc_tr_n = 0; orc_tr_cap = 0;
    return n;
}

int orc_collect_intv(const orc_index *idx, const orc_opts *o, const uint8_t *q, int len, uint64_t *out, int max)
{
    mopt_t opt; make_opt(o, &opt);
    intv_v mem = {0, 0, 0}, mem1 = {0, 0, 0}, tmpv[2] = {{0, 0, 0}, {0, 0, 0}};
    if (!idx->built) return 0;
    mem_collect_intv(&opt, idx, len, q, &mem, &mem1, tmpv);
    int n = (int)mem.n;
    for (int i = 0; i < n && i < max; ++i) {
        out[4 * i] = mem.a[i].x[0]; out[4 * i + 1] = mem.a[i].x[1]; out[4 * i + 2] = mem.a[i].x[2]; out[4 * i + 3] = mem.a[i].info;
    }
    free(mem.a); free(mem1.a); free(tmpv[0].a); free(tmpv[1].a);
    return n;
}

int orc_align_regions(const orc_index *idx, const orc_opts *o, const uint8_t *q, int len, int64_t id,
                      orc_region *out, int max_regs)
{
    mopt_t opt; make_opt(o, &opt);
    alnreg_v regs = {0, 0, 0};
    if (!idx->built) return 0;
    if (mem_align1(&opt, idx, len, q, id, &regs) < 0) return -1;
    int n = (int)regs.n;
    for (int i = 0; i < n && i < max_regs; ++i) {
        mem_alnreg_t *r = &regs.a[i];
        orc_region *x = &out[i];
        memset(x, 0, sizeof *x);
        x->rb = r->rb; x->re = r->re; x->qb = r->qb; x->qe = r->qe; x->rid = r->rid; x->score = r->score;
        x->truesc = r->truesc; x->sub = r->sub; x->csub = r->csub; x->sub_n = r->sub_n; x->w = r->w;
        x->seedcov = r->seedcov; x->secondary = r->secondary; x->seedlen0 = r->seedlen0; x->n_comp = r->n_comp;
        x->hash = r->hash;
        mem_aln_t a = mem_reg2aln(&opt, idx, len, q, r);
        x->flag = a.flag; x->is_rev = a.is_rev; x->n_cigar = a.n_cigar;
        for (int j = 0; j < a.n_cigar && j < 64; ++j) x->cigar[j] = a.cigar[j];
        free(a.cigar);
    }
    free(regs.a);
    return n;
}

typedef struct { char *s; size_t l, m; } kstr_t;
static void ks_puts(kstr_t *k, const char *s, size_t n)
{
    if (k->l + n + 1 > k->m) { k->m = (k->l + n + 1) * 2; k->s = realloc(k->s, k->m); }
    memcpy(k->s + k->l, s, n); k->l += n; k->s[k->l] = 0;
}
static void ks_printf_int(kstr_t *k, long long v) { char b[32]; int n = snprintf(b, sizeof b, "%lld", v); ks_puts(k, b, (size_t)n); }

/* BwaIndex::align_sequence, bwa.cpp:141-181, rendered as bwa_result rows (without query_id) */
char *orc_align_tsv(const orc_index *idx, const orc_opts *o, const uint8_t *ns, int64_t id)
{
    kstr_t out = {0, 0, 0};
    ks_puts(&out, "", 0);
    if (!idx->built) return out.s;                      /* pac_forward.empty() -> {} */
    mopt_t opt; make_opt(o, &opt);
    char *text = orc_nuclseq_to_text(ns);
    int len = (int)strlen(text);
    uint8_t *q = malloc((size_t)len + 1);
    for (int i = 0; i < len; ++i) q[i] = (uint8_t)nt4_of((unsigned char)text[i]);
    alnreg_v regs = {0, 0, 0};
    if (mem_align1(&opt, idx, len, q, id, &regs) < 0) { free(q); free(text); free(out.s); return NULL; }
    for (size_t r = 0; r < regs.n; ++r) {
        mem_alnreg_t *al = &regs.a[r];
        int64_t ref_offset = idx->anns.a[al->rid].offset;
        mem_aln_t d = mem_reg2aln(&opt, idx, len, q, al);
        ks_printf_int(&out, idx->anns.a[al->rid].id); ks_puts(&out, "\t", 1);
        if (al->rb >= idx->l_pac) ks_puts(&out, "*", 1);   /* Q7: out-of-bounds read in the reference */
        else {                                             /* extract_reference_subseq, bwa.cpp:55-68 */
            int64_t rl = al->re - al->rb;
            char *sub = malloc((size_t)rl + 1);
            for (int64_t i = 0; i < rl; ++i) sub[i] = "ACGT"[pac_raw_get(idx->pac.a, (uint64_t)(al->rb + i))];
            for (size_t h = 0; h < idx->holes.n; ++h) {
                const hole_t *hl = &idx->holes.a[h];
                int64_t lo = hl->offset > al->rb ? hl->offset : al->rb;
                int64_t hi = hl->offset + hl->len < al->re ? hl->offset + hl->len : al->re;
                for (int64_t i = lo; i < hi; ++i) sub[i - al->rb] = hl->amb;
            }
            ks_puts(&out, sub, (size_t)rl); free(sub);
        }
        ks_puts(&out, "\t", 1); ks_printf_int(&out, (int32_t)(al->rb - ref_offset));
        ks_puts(&out, "\t", 1); ks_printf_int(&out, (int32_t)(al->re - ref_offset));
        ks_puts(&out, "\t", 1); ks_printf_int(&out, (int32_t)(al->re - al->rb));
        ks_puts(&out, "\t", 1); ks_puts(&out, text + al->qb, (size_t)(al->qe - al->qb));
        ks_puts(&out, "\t", 1); ks_printf_int(&out, al->qb);
        ks_puts(&out, "\t", 1); ks_printf_int(&out, al->qe);
        ks_puts(&out, "\t", 1); ks_printf_int(&out, al->qe - al->qb);
        ks_puts(&out, "\t", 1); ks_puts(&out, (d.flag & 0x100) == 0 ? "t" : "f", 1);
        ks_puts(&out, "\t", 1); ks_puts(&out, (d.flag & 0x100) != 0 ? "t" : "f", 1);
        ks_puts(&out, "\t", 1); ks_puts(&out, d.is_rev ? "t" : "f", 1);
        ks_puts(&out, "\t", 1);
        for (int c = 0; c < d.n_cigar; ++c) {                  /* cigar_compressed_to_string + bam_cigar_opchr */
            ks_printf_int(&out, d.cigar[c] >> 4);
            ks_puts(&out, &"MIDNSHP=XB"[d.cigar[c] & 0xf], 1);
        }
        ks_puts(&out, "\t", 1); ks_printf_int(&out, d.score);
        ks_puts(&out, "\n", 1);
        free(d.cigar);
    }
    free(regs.a); free(q); free(text);
    return out.s;
}

/* glibc lrand48 from the zero state: X_{k+1} = (0x5DEECE66D X_k + 0xB) mod 2^48, output X >> 17 */
int64_t orc_lrand48_at(uint64_t pos)
{
    const uint64_t M = (1ULL << 48) - 1;
    uint64_t A = 1, C = 0, a = 0x5DEECE66DULL, c = 0xB, e = pos + 1;   /* compose the map e times */
    while (e) {
        if (e & 1) { C = (a * C + c) & M; A = (a * A) & M; }
        c = (a * c + c) & M; a = (a * a) & M;
        e >>= 1;
    }
    (void)A;
    return (int64_t)(C >> 17);
}

/* ---- batch (bench cpu_baseline) ------------------------------------------------------------- */
typedef struct {
    const orc_index *idx; const mopt_t *opt; const uint8_t *codes; const int64_t *off;
    int lo, hi; uint64_t first_call; int64_t nreg; uint64_t ck; int err; uint64_t ab[4];
} job_t;

static inline uint64_t fnv(uint64_t h, uint64_t v) { for (int i = 0; i < 8; ++i) { h ^= (v >> (8 * i)) & 0xff; h *= 0x100000001b3ULL; } return h; }

static void *batch_worker(void *arg)
{
    job_t *j = arg;
    alnreg_v regs = {0, 0, 0};
    uint64_t ck = 0;
    memset(orc_ab, 0, sizeof orc_ab);
    for (int r = j->lo; r < j->hi; ++r) {
        int len = (int)(j->off[r + 1] - j->off[r]);
        const uint8_t *q = j->codes + j->off[r];
        if (mem_align1(j->opt, j->idx, len, q, orc_lrand48_at(j->first_call + (uint64_t)r), &regs) < 0) { j->err = 1; break; }
        uint64_t h = 0xcbf29ce484222325ULL;
        h = fnv(h, (uint64_t)r);
        for (size_t i = 0; i < regs.n; ++i) {
            mem_alnreg_t *al = &regs.a[i];
            mem_aln_t d = mem_reg2aln(j->opt, j->idx, len, q, al);
            h = fnv(h, (uint64_t)al->rb); h = fnv(h, (uint64_t)al->re); h = fnv(h, (uint64_t)(uint32_t)al->qb);
            h = fnv(h, (uint64_t)(uint32_t)al->qe); h = fnv(h, (uint64_t)(uint32_t)al->score); h = fnv(h, (uint64_t)d.flag);
            for (int c = 0; c < d.n_cigar; ++c) h = fnv(h, d.cigar[c]);
            free(d.cigar);
        }
        ck += h;                /* order-independent sum of per-read hashes */
        j->nreg += (int64_t)regs.n;
    }
    j->ck = ck;
    memcpy(j->ab, orc_ab, sizeof orc_ab);
    free(regs.a);
    return NULL;
}

/* seeding only (bench C2 cpu_baseline): mem_collect_intv per read; checksum over (x[0], x[2], info) */
static void *seed_worker(void *arg)
{
    job_t *j = arg;
    intv_v mem = {0, 0, 0}, mem1 = {0, 0, 0}, tmpv[2] = {{0, 0, 0}, {0, 0, 0}};
    uint64_t ck = 0;
    memset(orc_ab, 0, sizeof orc_ab);
    for (int r = j->lo; r < j->hi; ++r) {
        int len = (int)(j->off[r + 1] - j->off[r]);
        mem_collect_intv(j->opt, j->idx, len, j->codes + j->off[r], &mem, &mem1, tmpv);
        uint64_t h = 0xcbf29ce484222325ULL;
        h = fnv(h, (uint64_t)r);
        for (size_t i = 0; i < mem.n; ++i) {
            h = fnv(h, mem.a[i].x[0]); h = fnv(h, mem.a[i].x[2]); h = fnv(h, mem.a[i].info);
        }
        ck += h;
        j->nreg += (int64_t)mem.n;
    }
    j->ck = ck;
    memcpy(j->ab, orc_ab, sizeof orc_ab);
    free(mem.a); free(mem1.a); free(tmpv[0].a); free(tmpv[1].a);
    return NULL;
}

int64_t orc_seed_batch(const orc_index *idx, const orc_opts *o, const uint8_t *codes, const int64_t *offsets, int n,
                       int threads, uint64_t *checksum)
{
    mopt_t opt; make_opt(o, &opt);
    if (!idx->built) { if (checksum) *checksum = 0; return 0; }
    if (threads < 1) threads = 1;
    pthread_t *th = malloc(sizeof(pthread_t) * (size_t)threads);
    job_t *jobs = calloc((size_t)threads, sizeof(job_t));
    for (int t = 0; t < threads; ++t) {
        jobs[t] = (job_t){ idx, &opt, codes, offsets, (int)((int64_t)n * t / threads), (int)((int64_t)n * (t + 1) / threads),
                           0, 0, 0, 0, {0, 0, 0, 0} };
        pthread_create(&th[t], NULL, seed_worker, &jobs[t]);
    }
    int64_t nint = 0; uint64_t ck = 0;
    memset(orc_ab_last, 0, sizeof orc_ab_last);
    for (int t = 0; t < threads; ++t) {
        pthread_join(th[t], NULL); nint += jobs[t].nreg; ck += jobs[t].ck;
        for (int c = 0; c < 4; ++c) orc_ab_last[c] += jobs[t].ab[c];
    }
    free(th); free(jobs);
    if (checksum) *checksum = ck;
    return nint;
}

int64_t orc_align_batch(const orc_index *idx, const orc_opts *o, const uint8_t *codes, const int64_t *offsets,
                        int n, uint64_t first_call, int threads, uint64_t *checksum)
{
    mopt_t opt; make_opt(o, &opt);
    if (!idx->built) { if (checksum) *checksum = 0; return 0; }
    if (threads < 1) threads = 1;
    pthread_t *th = malloc(sizeof(pthread_t) * (size_t)threads);
    job_t *jobs = calloc((size_t)threads, sizeof(job_t));
    for (int t = 0; t < threads; ++t) {
        jobs[t] = (job_t){ idx, &opt, codes, offsets, (int)((int64_t)n * t / threads), (int)((int64_t)n * (t + 1) / threads),
                           first_call, 0, 0, 0, {0, 0, 0, 0} };
        pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
    }
    int64_t nreg = 0; uint64_t ck = 0; int err = 0;
    memset(orc_ab_last, 0, sizeof orc_ab_last);
    for (int t = 0; t < threads; ++t) {
        pthread_join(th[t], NULL); nreg += jobs[t].nreg; ck += jobs[t].ck; err |= jobs[t].err;
        for (int c = 0; c < 4; ++c) orc_ab_last[c] += jobs[t].ab[c];
    }
    free(th); free(jobs);
    if (checksum) *checksum = ck;
    return err ? -1 : nreg;
}

/* ---- batch TSV (parity tests at config sizes) ----------------------------------------------- */
typedef struct {
    const orc_index *idx; const orc_opts *o; const uint8_t *const *reads; int lo, hi; uint64_t first_call;
    char **rows; int err;
} tsv_job_t;

static void *tsv_worker(void *arg)
{
    tsv_job_t *j = arg;
    for (int r = j->lo; r < j->hi; ++r) {
        j->rows[r] = orc_align_tsv(j->idx, j->o, j->reads[r], orc_lrand48_at(j->first_call + (uint64_t)r));
        if (!j->rows[r]) { j->err = 1; break; }
    }
    return NULL;
}

char *orc_align_tsv_batch(const orc_index *idx, const orc_opts *o, const uint8_t *const *reads, int n,
                          uint64_t first_call, int threads, int64_t *rows_per_read)
{
    if (threads < 1) threads = 1;
    char **rows = calloc((size_t)(n > 0 ? n : 1), sizeof(char *));
    pthread_t *th = malloc(sizeof(pthread_t) * (size_t)threads);
    tsv_job_t *jobs = calloc((size_t)threads, sizeof(tsv_job_t));
    for (int t = 0; t < threads; ++t) {
        jobs[t] = (tsv_job_t){ idx, o, reads, (int)((int64_t)n * t / threads), (int)((int64_t)n * (t + 1) / threads),
                               first_call, rows, 0 };
        pthread_create(&th[t], NULL, tsv_worker, &jobs[t]);
    }
    int err = 0;
    for (int t = 0; t < threads; ++t) { pthread_join(th[t], NULL); err |= jobs[t].err; }
    size_t total = 1;
    for (int r = 0; r < n; ++r) total += rows[r] ? strlen(rows[r]) : 0;
    char *out = err ? NULL : malloc(total), *p = out;
    for (int r = 0; r < n; ++r) {
        if (out) {
            size_t l = strlen(rows[r]);
            int64_t c = 0;
            for (size_t i = 0; i < l; ++i) c += rows[r][i] == '\n';
            if (rows_per_read) rows_per_read[r] = c;
            memcpy(p, rows[r], l); p += l;
        }
        free(rows[r]);
    }
    if (out) *p = 0;
    free(rows); free(th); free(jobs);
    return out;
}
