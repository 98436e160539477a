// dev_common.h -- device helpers shared by the HIP kernels (reference text access, bntseq
// coordinate helpers, DP accessors, scoring, wave reductions).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bsq_device.h"

namespace bsq {

#ifndef DEV
#define DEV __device__ __forceinline__
#endif

// ------------------------------------------------------------------------------------------------
// reference text access (bntseq.c _get_pac / bns_get_seq semantics)
// ------------------------------------------------------------------------------------------------
DEV int pac_get(const uint8_t *pac, int64_t i) { return (pac[i >> 2] >> ((~i & 3) << 1)) & 3; }
// base of the forward+reverse text at coordinate p in [0, 2*l_pac)
DEV int ref_at(const DIndex &ix, int64_t p)
{
    return p < ix.l_pac ? pac_get(ix.pac, p) : 3 - pac_get(ix.pac, (ix.l_pac << 1) - 1 - p);
}

// ------------------------------------------------------------------------------------------------
// wave-aggregated counter add (one atomic per wave and counter)
// ------------------------------------------------------------------------------------------------
DEV void wave_add(unsigned long long *dst, unsigned long long v)
{
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(dst, v);
}

DEV int read_of(const int32_t *sel, int i) { return sel ? sel[i] : i; }

// ------------------------------------------------------------------------------------------------
// bntseq helpers
// ------------------------------------------------------------------------------------------------
DEV int64_t depos(const DIndex &ix, int64_t pos, int &is_rev)
{
    return (is_rev = (pos >= ix.l_pac)) ? (ix.l_pac << 1) - 1 - pos : pos;
}

DEV int pos2rid(const DIndex &ix, int64_t pos_f)
{
    if (pos_f >= ix.l_pac) return -1;
    int left = 0, mid = 0, right = ix.n_anns;
    while (left < right) {
        mid = (left + right) >> 1;
        if (pos_f >= ix.ann_off[mid]) {
            if (mid == ix.n_anns - 1) break;
            if (pos_f < ix.ann_off[mid + 1]) break;
            left = mid + 1;
        } else right = mid;
    }
    return mid;
}

DEV int intv2rid(const DIndex &ix, int64_t rb, int64_t re)
{
    int is_rev;
    if (rb < ix.l_pac && re > ix.l_pac) return -2;
    int rid_b = pos2rid(ix, depos(ix, rb, is_rev));
    int rid_e = rb < re ? pos2rid(ix, depos(ix, re - 1, is_rev)) : rid_b;
    return rid_b == rid_e ? rid_b : -1;
}

struct QAcc {   // query[j] = base[start + dir*j]
    const uint8_t *base; int start, dir;
    DEV int operator()(int j) const { return base[start + dir * j]; }
};
struct TAcc {   // target[i] = ref_at(start + dir*i)
    const DIndex *ix; int64_t start; int dir;
    DEV int operator()(int i) const { return ref_at(*ix, start + (int64_t)dir * i); }
};

// substitution scores of bwa_fill_scmat's matrix, held in registers by the DP loops
struct Score {
    int match, mis, amb;
    // bitmask selects: a ?: chain here gets turned into an indexed load from a private (scratch) table
    DEV int operator()(int t, int q) const
    {
        const int eq = -(int)(t == q), nn = -(int)((t | q) >= 4);
        const int r = (match & eq) | (mis & ~eq);
        return (amb & nn) | (r & ~nn);
    }
};
DEV Score score_of(const DOpts &o) { Score s; s.match = o.mat_match; s.mis = o.mat_mismatch; s.amb = o.mat_amb; return s; }

DEV int mat_sc(const DOpts &o, int t, int q)
{
    return (t == 4 || q == 4) ? o.mat_amb : (t == q ? o.mat_match : o.mat_mismatch);
}

// (int)((double)x / d + k) -- libbwa's band and gap-length formulas -- in integers (d > 0, |x| < 2^31): the
// double quotient is within an ulp of x/d, which lies at least 1/d from the next integer unless it is one, and
// both the conversion and C's integer division truncate toward zero, so the two agree for every input
// d is a gap-extension penalty (a kernel argument, uniform across the wave): the SQL default 1 takes a scalar
// branch around the ~30-instruction integer division
DEV int idiv_plus(int x, int d, int k) { return d == 1 ? x + k : (x + k * d) / d; }

DEV int infer_bw(int l1, int l2, int score, int a, int q, int r)
{
    int w;
    if (l1 == l2 && l1 * a - score < (q + r - a) << 1) return 0;
    w = idiv_plus((l1 < l2 ? l1 : l2) * a - score - q, r, 2);
    int d = l1 - l2; d = d < 0 ? -d : d;
    if (w < d) w = d;
    return w;
}

// ksw_global2 on an n x n problem (bwa_gen_cigar2 with l_query == rlen) whose gapless diagonal scores
// `diag`: every other path through the band has g >= 1 insertions and as many deletions, so it scores at
// most (n - g)*mat_max - (o_ins + g*e_ins) - (o_del + g*e_del) <= (n-1)*mat_max - oe_ins - oe_del.  When
// the diagonal beats that bound strictly, every diagonal cell's M is strictly above its E and F (an E/F
// path to (i,i) completed along the diagonal would reach the bound), so the DP's traceback bits there are
// all 0, the walk from (n-1, n-1) is n diagonal steps and eh[qlen].x == diag, for any band w >= 0: the
// result is "nM" with score `diag`, exactly what the DP returns, so the DP is skipped.
DEV bool diagonal_wins(const DOpts &o, int n, int diag)
{
    const int64_t bound = (int64_t)(n - 1) * o.mat_max - (o.o_ins + o.e_ins) - (o.o_del + o.e_del);
    return (int64_t)diag > bound;
}

// Sequential reader of the target bases target(i) = ref_at(start + dir*i), i = 0, 1, 2, ...: keeps the
// current and the next 16-base pac word in registers so the per-row base never waits on memory.
struct TStream {
    const uint8_t *pac;
    int64_t fp;         // forward-strand pac position of the next base
    int fstep;          // +1 / -1 along the forward pac
    int comp;           // 3 on the reverse strand (base = 3 - pac)
    int64_t cur_w, max_w;
    uint32_t cur, nxt;
    DEV uint32_t load(int64_t w) const { return (w >= 0 && w <= max_w) ? *reinterpret_cast<const uint32_t *>(pac + 4 * w) : 0u; }
    DEV void init(const DIndex &ix, int64_t start, int dir)
    {
        pac = ix.pac;
        max_w = (ix.l_pac >> 4);
        if (start < ix.l_pac) { fp = start; fstep = dir; comp = 0; }
        else { fp = (ix.l_pac << 1) - 1 - start; fstep = -dir; comp = 3; }
        cur_w = fp >> 4;
        cur = load(cur_w);
        nxt = load(cur_w + fstep);
    }
    DEV int next()
    {
        const int64_t w = fp >> 4;
        if (w != cur_w) { cur = w == cur_w + fstep ? nxt : load(w); cur_w = w; nxt = load(w + fstep); }
        const int byte = (int)((fp >> 2) & 3), sh = (int)((~fp & 3) << 1);
        const int b = (int)((cur >> (8 * byte + sh)) & 3u);
        fp += fstep;
        return b ^ comp;
    }
};

}  // namespace bsq
