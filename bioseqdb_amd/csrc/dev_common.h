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

DEV int mat_sc(const DOpts &o, int t, int q)
{
    return (t == 4 || q == 4) ? o.mat_amb : (t == q ? o.mat_match : o.mat_mismatch);
}

DEV int infer_bw(int l1, int l2, int score, int a, int q, int r)
{
    int w;
    if (l1 == l2 && l1 * a - score < (q + r - a) << 1) return 0;
    w = (int)((double)((l1 < l2 ? l1 : l2) * a - score - q) / r + 2.);
    int d = l1 - l2; d = d < 0 ? -d : d;
    if (w < d) w = d;
    return w;
}


}  // namespace bsq
