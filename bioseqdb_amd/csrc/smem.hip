// smem.hip -- main-pass SMEM seeding kernel (libbwa mem_collect_intv: bwt_smem1 x2 passes +
// bwt_seed_strategy1), one read per lane, with the SMEM working list held in LDS.
//
// Layout choices:
//  * interval coordinates are u32 when the text has < 2^32 rows (the 100 Mbp configs);
//  * bwt_extend computes only the interval of the requested base (no dynamically indexed ok[4]);
//  * the forward/backward list of bwt_smem1 lives in LDS, interleaved by lane (conflict-free), and
//    is compacted in place in the backward phase (each prev entry yields at most one curr entry).
//    After the forward phase libbwa only reads x[0], x[2] and the end position of list entries
//    (backward extensions never read x[1]), so an entry is 10 bytes;
//  * smem1's per-call output (mem1) is staged at the tail of the read's output slot.
// Reads that exceed the LDS list or the output slot are flagged and re-run by the large-capacity
// kernel k_smem (align_kernels.hip).  Output is identical to k_smem, interval for interval.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bsq_device.h"

namespace bsq {

#define DEV __device__ __forceinline__

template <typename X>
struct FM {
    const OccBlock *occ;
    X l2_0, l2_1, l2_2, l2_3, l2_4, primary;
    DEV X L2(int c) const { return c == 0 ? l2_0 : c == 1 ? l2_1 : c == 2 ? l2_2 : c == 3 ? l2_3 : l2_4; }
};

template <typename X>
DEV void occ4x(const FM<X> &fm, X k, X c[4])
{
    if (k == (X)-1) { c[0] = c[1] = c[2] = c[3] = 0; return; }
    k -= (k >= fm.primary);
    const uint4 *p = reinterpret_cast<const uint4 *>(fm.occ + (k >> 7));
    uint4 w0 = p[0], w1 = p[1], w2 = p[2], w3 = p[3];
    const uint32_t r = (uint32_t)(k & 127) + 1;
    uint64_t h0 = (uint64_t)w2.y << 32 | w2.x, h1 = (uint64_t)w2.w << 32 | w2.z;
    uint64_t l0 = (uint64_t)w3.y << 32 | w3.x, l1 = (uint64_t)w3.w << 32 | w3.z;
    uint64_t m0 = r >= 64 ? ~0ull : ((1ull << r) - 1);
    uint64_t m1 = r >= 128 ? ~0ull : (r > 64 ? ((1ull << (r - 64)) - 1) : 0ull);
    uint32_t n3 = __popcll(h0 & l0 & m0) + __popcll(h1 & l1 & m1);
    uint32_t n2 = __popcll(h0 & ~l0 & m0) + __popcll(h1 & ~l1 & m1);
    uint32_t n1 = __popcll(~h0 & l0 & m0) + __popcll(~h1 & l1 & m1);
    if (sizeof(X) == 4) {
        c[0] = (X)w0.x + (r - n1 - n2 - n3);
        c[1] = (X)w0.z + n1;
        c[2] = (X)w1.x + n2;
        c[3] = (X)w1.z + n3;
    } else {
        c[0] = (X)((uint64_t)w0.y << 32 | w0.x) + (r - n1 - n2 - n3);
        c[1] = (X)((uint64_t)w0.w << 32 | w0.z) + n1;
        c[2] = (X)((uint64_t)w1.y << 32 | w1.x) + n2;
        c[3] = (X)((uint64_t)w1.w << 32 | w1.z) + n3;
    }
}

template <typename X>
DEV X pick(const X v[4], int c) { return c == 0 ? v[0] : c == 1 ? v[1] : c == 2 ? v[2] : v[3]; }

// bwt_extend restricted to base c: returns (x_new_side, x_other_side, x2).  `a` is the interval end
// used for the rank queries (x[1] forward, x[0] backward), `o` the other one.
template <typename X>
DEV void extend1(const FM<X> &fm, X a, X o, X x2, int c, X &na, X &no, X &nx2, uint64_t &nblk)
{
    X tk[4], tl[4];
    const X k = a - 1, l = a - 1 + x2;
    occ4x(fm, k, tk);
    occ4x(fm, l, tl);
    {
        X kk = k == (X)-1 ? k : k - (k >= fm.primary), ll = l - (l >= fm.primary);
        nblk += (k == (X)-1 || (kk >> 7) == (ll >> 7)) ? 1 : 2;
    }
    const X d3 = tl[3] - tk[3], d2 = tl[2] - tk[2], d1 = tl[1] - tk[1];
    na = fm.L2(c) + 1 + pick(tk, c);
    nx2 = pick(tl, c) - pick(tk, c);
    no = o + (X)(a <= fm.primary && a + x2 - 1 >= fm.primary) + (c < 3 ? d3 : 0) + (c < 2 ? d2 : 0) + (c < 1 ? d1 : 0);
}

// LDS list of (x0, x2, end) entries for one lane: entry e at base[e * stride]
template <typename X>
struct LList {
    X *x0, *x2;
    uint16_t *end;
    int stride, cap;
    DEV void set(int e, X a, X b, int en) { x0[e * stride] = a; x2[e * stride] = b; end[e * stride] = (uint16_t)en; }
};

struct OutSlot {   // the read's output intervals (global), mem grows from the front, mem1 from the back
    Intv *a;
    int n, cap, n1;
};

template <typename X>
DEV int smem1_lds(const FM<X> &fm, int len, const uint8_t *q, int x, int min_intv, LList<X> &L, OutSlot &S,
                  bool &ovf, uint64_t &nblk)
{
    S.n1 = 0;
    if (q[x] > 3) return x + 1;
    if (min_intv < 1) min_intv = 1;
    int c0 = q[x];
    X ik0 = fm.L2(c0) + 1, ik2 = fm.L2(c0 + 1) - fm.L2(c0), ik1 = fm.L2(3 - c0) + 1;
    int ikend = x + 1;
    int n = 0, i;
    int qi = x + 1 < len ? q[x + 1] : 0;
    for (i = x + 1; i < len; ++i) {
        const int cur = qi;
        qi = i + 1 < len ? q[i + 1] : 0;   // prefetch the next base
        if (cur < 4) {
            const int c = 3 - cur;
            X n1, n0, n2;
            extend1(fm, ik1, ik0, ik2, c, n1, n0, n2, nblk);
            if (n2 != ik2) {
                if (n >= L.cap) { ovf = true; return len; }
                L.set(n++, ik0, ik2, ikend);
                if (n2 < (X)min_intv) break;
            }
            ik0 = n0; ik1 = n1; ik2 = n2; ikend = i + 1;
        } else {
            if (n >= L.cap) { ovf = true; return len; }
            L.set(n++, ik0, ik2, ikend);
            break;
        }
    }
    if (i == len) {
        if (n >= L.cap) { ovf = true; return len; }
        L.set(n++, ik0, ik2, ikend);
    }
    for (int j = 0; j < (n >> 1); ++j) {   // reverse: longest match first
        const int a = j * L.stride, b = (n - 1 - j) * L.stride;
        X t0 = L.x0[a], t2 = L.x2[a];
        uint16_t te = L.end[a];
        L.x0[a] = L.x0[b]; L.x2[a] = L.x2[b]; L.end[a] = L.end[b];
        L.x0[b] = t0; L.x2[b] = t2; L.end[b] = te;
    }
    const int ret = L.end[0];
    int last_start = 0x7fffffff;
    for (i = x - 1; i >= -1; --i) {
        const int c = i < 0 ? -1 : (q[i] < 4 ? q[i] : -1);
        int nc = 0;
        X last_x2 = 0;
        for (int j = 0; j < n; ++j) {
            const X p0 = L.x0[j * L.stride], p2 = L.x2[j * L.stride];
            const int pe = L.end[j * L.stride];
            bool keep_hit;
            X o0 = 0, o1, o2 = 0;
            if (c >= 0) {
                extend1(fm, p0, (X)0, p2, c, o0, o1, o2, nblk);   // x[1] is dead in the backward phase
                keep_hit = o2 < (X)min_intv;
            } else keep_hit = true;
            if (keep_hit) {
                if (nc == 0 && (S.n1 == 0 || i + 1 < last_start)) {
                    if (S.n + S.n1 >= S.cap) { ovf = true; return len; }
                    Intv &m = S.a[S.cap - 1 - S.n1];
                    m.x[0] = p0; m.x[1] = 0; m.x[2] = p2;
                    m.info = (uint64_t)(uint32_t)(i + 1) << 32 | (uint32_t)pe;
                    ++S.n1;
                    last_start = i + 1;
                }
            } else if (nc == 0 || o2 != last_x2) {
                L.set(nc++, o0, o2, pe);
                last_x2 = o2;
            }
        }
        if (nc == 0) break;
        n = nc;
    }
    return ret;
}

template <typename X>
DEV int seed_strategy1_x(const FM<X> &fm, int len, const uint8_t *q, int x, int min_len, int max_intv, Intv &mem,
                         uint64_t &nblk)
{
    mem.x[0] = mem.x[1] = mem.x[2] = mem.info = 0;
    if (q[x] > 3) return x + 1;
    const int c0 = q[x];
    X ik0 = fm.L2(c0) + 1, ik2 = fm.L2(c0 + 1) - fm.L2(c0), ik1 = fm.L2(3 - c0) + 1;
    int qi = x + 1 < len ? q[x + 1] : 0;
    for (int i = x + 1; i < len; ++i) {
        const int cur = qi;
        qi = i + 1 < len ? q[i + 1] : 0;
        if (cur < 4) {
            const int c = 3 - cur;
            X n1, n0, n2;
            extend1(fm, ik1, ik0, ik2, c, n1, n0, n2, nblk);
            if (n2 < (X)max_intv && i - x >= min_len) {
                mem.x[0] = n0; mem.x[1] = n1; mem.x[2] = n2;
                mem.info = (uint64_t)x << 32 | (uint64_t)(i + 1);
                return i + 1;
            }
            ik0 = n0; ik1 = n1; ik2 = n2;
        } else return i + 1;
    }
    return len;
}

DEV void wave_add2(unsigned long long *dst, unsigned long long v)
{
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(dst, v);
}

template <typename X>
__global__ void __launch_bounds__(256) k_smem_lds(DIndex ix, DOpts o, Caps cp, const uint8_t *codes, const int64_t *offs,
                                                  int n, Intv *intv_out, int32_t *n_intv, uint32_t *status,
                                                  Counters *ctr, int lcap)
{
    extern __shared__ uint8_t lds_raw[];
    const int T = blockDim.x, t = threadIdx.x;
    LList<X> L;
    L.x0 = reinterpret_cast<X *>(lds_raw) + t;
    L.x2 = reinterpret_cast<X *>(lds_raw) + (size_t)T * lcap + t;
    L.end = reinterpret_cast<uint16_t *>(lds_raw + (size_t)2 * T * lcap * sizeof(X)) + t;
    L.stride = T;
    L.cap = lcap;
    FM<X> fm;
    fm.occ = ix.occ;
    fm.l2_0 = (X)ix.L2[0]; fm.l2_1 = (X)ix.L2[1]; fm.l2_2 = (X)ix.L2[2]; fm.l2_3 = (X)ix.L2[3]; fm.l2_4 = (X)ix.L2[4];
    fm.primary = (X)ix.primary;
    uint64_t nblk = 0;
    const int li = blockIdx.x * T + t;
    if (li < n) {
        const uint8_t *q = codes + offs[li];
        const int len = (int)(offs[li + 1] - offs[li]);
        bool ovf = false;
        OutSlot S{intv_out + (size_t)li * cp.intv, 0, cp.intv, 0};
        const int split_len = (int)(o.min_seed_len * o.split_factor + .499);
        auto take_mem1 = [&](bool pass2) {
            // mem1 (reversed emission order) sits at S.a[cap-n1 .. cap); filter-append in order
            for (int k = 0; k < S.n1; ++k) {
                Intv m = S.a[S.cap - S.n1 + k];
                uint32_t st = (uint32_t)(m.info >> 32), en = (uint32_t)m.info;
                bool keep = pass2 ? (uint64_t)(en - st) >= (uint64_t)o.min_seed_len : (int)(en - st) >= o.min_seed_len;
                if (keep) S.a[S.n++] = m;
            }
            S.n1 = 0;
        };
        int x = 0;
        while (x < len && !ovf) {
            if (q[x] < 4) {
                x = smem1_lds(fm, len, q, x, 1, L, S, ovf, nblk);
                if (!ovf) take_mem1(false);
            } else ++x;
        }
        const int old_n = S.n;
        for (int k = 0; k < old_n && !ovf; ++k) {
            const Intv p = S.a[k];
            const int start = (int)(p.info >> 32), end = (int)(uint32_t)p.info;
            if (end - start < split_len || p.x[2] > (uint64_t)o.split_width) continue;
            smem1_lds(fm, len, q, (start + end) >> 1, (int)p.x[2] + 1, L, S, ovf, nblk);
            if (!ovf) take_mem1(true);
        }
        if (o.max_mem_intv > 0) {
            x = 0;
            while (x < len && !ovf) {
                if (q[x] < 4) {
                    Intv m;
                    x = seed_strategy1_x(fm, len, q, x, o.min_seed_len, o.max_mem_intv, m, nblk);
                    if (m.x[2] > 0) {
                        if (S.n >= S.cap) { ovf = true; break; }
                        S.a[S.n++] = m;
                    }
                } else ++x;
            }
        }
        if (ovf) {
            status[li] |= ST_OVERFLOW;
            n_intv[li] = 0;
        } else {
            for (int i = 1; i < S.n; ++i) {   // equal keys are identical intervals: any correct sort is exact
                Intv tv = S.a[i];
                int j = i;
                while (j > 0 && tv.info < S.a[j - 1].info) { S.a[j] = S.a[j - 1]; --j; }
                S.a[j] = tv;
            }
            n_intv[li] = S.n;
        }
    }
    wave_add2(&ctr[STG_SMEM].occ_blocks, nblk);
}

// LDS bytes per thread for `lcap` list entries
template <typename X>
static size_t lds_bytes(int threads, int lcap) { return (size_t)threads * lcap * (2 * sizeof(X) + 2); }

hipError_t launch_smem_lds(hipStream_t st, const DIndex &ix, const DOpts &o, const Caps &cp, const uint8_t *codes,
                           const int64_t *offs, int n, Intv *intv, int32_t *n_intv, uint32_t *status, Counters *ctr,
                           int lcap)
{
    const int T = 256;
    const int grid = (n + T - 1) / T;
    if (grid == 0) return hipSuccess;
    if (ix.seq_len < 0xFFFFFFFFull) {
        size_t sh = lds_bytes<uint32_t>(T, lcap);
        hipLaunchKernelGGL(k_smem_lds<uint32_t>, dim3(grid), dim3(T), sh, st, ix, o, cp, codes, offs, n, intv, n_intv,
                           status, ctr, lcap);
    } else {
        size_t sh = lds_bytes<uint64_t>(T, lcap);
        hipLaunchKernelGGL(k_smem_lds<uint64_t>, dim3(grid), dim3(T), sh, st, ix, o, cp, codes, offs, n, intv, n_intv,
                           status, ctr, lcap);
    }
    return hipGetLastError();
}

}  // namespace bsq
