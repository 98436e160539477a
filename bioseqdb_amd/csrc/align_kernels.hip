// align_kernels.hip -- HIP (gfx950) kernels of the BWA-MEM alignment path behind bioseqdb's
// nuclseq_search_bwa / nuclseq_multi_search_bwa (reference: bioseqdb/bwa.cpp:141-181, which calls
// libbwa mem_align1 + mem_reg2aln).  The libbwa algorithm is re-expressed as five stage kernels over
// device-resident index data; results must equal libbwa's bit for bit (checked against oracle/).
//
//   k_smem     mem_collect_intv   (bwt_smem1 x2 passes + bwt_seed_strategy1, sorted by info)
//   k_chain    mem_chain + mem_chain_flt (SA lookups, kbtree with t = 5, klib introsort by weight)
//   k_extend   mem_chain2aln (ksw_extend2) + mem_sort_dedup_patch (ksw_global2) + mem_mark_primary_se
//   k_reg2aln  mem_reg2aln (infer_bw, bwa_gen_cigar2 / ksw_global2 traceback, clipping)
//   k_pack     compaction of per-read slots into the bsq_hits layout
//
// Round-1 mapping: one read per lane (inter-task parallelism) with private scratch in HBM;
// reads that overflow the small per-read slots are re-run by the host with large capacities.
// Restates algorithms of BWA (lh3/bwa, Apache-2.0) and klib (MIT) for bit-exact results; see NOTICE.
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <algorithm>
#include <stdint.h>

#include "bsq_device.h"
#include "dev_common.h"
#include "../../include/bsq.h"
#include "bsq_internal.h"

namespace bsq {

#define DEV __device__ __forceinline__
#define DEVN __device__ __noinline__

// ------------------------------------------------------------------------------------------------
// FM index: rank over the $-removed BWT (same function as libbwa bwt_occ4)
// ------------------------------------------------------------------------------------------------
DEV void occ_block(const OccBlock *blk, uint32_t r, uint64_t c[4])
{
    // counts of each base in the first r (1..128) rows of the block, added to the block prefix
    const uint4 *p = reinterpret_cast<const uint4 *>(blk);
    uint4 w0 = p[0], w1 = p[1], w2 = p[2], w3 = p[3];
    uint64_t c0 = (uint64_t)w0.y << 32 | w0.x, c1 = (uint64_t)w0.w << 32 | w0.z;
    uint64_t c2 = (uint64_t)w1.y << 32 | w1.x, c3 = (uint64_t)w1.w << 32 | w1.z;
    uint64_t h0 = (uint64_t)w2.y << 32 | w2.x, h1 = (uint64_t)w2.w << 32 | w2.z;
    uint64_t l0 = (uint64_t)w3.y << 32 | w3.x, l1 = (uint64_t)w3.w << 32 | w3.z;
    uint64_t m0 = r >= 64 ? ~0ull : ((1ull << r) - 1);
    uint64_t m1 = r >= 128 ? ~0ull : (r > 64 ? ((1ull << (r - 64)) - 1) : 0ull);
    uint32_t n3 = __popcll(h0 & l0 & m0) + __popcll(h1 & l1 & m1);
    uint32_t n2 = __popcll(h0 & ~l0 & m0) + __popcll(h1 & ~l1 & m1);
    uint32_t n1 = __popcll(~h0 & l0 & m0) + __popcll(~h1 & l1 & m1);
    c[0] = c0 + (r - n1 - n2 - n3);
    c[1] = c1 + n1;
    c[2] = c2 + n2;
    c[3] = c3 + n3;
}

DEV void occ4(const DIndex &ix, uint64_t k, uint64_t c[4])
{
    if (k == (uint64_t)-1) { c[0] = c[1] = c[2] = c[3] = 0; return; }
    k -= (k >= ix.primary);
    occ_block(ix.occ + (k >> 7), (uint32_t)(k & 127) + 1, c);
}

// bwt_extend: both ranks (bwt_2occ4), one or two 64-B block fetches
DEV void bwt_extend(const DIndex &ix, const Intv &ik, Intv ok[4], int is_back, uint64_t &nblk)
{
    uint64_t tk[4], tl[4];
    const int nb = !is_back;
    uint64_t k = ik.x[nb] - 1, l = ik.x[nb] - 1 + ik.x[2];
    occ4(ix, k, tk);
    occ4(ix, l, tl);
    {
        uint64_t kk = k == (uint64_t)-1 ? k : k - (k >= ix.primary), ll = l - (l >= ix.primary);
        nblk += (k == (uint64_t)-1 || (kk >> 7) == (ll >> 7)) ? 2 : 4;   // 32-B units
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        ok[i].x[nb] = ix.L2[i] + 1 + tk[i];
        ok[i].x[2] = tl[i] - tk[i];
    }
    const int b = is_back;
    ok[3].x[b] = ik.x[b] + (ik.x[nb] <= ix.primary && ik.x[nb] + ik.x[2] - 1 >= ix.primary);
    ok[2].x[b] = ok[3].x[b] + ok[3].x[2];
    ok[1].x[b] = ok[2].x[b] + ok[2].x[2];
    ok[0].x[b] = ok[1].x[b] + ok[1].x[2];
}

DEV void set_intv(const DIndex &ix, int c, Intv &ik)
{
    ik.x[0] = ix.L2[c] + 1;
    ik.x[2] = ix.L2[c + 1] - ix.L2[c];
    ik.x[1] = ix.L2[3 - c] + 1;
    ik.info = 0;
}

DEV uint64_t sa_at(const DIndex &ix, uint64_t row) { return ix.sa32 ? (uint64_t)ix.sa32[row] : ix.sa64[row]; }

// ------------------------------------------------------------------------------------------------
// bounded vectors in private scratch
// ------------------------------------------------------------------------------------------------
template <class P>
struct IVT {
    P a;
    int n, cap;
    DEV bool push(const Intv &v, bool &ovf)
    {
        if (n >= cap) { ovf = true; return false; }
        a[n++] = v;
        return true;
    }
    DEV void reverse()
    {
        for (int j = 0; j < (n >> 1); ++j) { Intv t = a[n - 1 - j]; a[n - 1 - j] = a[j]; a[j] = t; }
    }
};
using IV = IVT<Intv *>;

// bwt_smem1a with max_intv = 0 (bwt_smem1)
DEVN int smem1(const DIndex &ix, int len, const uint8_t *q, int x, int min_intv, IV &mem, IV &va, IV &vb,
               bool &ovf, uint64_t &nblk)
{
    mem.n = 0;
    if (q[x] > 3) return x + 1;
    if (min_intv < 1) min_intv = 1;
    IV *prev = &va, *curr = &vb;
    Intv ik, ok[4];
    set_intv(ix, q[x], ik);
    ik.info = (uint64_t)(x + 1);
    int i;
    curr->n = 0;
    for (i = x + 1; i < len; ++i) {
        int qi = q[i];
        if (qi < 4) {
            int c = 3 - qi;
            bwt_extend(ix, ik, ok, 0, nblk);
            if (ok[c].x[2] != ik.x[2]) {
                if (!curr->push(ik, ovf)) return len;
                if (ok[c].x[2] < (uint64_t)min_intv) break;
            }
            ik = ok[c];
            ik.info = (uint64_t)(i + 1);
        } else {
            if (!curr->push(ik, ovf)) return len;
            break;
        }
    }
    if (i == len && !curr->push(ik, ovf)) return len;
    curr->reverse();
    int ret = (int)curr->a[0].info;
    { IV *t = curr; curr = prev; prev = t; }
    for (i = x - 1; i >= -1; --i) {
        int c = i < 0 ? -1 : (q[i] < 4 ? q[i] : -1);
        curr->n = 0;
        for (int j = 0; j < prev->n; ++j) {
            Intv p = prev->a[j];
            bool keep_hit;
            if (c >= 0) {
                bwt_extend(ix, p, ok, 1, nblk);
                keep_hit = ok[c].x[2] < (uint64_t)min_intv;
            } else keep_hit = true;
            if (keep_hit) {
                if (curr->n == 0) {
                    if (mem.n == 0 || (uint64_t)(i + 1) < (mem.a[mem.n - 1].info >> 32)) {
                        p.info |= (uint64_t)(i + 1) << 32;
                        if (!mem.push(p, ovf)) return len;
                    }
                }
            } else if (curr->n == 0 || ok[c].x[2] != curr->a[curr->n - 1].x[2]) {
                Intv t = ok[c];
                t.info = p.info;
                if (!curr->push(t, ovf)) return len;
            }
        }
        if (curr->n == 0) break;
        { IV *t = curr; curr = prev; prev = t; }
    }
    mem.reverse();
    return ret;
}

DEV int seed_strategy1(const DIndex &ix, int len, const uint8_t *q, int x, int min_len, int max_intv, Intv &mem,
                       uint64_t &nblk)
{
    Intv ik, ok[4];
    mem.x[0] = mem.x[1] = mem.x[2] = mem.info = 0;
    if (q[x] > 3) return x + 1;
    set_intv(ix, q[x], ik);
    for (int i = x + 1; i < len; ++i) {
        int qi = q[i];
        if (qi < 4) {
            int c = 3 - qi;
            bwt_extend(ix, ik, ok, 0, nblk);
            if (ok[c].x[2] < (uint64_t)max_intv && i - x >= min_len) {
                mem = ok[c];
                mem.info = (uint64_t)x << 32 | (uint64_t)(i + 1);
                return i + 1;
            }
            ik = ok[c];
        } else return i + 1;
    }
    return len;
}

// ------------------------------------------------------------------------------------------------
// k_smem: mem_collect_intv per read
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_smem(DIndex ix, DOpts o, Caps cp, const uint8_t *codes,
                                              const int64_t *offs, const int32_t *sel, int n, Intv *intv_out,
                                              int32_t *n_intv, uint32_t *status, uint8_t *scratch,
                                              Counters *ctr)
{
    const int nthr = gridDim.x * blockDim.x;
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t nblk = 0;
    const int vcap = cp.max_len + 2;
    Intv *sbase = reinterpret_cast<Intv *>(scratch + (size_t)tid * cp.scratch);
    for (int li = tid; li < n; li += nthr) {
        const int r = read_of(sel, li);
        const uint8_t *q = codes + offs[r];
        const int len = (int)(offs[r + 1] - offs[r]);
        bool ovf = false;
        IVT<SP<Intv>> mem{SP<Intv>{intv_out + intv_slot_at_d(li, 0, cp.intv)}, 0, cp.intv};
        IV mem1{sbase, 0, vcap}, va{sbase + vcap, 0, vcap}, vb{sbase + 2 * vcap, 0, vcap};
        const int split_len = (int)(o.min_seed_len * o.split_factor + .499);
        int x = 0;
        // pass 1: SMEMs
        while (x < len && !ovf) {
            if (q[x] < 4) {
                x = smem1(ix, len, q, x, 1, mem1, va, vb, ovf, nblk);
                for (int i = 0; i < mem1.n && !ovf; ++i) {
                    const Intv &p = mem1.a[i];
                    int slen = (int)((uint32_t)p.info - (uint32_t)(p.info >> 32));
                    if (slen >= o.min_seed_len) mem.push(p, ovf);
                }
            } else ++x;
        }
        // pass 2: re-seed inside long SMEMs with few occurrences
        const int old_n = mem.n;
        for (int k = 0; k < old_n && !ovf; ++k) {
            Intv p = mem.a[k];
            int start = (int)(p.info >> 32), end = (int)(int32_t)p.info;
            if (end - start < split_len || p.x[2] > (uint64_t)o.split_width) continue;
            smem1(ix, len, q, (start + end) >> 1, (int)p.x[2] + 1, mem1, va, vb, ovf, nblk);
            for (int i = 0; i < mem1.n && !ovf; ++i)
                if ((uint32_t)mem1.a[i].info - (mem1.a[i].info >> 32) >= (uint64_t)o.min_seed_len) mem.push(mem1.a[i], ovf);
        }
        // pass 3: LAST-like seeds
        if (o.max_mem_intv > 0) {
            x = 0;
            while (x < len && !ovf) {
                if (q[x] < 4) {
                    Intv m;
                    x = seed_strategy1(ix, len, q, x, o.min_seed_len, o.max_mem_intv, m, nblk);
                    if (m.x[2] > 0) mem.push(m, ovf);
                } else ++x;
            }
        }
        if (ovf) {
            status[li] |= ST_OVERFLOW;
            n_intv[li] = 0;
            continue;
        }
        // sort by info (equal keys are identical intervals, so any order-correct sort is exact)
        for (int i = 1; i < mem.n; ++i) {
            Intv t = mem.a[i];
            int j = i;
            while (j > 0 && t.info < mem.a[j - 1].info) { mem.a[j] = mem.a[j - 1]; --j; }
            mem.a[j] = t;
        }
        n_intv[li] = mem.n;
    }
    wave_add(&ctr[STG_SMEM].occ_blocks, nblk);
}

// ------------------------------------------------------------------------------------------------
// klib ks_introsort (ksort.h) over an index array; lt(x, y) compares element ids.  The pivot,
// partition and final insertion sort follow klib exactly, so ties land where libbwa puts them.
// ------------------------------------------------------------------------------------------------
template <class A, class LT>
DEV void ks_insertsort(A a, int n, LT lt)
{
    for (int i = 1; i < n; ++i)
        for (int j = i; j > 0 && lt(a[j], a[j - 1]); --j) { int t = a[j]; a[j] = a[j - 1]; a[j - 1] = t; }
}

template <class A, class LT>
DEV void ks_combsort(A a, int n, LT lt)
{
    const double shrink_factor = 1.2473309501039786540366528676643;
    int do_swap;
    size_t gap = (size_t)n;
    do {
        if (gap > 2) {
            gap = (size_t)(gap / shrink_factor);
            if (gap == 9 || gap == 10) gap = 11;
        }
        do_swap = 0;
        for (int i = 0; i < n - (int)gap; ++i) {
            int j = i + (int)gap;
            if (lt(a[j], a[i])) { int t = a[i]; a[i] = a[j]; a[j] = t; do_swap = 1; }
        }
    } while (do_swap || gap > 2);
    if (gap != 1) ks_insertsort(a, n, lt);
}

// stk: 3 x 64 ints of the thread's global scratch (the partition stack, touched only by partitions of more
// than 16 elements): a private array here would give every wave of the kernel a scratch segment
// Returns the number of partition scans that reached the bound `i == t` while `lt(a[t], rp)` still held, i.e.
// scans that klib's sentinel would NOT have stopped (the runaway the round-2 hang would need).  With strict
// comparators the sentinel a[t] == rp is never swapped, so this is 0; the kernels add it to Counters::sort_guard
// and the tests and bench assert 0 (a non-zero count names the read to start a root cause from).
template <class A, class LT, class S>
DEV int ks_introsort(A a, int n, LT lt, S stk)
{
    int guard = 0;
    if (n < 1) return 0;
    if (n == 2) {
        if (lt(a[1], a[0])) { int t = a[0]; a[0] = a[1]; a[1] = t; }
        return 0;
    }
    int d;
    for (d = 2; (1ul << d) < (unsigned long)n; ++d);
    S stk_l = stk, stk_r = stk + 64, stk_d = stk + 128;
    int top = 0;
    int s = 0, t = n - 1;
    d <<= 1;
    while (1) {
        if (s < t) {
            if (--d == 0) {
                ks_combsort(a + s, t - s + 1, lt);
                t = s;
                continue;
            }
            int i = s, j = t, k = i + ((j - i) >> 1) + 1;
            if (lt(a[k], a[i])) {
                if (lt(a[k], a[j])) k = j;
            } else k = lt(a[j], a[i]) ? i : j;
            int rp = a[k];
            if (k != t) { int x = a[k]; a[k] = a[t]; a[t] = x; }
            for (;;) {
                // a[t] == rp is klib's sentinel (lt(rp, rp) is false), so `i < t` never changes where the scan
                // stops; the explicit bound keeps the compiler from miscompiling this loop when `a` is a
                // lane-interleaved index array (k_extend with S = 64 scratch hung deterministically on an unbounded
                // scan and never with S = 1; with the bound both are exact)
#ifdef BSQ_INTROSORT_UNBOUNDED   // tools/hang_isa.sh only: klib's scan exactly as written (sentinel a[t] == rp)
                do ++i; while (lt(a[i], rp));
#else
                do ++i; while (i < t && lt(a[i], rp));
                if (i == t && lt(a[t], rp)) ++guard;   // stopped by the bound, not by the sentinel
#endif
                do --j; while (i <= j && lt(rp, a[j]));
                if (j <= i) break;
                int x = a[i]; a[i] = a[j]; a[j] = x;
            }
            { int x = a[i]; a[i] = a[t]; a[t] = x; }
            if (i - s > t - i) {
                if (i - s > 16) { stk_l[top] = s; stk_r[top] = i - 1; stk_d[top] = d; ++top; }
                s = t - i > 16 ? i + 1 : t;
            } else {
                if (t - i > 16) { stk_l[top] = i + 1; stk_r[top] = t; stk_d[top] = d; ++top; }
                t = i - s > 16 ? i - 1 : s;
            }
        } else {
            if (top == 0) { ks_insertsort(a, n, lt); return guard; }
            --top; s = stk_l[top]; t = stk_r[top]; d = stk_d[top];
        }
    }
}

// ------------------------------------------------------------------------------------------------
// k_chain: mem_chain (kbtree t = 5, KB_DEFAULT_SIZE 512) + mem_chain_flt
// ------------------------------------------------------------------------------------------------
// The chaining state is lane-private but lives in global scratch.  Element i of a lane's array sits at
// [i * 64 + lane] of its wave's region (SP below), so when the lanes of a wave touch the same element
// index the accesses fall on adjacent addresses instead of 64 separate per-lane areas.
struct SeedNode { int64_t rbeg; int32_t qbeg, len, next, pad; };
struct ChainNode { int64_t pos; int32_t rid, n, head, tail, w, kept, first, pad; };
struct KNode { int32_t n, is_internal; int32_t key[9]; int32_t ptr[10]; };
#define KB_T 5

template <int S>
struct ChainCtx {
    SP<SeedNode, S> seeds; int n_seeds, cap_seeds;
    SP<ChainNode, S> ch; int n_ch, cap_ch;
    SP<KNode, S> nodes; int n_nodes, cap_nodes;
    int root, n_keys;
    bool ovf;
};

template <int S>
DEV int kb_getp_aux(const ChainCtx<S> &C, const KNode &x, int64_t kpos, int *r)
{
    int tr, *rr = r ? r : &tr, begin = 0, end = x.n;
    if (x.n == 0) return -1;
    while (begin < end) {
        int mid = (begin + end) >> 1;
        if (C.ch[x.key[mid]].pos < kpos) begin = mid + 1;
        else end = mid;
    }
    if (begin == x.n) { *rr = 1; return x.n - 1; }
    int64_t bp = C.ch[x.key[begin]].pos;
    if ((*rr = (bp < kpos) - (kpos < bp)) < 0) --begin;
    return begin;
}

template <int S>
DEV int kb_intervalp_lower(const ChainCtx<S> &C, int64_t kpos)
{
    int i, r = 0, x = C.root, lower = -1;
    while (x >= 0) {
        const KNode &nd = C.nodes[x];
        i = kb_getp_aux(C, nd, kpos, &r);
        if (i >= 0 && r == 0) return nd.key[i];
        if (i >= 0) lower = nd.key[i];
        if (nd.is_internal == 0) return lower;
        x = nd.ptr[i + 1];
    }
    return lower;
}

template <int S>
DEV int kb_new_node(ChainCtx<S> &C)
{
    if (C.n_nodes >= C.cap_nodes) { C.ovf = true; return -1; }
    KNode &z = C.nodes[C.n_nodes];
    z.n = 0; z.is_internal = 0;
    return C.n_nodes++;
}

template <int S>
DEV bool kb_split(ChainCtx<S> &C, int xi, int i, int yi)
{
    int zi = kb_new_node(C);
    if (zi < 0) return false;
    KNode &x = C.nodes[xi], &y = C.nodes[yi], &z = C.nodes[zi];
    z.is_internal = y.is_internal;
    z.n = KB_T - 1;
    for (int j = 0; j < KB_T - 1; ++j) z.key[j] = y.key[KB_T + j];
    if (y.is_internal) for (int j = 0; j < KB_T; ++j) z.ptr[j] = y.ptr[KB_T + j];
    y.n = KB_T - 1;
    for (int j = x.n; j >= i + 1; --j) x.ptr[j + 1] = x.ptr[j];
    x.ptr[i + 1] = zi;
    for (int j = x.n - 1; j >= i; --j) x.key[j + 1] = x.key[j];
    x.key[i] = y.key[KB_T - 1];
    ++x.n;
    return true;
}

template <int S>
DEV void kb_putp(ChainCtx<S> &C, int key)
{
    ++C.n_keys;
    int r = C.root;
    if (C.nodes[r].n == 2 * KB_T - 1) {
        int s = kb_new_node(C);
        if (s < 0) return;
        C.root = s;
        C.nodes[s].is_internal = 1; C.nodes[s].n = 0;
        C.nodes[s].ptr[0] = r;
        if (!kb_split(C, s, 0, r)) return;
        r = s;
    }
    const int64_t kpos = C.ch[key].pos;
    for (;;) {
        KNode &x = C.nodes[r];
        if (x.is_internal == 0) {
            int i = kb_getp_aux(C, x, kpos, 0);
            for (int j = x.n - 1; j >= i + 1; --j) x.key[j + 1] = x.key[j];
            x.key[i + 1] = key;
            ++x.n;
            return;
        }
        int i = kb_getp_aux(C, x, kpos, 0) + 1;
        if (C.nodes[x.ptr[i]].n == 2 * KB_T - 1) {
            if (!kb_split(C, r, i, x.ptr[i])) return;
            int64_t kp = C.ch[C.nodes[r].key[i]].pos;
            if (((kp < kpos) - (kpos < kp)) > 0) ++i;
        }
        r = C.nodes[r].ptr[i];
    }
}

template <int S>
DEV bool test_and_merge(ChainCtx<S> &C, const DOpts &o, int64_t l_pac, int ci, const SeedNode &p, int seed_rid)
{
    ChainNode &c = C.ch[ci];
    const SeedNode &first = C.seeds[c.head], &last = C.seeds[c.tail];
    int64_t qend = last.qbeg + last.len, rend = last.rbeg + last.len;
    if (seed_rid != c.rid) return false;
    if (p.qbeg >= first.qbeg && p.qbeg + p.len <= qend && p.rbeg >= first.rbeg && p.rbeg + p.len <= rend) return true;
    if ((last.rbeg < l_pac || first.rbeg < l_pac) && p.rbeg >= l_pac) return false;
    int64_t x = p.qbeg - last.qbeg, y = p.rbeg - last.rbeg;
    if (y >= 0 && x - y <= o.w && y - x <= o.w && x - last.len < o.max_chain_gap && y - last.len < o.max_chain_gap) {
        if (C.n_seeds >= C.cap_seeds) { C.ovf = true; return true; }
        int si = C.n_seeds++;
        C.seeds[si] = p;
        C.seeds[si].next = -1;
        C.seeds[c.tail].next = si;
        c.tail = si;
        ++c.n;
        return true;
    }
    return false;
}

template <int S>
DEV int chain_weight(const ChainCtx<S> &C, const ChainNode &c)
{
    int64_t end = 0;
    int w = 0, tmp;
    for (int s = c.head; s >= 0; s = C.seeds[s].next) {
        const SeedNode &sd = C.seeds[s];
        if (sd.qbeg >= end) w += sd.len;
        else if (sd.qbeg + sd.len > end) w += (int)(sd.qbeg + sd.len - end);
        end = end > sd.qbeg + sd.len ? end : sd.qbeg + sd.len;
    }
    tmp = w; w = 0; end = 0;
    for (int s = c.head; s >= 0; s = C.seeds[s].next) {
        const SeedNode &sd = C.seeds[s];
        if (sd.rbeg >= end) w += sd.len;
        else if (sd.rbeg + sd.len > end) w += (int)(sd.rbeg + sd.len - end);
        end = end > sd.rbeg + sd.len ? end : sd.rbeg + sd.len;
    }
    w = w < tmp ? w : tmp;
    return w < (1 << 30) ? w : (1 << 30) - 1;
}

template <int S>
__global__ void __launch_bounds__(256) k_chain(DIndex ix, DOpts o, Caps cp, const int64_t *offs, const int32_t *sel,
                                               int n, const Intv *intv, const int32_t *n_intv, ChainDesc *chains_out,
                                               Seed *seeds_out, int32_t *n_chains, uint32_t *status,
                                               uint8_t *scratch, Counters *ctr, int only_marked)
{
    const int nthr = gridDim.x * blockDim.x;
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t nsa = 0;
    int guard = 0;
    // S = 64: this wave's 64 * cp.scratch bytes, each array lane-interleaved (SP); the workspace holds whole
    // waves.  S = 1 (retry workspaces): the thread's own cp.scratch bytes, arrays contiguous.
    const int lane = S == 1 ? 0 : (tid & 63);
    uint8_t *wb = scratch + (S == 1 ? (size_t)tid : (size_t)(tid >> 6) * 64) * (size_t)cp.scratch;
    ChainCtx<S> C;
    C.cap_seeds = cp.seeds;
    C.cap_ch = cp.chains;
    C.cap_nodes = cp.chains / 2 + 8;
    size_t off = 0;
    C.seeds = SP<SeedNode, S>{reinterpret_cast<SeedNode *>(wb) + lane};
    off += (size_t)C.cap_seeds * S * sizeof(SeedNode);
    C.ch = SP<ChainNode, S>{reinterpret_cast<ChainNode *>(wb + off) + lane};
    off += (size_t)C.cap_ch * S * sizeof(ChainNode);
    C.nodes = SP<KNode, S>{reinterpret_cast<KNode *>(wb + off) + lane};
    off += (size_t)C.cap_nodes * S * sizeof(KNode);
    SP<int, S> ord{reinterpret_cast<int *>(wb + off) + lane};
    SP<int, S> kept_list = ord + cp.chains;
    SP<int, S> stk = kept_list + cp.chains;   // introsort stack (192 ints), then the B-tree walk's (3 x 24)
    for (int li = tid; li < n; li += nthr) {
        if (only_marked && n_chains[li] != -1) continue;   // second launch after k_chain_s: the reads it left
        n_chains[li] = 0;
        if (status[li]) continue;
        const int r = read_of(sel, li);
        const int len = (int)(offs[r + 1] - offs[r]);
        if (len < o.min_seed_len) continue;
        C.n_seeds = 0; C.n_ch = 0; C.n_nodes = 0; C.n_keys = 0; C.ovf = false;
        C.root = kb_new_node(C);
        const SP<const Intv> mem{intv + intv_slot_at_d(li, 0, cp.intv)};
        const int nm = n_intv[li];
        for (int i = 0; i < nm && !C.ovf; ++i) {
            const Intv p = mem[i];
            const int slen = (int)((uint32_t)p.info - (uint32_t)(p.info >> 32));
            const int step = p.x[2] > (uint64_t)o.max_occ ? (int)(p.x[2] / (uint64_t)o.max_occ) : 1;
            int count = 0;
            for (int64_t k = 0; (uint64_t)k < p.x[2] && count < o.max_occ && !C.ovf; k += step, ++count) {
                SeedNode s;
                s.rbeg = (int64_t)sa_at(ix, p.x[0] + (uint64_t)k);
                ++nsa;
                s.qbeg = (int32_t)(p.info >> 32);
                s.len = slen;
                s.next = -1;
                const int rid = intv2rid(ix, s.rbeg, s.rbeg + s.len);
                if (rid < 0) continue;
                bool to_add = false;
                if (C.n_keys) {
                    int lower = kb_intervalp_lower(C, s.rbeg);
                    if (lower < 0 || !test_and_merge(C, o, ix.l_pac, lower, s, rid)) to_add = true;
                } else to_add = true;
                if (to_add) {
                    if (C.n_ch >= C.cap_ch || C.n_seeds >= C.cap_seeds) { C.ovf = true; break; }
                    int si = C.n_seeds++;
                    C.seeds[si] = s;
                    int ci = C.n_ch++;
                    ChainNode &c = C.ch[ci];
                    c.pos = s.rbeg; c.rid = rid; c.n = 1; c.head = c.tail = si; c.w = 0; c.kept = 0; c.first = -1;
                    kb_putp(C, ci);
                }
            }
        }
        if (C.ovf) { status[li] |= ST_OVERFLOW; continue; }
        // in-order traversal of the B-tree -> chain order
        int nord = 0;
        {   // iterative in-order walk == kbtree's __kb_traverse
            SP<int, S> stn = stk + 192, sti = stn + 24, std_ = sti + 24;
            int sp = 0;
            stn[0] = C.root; sti[0] = 0; std_[0] = 0;
            if (!C.nodes[C.root].is_internal) {   // a lone leaf root (<= 9 chains, the common case): its keys
                const KNode &nd = C.nodes[C.root];
                for (int i = 0; i < nd.n; ++i) ord[nord++] = nd.key[i];
                sp = -1;
            }
            while (sp >= 0) {
                const KNode &nd = C.nodes[stn[sp]];
                const int i = sti[sp];
                if (i > nd.n) { --sp; continue; }
                if (nd.is_internal && !std_[sp]) {      // descend into child i first
                    std_[sp] = 1;
                    ++sp; stn[sp] = nd.ptr[i]; sti[sp] = 0; std_[sp] = 0;
                    continue;
                }
                if (i < nd.n) ord[nord++] = nd.key[i];
                sti[sp] = i + 1; std_[sp] = 0;
            }
        }
        // mem_chain_flt
        int n_chn = 0;
        for (int i = 0; i < nord; ++i) {
            ChainNode &c = C.ch[ord[i]];
            c.first = -1; c.kept = 0;
            c.w = chain_weight(C, c);
            if (c.w >= o.min_chain_weight) ord[n_chn++] = ord[i];
        }
        if (n_chn > 0) {
            const SP<ChainNode, S> ch = C.ch;
            guard += ks_introsort(ord, n_chn, [ch](int a, int b) { return ch[a].w > ch[b].w; }, stk);
            ch[ord[0]].kept = 3;
            int nk = 0;
            kept_list[nk++] = 0;
            for (int i = 1; i < n_chn; ++i) {
                int large_ovlp = 0, k;
                ChainNode &ci = ch[ord[i]];
                const int bi = C.seeds[ci.head].qbeg, ei = C.seeds[ci.tail].qbeg + C.seeds[ci.tail].len;
                for (k = 0; k < nk; ++k) {
                    int j = kept_list[k];
                    ChainNode &cj = ch[ord[j]];
                    const int bj = C.seeds[cj.head].qbeg, ej = C.seeds[cj.tail].qbeg + C.seeds[cj.tail].len;
                    int b_max = bj > bi ? bj : bi;
                    int e_min = ej < ei ? ej : ei;
                    if (e_min > b_max) {   // is_alt is always 0 on this path
                        int li2 = ei - bi, lj = ej - bj;
                        int min_l = li2 < lj ? li2 : lj;
                        if (e_min - b_max >= min_l * o.mask_level && min_l < o.max_chain_gap) {
                            large_ovlp = 1;
                            if (cj.first < 0) cj.first = i;
                            if (ci.w < cj.w * o.drop_ratio && cj.w - ci.w >= o.min_seed_len << 1) break;
                        }
                    }
                }
                if (k == nk) {
                    kept_list[nk++] = i;
                    ci.kept = large_ovlp ? 2 : 3;
                }
            }
            for (int i = 0; i < nk; ++i) {
                ChainNode &c = ch[ord[kept_list[i]]];
                if (c.first >= 0) ch[ord[c.first]].kept = 1;
            }
            int i, k;
            for (i = k = 0; i < n_chn; ++i) {
                if (ch[ord[i]].kept == 0 || ch[ord[i]].kept == 3) continue;
                if (++k >= o.max_chain_extend) break;
            }
            for (; i < n_chn; ++i)
                if (ch[ord[i]].kept < 3) ch[ord[i]].kept = 0;
            // write kept chains with contiguous seeds
            ChainDesc *cd = chains_out + (size_t)li * cp.chains;
            Seed *so = seeds_out + (size_t)li * cp.seeds;
            int nc = 0, ns = 0;
            for (i = 0; i < n_chn; ++i) {
                const ChainNode &c = ch[ord[i]];
                if (c.kept == 0) continue;
                cd[nc].seed_off = ns; cd[nc].n = c.n; cd[nc].rid = c.rid; cd[nc].w = c.w;
                for (int s = c.head; s >= 0; s = C.seeds[s].next) {
                    so[ns].rbeg = C.seeds[s].rbeg; so[ns].qbeg = C.seeds[s].qbeg; so[ns].len = C.seeds[s].len;
                    ++ns;
                }
                ++nc;
            }
            n_chains[li] = nc;
        }
    }
    wave_add(&ctr[STG_CHAIN].sa_values, nsa);
    wave_add(&ctr[STG_CHAIN].sort_guard, (unsigned long long)guard);
}

// ------------------------------------------------------------------------------------------------
// k_chain_s: mem_chain + mem_chain_flt for the reads whose chaining state fits a small LDS share: at most CS_NS
// seeds and CS_NC chains, i.e. a kbtree that never grows past its root leaf (the 10th key splits it).  The state
// lives in LDS, lane-interleaved (one-wave blocks), instead of k_chain's global scratch, so the tree operations
// and the chain filter cost LDS round trips and no memory traffic; the intervals of four MEMs and their first SA
// values are loaded together (one round trip each instead of one per MEM).  On the root leaf kbtree reduces to a
// sorted key array: kb_intervalp_lower returns the first key whose pos equals the probe, else the last one below
// it; kb_putp inserts after the first key not below the probe (after the first equal one).  A read that outgrows
// the share is marked (n_chains = -1) and chained from scratch by k_chain<64>'s second launch (launch_chain).
// ------------------------------------------------------------------------------------------------
constexpr int CS_NS = 12, CS_NC = 2 * KB_T - 1;
extern __shared__ uint8_t g_lds_cs[];

struct CsLds {   // element e of lane l of an array of element size z: base + (e * 64 + l) * z
    static constexpr int RB = 0;                      // i64 seed rbeg
    static constexpr int QL = RB + CS_NS * 64 * 8;    // u32 seed qbeg | len << 16
    static constexpr int NX = QL + CS_NS * 64 * 4;    // u8 seed next (0xff: last)
    static constexpr int CW = NX + CS_NS * 64;        // i32 chain w
    static constexpr int CR = CW + CS_NC * 64 * 4;    // i32 chain rid
    static constexpr int CH = CR + CS_NC * 64 * 4;    // u8 chain head, tail, n, kept, first (i8), then the leaf's
    static constexpr int CT = CH + CS_NC * 64;        // keys, ord and the kept list
    static constexpr int CN = CT + CS_NC * 64;
    static constexpr int CK = CN + CS_NC * 64;
    static constexpr int CF = CK + CS_NC * 64;
    static constexpr int LF = CF + CS_NC * 64;
    static constexpr int OR = LF + CS_NC * 64;
    static constexpr int KL = OR + CS_NC * 64;
    static constexpr int BYTES = KL + CS_NC * 64;
    int l;
    DEV int64_t &rb(int e) const { return *reinterpret_cast<int64_t *>(g_lds_cs + RB + (e * 64 + l) * 8); }
    DEV uint32_t &ql(int e) const { return *reinterpret_cast<uint32_t *>(g_lds_cs + QL + (e * 64 + l) * 4); }
    DEV uint8_t &nx(int e) const { return g_lds_cs[NX + e * 64 + l]; }
    DEV int32_t &cw(int c) const { return *reinterpret_cast<int32_t *>(g_lds_cs + CW + (c * 64 + l) * 4); }
    DEV int32_t &cr(int c) const { return *reinterpret_cast<int32_t *>(g_lds_cs + CR + (c * 64 + l) * 4); }
    DEV uint8_t &ch(int c) const { return g_lds_cs[CH + c * 64 + l]; }
    DEV uint8_t &ct(int c) const { return g_lds_cs[CT + c * 64 + l]; }
    DEV uint8_t &cn(int c) const { return g_lds_cs[CN + c * 64 + l]; }
    DEV uint8_t &ck(int c) const { return g_lds_cs[CK + c * 64 + l]; }
    DEV int8_t &cf(int c) const { return reinterpret_cast<int8_t &>(g_lds_cs[CF + c * 64 + l]); }
    DEV uint8_t &lf(int i) const { return g_lds_cs[LF + i * 64 + l]; }
    DEV int qb(int e) const { return (int)(ql(e) & 0xffffu); }
    DEV int ln(int e) const { return (int)(ql(e) >> 16); }
};

struct CsIdx {   // an index array of CsLds (ord, kept list) for ks_introsort
    int off;
    DEV uint8_t &operator[](int i) const { return g_lds_cs[off + i * 64]; }
    DEV CsIdx operator+(int i) const { return CsIdx{off + i * 64}; }
};

// lower_bound of kpos over the leaf's keys by chain pos (the pos of a chain is its first seed's rbeg)
DEV int cs_lower(const CsLds &L, int nk, int64_t kpos)
{
    int lo = 0, hi = nk;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (L.rb(L.ch(L.lf(mid))) < kpos) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__global__ void __launch_bounds__(64) k_chain_s(DIndex ix, DOpts o, Caps cp, const int64_t *offs, int n, const Intv *intv,
                                                const int32_t *n_intv, ChainDesc *chains_out, Seed *seeds_out,
                                                int32_t *n_chains, const uint32_t *status, Counters *ctr)
{
    const int nthr = gridDim.x * 64, tid = blockIdx.x * 64 + threadIdx.x;
    const CsLds L{(int)threadIdx.x};
    const int NS = cp.seeds < CS_NS ? cp.seeds : CS_NS, NC = cp.chains < CS_NC ? cp.chains : CS_NC;
    uint64_t nsa = 0;
    int guard = 0;
    for (int li = tid; li < n; li += nthr) {
        n_chains[li] = 0;
        if (status[li]) continue;
        const int len = (int)(offs[li + 1] - offs[li]);
        if (len < o.min_seed_len) continue;
        bool big = len > 0xffff;   // qbeg and len are kept in 16 bits
        int ns = 0, nk = 0;        // seeds; chains (= the keys of the root leaf)
        uint64_t rsa = 0;
        const SP<const Intv> mem{intv + intv_slot_at_d(li, 0, cp.intv)};
        const int nm = n_intv[li];
        for (int i0 = 0; i0 < nm && !big; i0 += 4) {
            uint64_t a0[4], a2[4], ai[4], s0[4];   // x[0], x[2], info and the first SA value of MEMs i0 .. i0 + 3
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                a0[u] = a2[u] = ai[u] = 0;
                if (i0 + u < nm) { const Intv &m = mem[i0 + u]; a0[u] = m.x[0]; a2[u] = m.x[2]; ai[u] = m.info; }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) s0[u] = a2[u] > 0 ? sa_at(ix, a0[u]) : 0;
            const int ue = nm - i0 < 4 ? nm - i0 : 4;
            for (int u = 0; u < ue && !big; ++u) {
                const uint64_t px0 = u == 0 ? a0[0] : u == 1 ? a0[1] : u == 2 ? a0[2] : a0[3];
                const uint64_t px2 = u == 0 ? a2[0] : u == 1 ? a2[1] : u == 2 ? a2[2] : a2[3];
                const uint64_t pin = u == 0 ? ai[0] : u == 1 ? ai[1] : u == 2 ? ai[2] : ai[3];
                const uint64_t sa0 = u == 0 ? s0[0] : u == 1 ? s0[1] : u == 2 ? s0[2] : s0[3];
                const int slen = (int)((uint32_t)pin - (uint32_t)(pin >> 32));
                const int qbeg = (int)(pin >> 32);
                const int step = px2 > (uint64_t)o.max_occ ? (int)(px2 / (uint64_t)o.max_occ) : 1;
                int count = 0;
                for (int64_t k = 0; (uint64_t)k < px2 && count < o.max_occ && !big; k += step, ++count) {
                    const int64_t rbeg = (int64_t)(k == 0 ? sa0 : sa_at(ix, px0 + (uint64_t)k));
                    ++rsa;
                    const int rid = intv2rid(ix, rbeg, rbeg + slen);
                    if (rid < 0) continue;
                    bool to_add = true;
                    if (nk) {
                        const int lo = cs_lower(L, nk, rbeg);
                        const int lower = lo < nk && L.rb(L.ch(L.lf(lo))) == rbeg ? L.lf(lo) : lo > 0 ? L.lf(lo - 1) : -1;
                        if (lower >= 0 && rid == L.cr(lower)) {   // test_and_merge
                            const int hd = L.ch(lower), tl = L.ct(lower);
                            const int64_t frb = L.rb(hd), lrb = L.rb(tl);
                            const int fqb = L.qb(hd), lqb = L.qb(tl), lln = L.ln(tl);
                            const int64_t qend = lqb + lln, rend = lrb + lln;
                            if (qbeg >= fqb && qbeg + slen <= qend && rbeg >= frb && rbeg + slen <= rend) {
                                to_add = false;   // contained
                            } else if (!((lrb < ix.l_pac || frb < ix.l_pac) && rbeg >= ix.l_pac)) {
                                const int64_t x = qbeg - lqb, y = rbeg - lrb;
                                if (y >= 0 && x - y <= o.w && y - x <= o.w && x - lln < o.max_chain_gap &&
                                    y - lln < o.max_chain_gap) {
                                    to_add = false;
                                    if (ns >= NS) { big = true; break; }
                                    const int si = ns++;
                                    L.rb(si) = rbeg; L.ql(si) = (uint32_t)qbeg | (uint32_t)slen << 16; L.nx(si) = 0xff;
                                    L.nx(tl) = (uint8_t)si;
                                    L.ct(lower) = (uint8_t)si;
                                    L.cn(lower) = (uint8_t)(L.cn(lower) + 1);
                                }
                            }
                        }
                    }
                    if (to_add) {
                        if (nk >= NC || ns >= NS) { big = true; break; }
                        const int si = ns++, ci = nk;
                        L.rb(si) = rbeg; L.ql(si) = (uint32_t)qbeg | (uint32_t)slen << 16; L.nx(si) = 0xff;
                        L.cr(ci) = rid; L.cn(ci) = 1; L.ch(ci) = L.ct(ci) = (uint8_t)si; L.cw(ci) = 0; L.ck(ci) = 0; L.cf(ci) = -1;
                        // kb_putp on the leaf: after the first key not below rbeg if it equals rbeg, else before it
                        const int lo = nk ? cs_lower(L, nk, rbeg) : 0;
                        const int at = nk == 0 ? 0 : lo == nk ? nk : (L.rb(L.ch(L.lf(lo))) > rbeg ? lo : lo + 1);
                        for (int j = nk - 1; j >= at; --j) L.lf(j + 1) = L.lf(j);
                        L.lf(at) = (uint8_t)ci;
                        ++nk;
                    }
                }
            }
        }
        if (big) { n_chains[li] = -1; continue; }
        nsa += rsa;
        // in-order traversal of the leaf = its keys; mem_chain_flt
        const CsIdx ord{CsLds::OR + L.l}, kept_list{CsLds::KL + L.l};
        int n_chn = 0;
        for (int i = 0; i < nk; ++i) {
            const int ci = L.lf(i);
            L.cf(ci) = -1; L.ck(ci) = 0;
            int64_t end = 0;
            int w = 0;
            for (int e = L.ch(ci); e != 0xff; e = L.nx(e)) {
                const int qb = L.qb(e), sl = L.ln(e);
                if (qb >= end) w += sl;
                else if (qb + sl > end) w += (int)(qb + sl - end);
                end = end > qb + sl ? end : qb + sl;
            }
            const int tmp = w;
            w = 0; end = 0;
            for (int e = L.ch(ci); e != 0xff; e = L.nx(e)) {
                const int64_t rb = L.rb(e);
                const int sl = L.ln(e);
                if (rb >= end) w += sl;
                else if (rb + sl > end) w += (int)(rb + sl - end);
                end = end > rb + sl ? end : rb + sl;
            }
            w = w < tmp ? w : tmp;
            w = w < (1 << 30) ? w : (1 << 30) - 1;
            L.cw(ci) = w;
            if (w >= o.min_chain_weight) ord[n_chn++] = (uint8_t)ci;
        }
        if (n_chn > 0) {
            guard += ks_introsort(ord, n_chn, [L](int a, int b) { return L.cw(a) > L.cw(b); }, SP<int>{nullptr});
            L.ck(ord[0]) = 3;
            int nkl = 0;
            kept_list[nkl++] = 0;
            for (int i = 1; i < n_chn; ++i) {
                int large_ovlp = 0, k;
                const int ci = ord[i];
                const int bi = L.qb(L.ch(ci)), ei = L.qb(L.ct(ci)) + L.ln(L.ct(ci));
                for (k = 0; k < nkl; ++k) {
                    const int j = kept_list[k], cj = ord[j];
                    const int bj = L.qb(L.ch(cj)), ej = L.qb(L.ct(cj)) + L.ln(L.ct(cj));
                    const int b_max = bj > bi ? bj : bi, e_min = ej < ei ? ej : ei;
                    if (e_min > b_max) {   // is_alt is always 0 on this path
                        const int li2 = ei - bi, lj = ej - bj, min_l = li2 < lj ? li2 : lj;
                        if (e_min - b_max >= min_l * o.mask_level && min_l < o.max_chain_gap) {
                            large_ovlp = 1;
                            if (L.cf(cj) < 0) L.cf(cj) = (int8_t)i;
                            if (L.cw(ci) < L.cw(cj) * o.drop_ratio && L.cw(cj) - L.cw(ci) >= o.min_seed_len << 1) break;
                        }
                    }
                }
                if (k == nkl) {
                    kept_list[nkl++] = (uint8_t)i;
                    L.ck(ci) = large_ovlp ? 2 : 3;
                }
            }
            for (int i = 0; i < nkl; ++i) {
                const int ci = ord[kept_list[i]];
                if (L.cf(ci) >= 0) L.ck(ord[L.cf(ci)]) = 1;
            }
            int i, k;
            for (i = k = 0; i < n_chn; ++i) {
                const int kp = L.ck(ord[i]);
                if (kp == 0 || kp == 3) continue;
                if (++k >= o.max_chain_extend) break;
            }
            for (; i < n_chn; ++i)
                if (L.ck(ord[i]) < 3) L.ck(ord[i]) = 0;
            ChainDesc *cd = chains_out + (size_t)li * cp.chains;
            Seed *so = seeds_out + (size_t)li * cp.seeds;
            int nc = 0, nso = 0;
            for (i = 0; i < n_chn; ++i) {
                const int ci = ord[i];
                if (L.ck(ci) == 0) continue;
                cd[nc].seed_off = nso; cd[nc].n = L.cn(ci); cd[nc].rid = L.cr(ci); cd[nc].w = L.cw(ci);
                for (int e = L.ch(ci); e != 0xff; e = L.nx(e)) {
                    so[nso].rbeg = L.rb(e); so[nso].qbeg = L.qb(e); so[nso].len = L.ln(e);
                    ++nso;
                }
                ++nc;
            }
            n_chains[li] = nc;
        }
    }
    wave_add(&ctr[STG_CHAIN].sa_values, nsa);
    wave_add(&ctr[STG_CHAIN].sort_guard, (unsigned long long)guard);
}

// ------------------------------------------------------------------------------------------------
// ksw_extend2 / ksw_global2 (ksw.c) over accessor-defined query and target
// ------------------------------------------------------------------------------------------------
// eh row storage for ksw_extend2: global int2, or LDS packed u16 pairs interleaved by lane
// (lane l's column j at lds[j * 64 + l]: every lane hits its own bank, so accesses never conflict).
// ksw_extend2 keeps h and e in [0, h0 + qlen*max] (every candidate is clamped at 0), so u16 is exact
// whenever the host-side bound check passes.
template <class P>   // int2 * (contiguous) or SP<int2, S> (lane-interleaved)
struct EhG {
    static constexpr bool kRing = false;
    P p;
    bool *ovf = nullptr;
    DEV int2 get(int j) const { return p[j]; }
    DEV void set(int j, int2 v) const { p[j] = v; }
    // the cell loop's cursor over consecutive columns (EhRing keeps an LDS byte address instead)
    using Cur = int;
    DEV Cur cur(int j) const { return j; }
    DEV Cur adv(Cur c) const { return c + 1; }
    DEV int2 at(Cur c) const { return get(c); }
    DEV void put(Cur c, int2 v) const { set(c, v); }
};
extern __shared__ uint32_t g_lds_eh[];   // dynamic LDS of k_extend<true>
struct EhL {   // offset-based so the accesses stay in the LDS address space (ds_read/ds_write, not flat)
    static constexpr bool kRing = false;
    int base;
    bool *ovf = nullptr;
    DEV int2 get(int j) const { uint32_t v = g_lds_eh[base + j * 64]; return make_int2((int)(v & 0xffffu), (int)(v >> 16)); }
    DEV void set(int j, int2 v) const { g_lds_eh[base + j * 64] = (uint32_t)v.x | ((uint32_t)v.y << 16); }
    using Cur = int;
    DEV Cur cur(int j) const { return j; }
    DEV Cur adv(Cur c) const { return c + 1; }
    DEV int2 at(Cur c) const { return get(c); }
    DEV void put(Cur c, int2 v) const { set(c, v); }
};

#define EXT_LDS_COLS 64   // ring columns (a power of two)
// 64-column ring of u16 pairs in LDS (column j at slot j & 63, lane-interleaved): ksw_extend2 only touches
// columns [beg, end] of the current row and beg never decreases, so the ring holds every live column while
// the window stays under 64 columns; columns are given their initial value when the band first reaches
// them.  A wider window sets *ovf (the read is re-run by the large-capacity retry pass).
struct EhRing {
    static constexpr bool kRing = true;
    bool *ovf;
    int base;
    DEV int2 get(int j) const { uint32_t v = g_lds_eh[base + (j & (EXT_LDS_COLS - 1)) * 64]; return make_int2((int)(v & 0xffffu), (int)(v >> 16)); }
    DEV void set(int j, int2 v) const { g_lds_eh[base + (j & (EXT_LDS_COLS - 1)) * 64] = (uint32_t)v.x | ((uint32_t)v.y << 16); }
    // Cell-loop cursor: the slot's byte offset 4 * (lane + (j & 63) * 64) (base is the lane, < 64, and the ring is the
    // first 16 KB of the dynamic LDS), advanced by one add and one and per column instead of recomputed for every
    // access (the loop reads column j + 1 and stores column j: the store's slot is the previous read's).
    using Cur = uint32_t;
    DEV Cur cur(int j) const { return 4u * ((uint32_t)base + ((uint32_t)j & (EXT_LDS_COLS - 1)) * 64u); }
    DEV Cur adv(Cur c) const { return (c + 256u) & (EXT_LDS_COLS * 256u - 1u); }
    DEV int2 at(Cur c) const
    {
        const uint32_t v = *reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(g_lds_eh) + c);
        return make_int2((int)(v & 0xffffu), (int)(v >> 16));
    }
    DEV void put(Cur c, int2 v) const
    {
        *reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(g_lds_eh) + c) = (uint32_t)v.x | ((uint32_t)v.y << 16);
    }
};

// Query accessors whose values are pre-scaled codes (4 * code) with readable padding one column past either
// end of every query window (QLane: the read staged in LDS): the cell score is then a 4-bit field of a
// per-row profile word, and the next column is read without a bounds select.
template <class QA> struct QPre { static constexpr bool v = false; };

template <class EH, class QA>
DEV int ksw_extend2_body(const DOpts &o, int qlen, QA query, int tlen, TAcc target, int o_del, int e_del, int o_ins,
                         int e_ins, int w, int end_bonus, int zdrop, int h0, int *_qle, int *_tle, int *_gtle,
                         int *_gscore, int *_max_off, EH eh, uint64_t &cells)
{
    int i, j, oe_del = o_del + e_del, oe_ins = o_ins + e_ins, beg, end, max, max_i, max_j, max_ins, max_del, max_ie,
        gscore, max_off;
    const Score sc = score_of(o);
    if (qlen < 0) qlen = 0;
    // eh[0] = h0, eh[1] = max(h0 - oe_ins, 0), eh[j>=2] = eh[j-1] - e_ins while eh[j-1] > e_ins, else 0
    const int v1 = h0 > oe_ins ? h0 - oe_ins : 0;
    auto init_h = [&](int jj) { return jj == 0 ? h0 : (jj == 1 ? v1 : (v1 - (jj - 1) * e_ins > 0 ? v1 - (jj - 1) * e_ins : 0)); };
    int hi = EH::kRing ? (qlen < EXT_LDS_COLS - 1 ? qlen : EXT_LDS_COLS - 1) : qlen;   // columns <= hi hold their values
    for (j = 0; j <= hi; ++j) eh.set(j, make_int2(init_h(j), 0));
    max = o.mat_max > 0 ? o.mat_max : 0;
    max_ins = idiv_plus(qlen * max + end_bonus - o_ins, e_ins, 1);
    max_ins = max_ins > 1 ? max_ins : 1;
    w = w < max_ins ? w : max_ins;
    max_del = idiv_plus(qlen * max + end_bonus - o_del, e_del, 1);
    max_del = max_del > 1 ? max_del : 1;
    w = w < max_del ? w : max_del;
    max = h0, max_i = max_j = -1; max_ie = -1, gscore = -1;
    max_off = 0;
    beg = 0, end = qlen;
    TStream ts;
    if (tlen > 0) ts.init(*target.ix, target.start, target.dir);
    constexpr bool pre = QPre<QA>::v;
    // profile of this row's target base: field q (4 bits at 4q) = score(tb, q) + 8 (pre-scaled path; the launch
    // checks that every score of the matrix lies in [-8, 7])
    const uint32_t prof_mis = (uint32_t)(sc.mis + 8) * 0x1111u | (uint32_t)(sc.amb + 8) << 16;
    for (i = 0; i < tlen; ++i) {
        int t, f = 0, h1, m = 0, mj = -1;
        const int tb = ts.next();
        const uint32_t prof = prof_mis + ((uint32_t)(sc.match - sc.mis) << (4 * tb));   // tb < 4 (pac bases)
        if (beg < i - w) beg = i - w;
        if (end > i + w + 1) end = i + w + 1;
        if (end > qlen) end = qlen;
        if (beg == 0) {
            h1 = h0 - (o_del + e_del * (i + 1));
            if (h1 < 0) h1 = 0;
        } else h1 = 0;
        if (EH::kRing && end > hi) {   // materialise the columns the band reaches for the first time
            if (end - beg >= EXT_LDS_COLS - 1) { *eh.ovf = true; break; }
            for (j = hi + 1; j <= end; ++j) eh.set(j, make_int2(init_h(j), 0));
            hi = end;
        }
        cells += (uint64_t)(end > beg ? end - beg : 0);
        // The row reads column j+1 (eh and query) before it stores column j: the two never share a slot
        // (the ring window is < 63 columns), so each cell's LDS round trip overlaps the previous cell's
        // arithmetic.  The zero-trimming scans libbwa runs after the row (first non-zero column in
        // [beg, end), last non-zero in [beg, end]) are tracked here from the values being stored; every
        // stored h and e is >= 0, so "non-zero" is (h | e) != 0.
        int nzf = beg < end ? end : beg, nzl = -1;   // (the serial scan's start values)
        if (EH::kRing && pre && beg < end) {
            // LDS ring: each cell first stores the previous cell's column (deferred by one cell), then reads column
            // j + 2, then computes column j from values read two cells earlier.  Every LDS operation of a cell is thus
            // issued before its arithmetic, and the wait at the next cell's top finds them done -- with the store
            // last in the cell (the loop above), each trip waited out a whole LDS store latency.  The deferred store
            // starts as a rewrite of column beg's own old value; reads of columns end + 1 (stale slot) and query
            // index qlen + 1 (inside the staged rows or the ring) are never used.
            typename EH::Cur c0 = eh.cur(beg), c1 = eh.adv(c0);
            int2 p0 = eh.at(c0), p1 = eh.at(c1);
            int q0 = query(beg), q1 = query(beg + 1);
            typename EH::Cur sc = c0;
            int2 sv = p0;
#pragma unroll 2
            for (j = beg; j < end; ++j) {
                eh.put(sc, sv);
                const typename EH::Cur c2 = eh.adv(c1);
                const int2 p2 = eh.at(c2);
                const int q2 = query(j + 2);
                int h, M = p0.x, e = p0.y;
                const int hx = h1;
                M = M ? M + (int)__builtin_amdgcn_ubfe(prof, (uint32_t)q0, 4u) - 8 : 0;
                h = M > e ? M : e;
                h = h > f ? h : f;
                h1 = h;
                mj = m > h ? mj : j;
                m = m > h ? m : h;
                t = M - oe_del; t = t > 0 ? t : 0;
                e -= e_del; e = e > t ? e : t;
                sc = c0; sv = make_int2(hx, e);
                if ((hx | e) != 0) { nzl = j; nzf = nzf < j ? nzf : j; }
                t = M - oe_ins; t = t > 0 ? t : 0;
                f -= e_ins; f = f > t ? f : t;
                p0 = p1; p1 = p2; q0 = q1; q1 = q2; c0 = c1; c1 = c2;
            }
            eh.put(sc, sv);
        } else if (beg < end) {
            typename EH::Cur cj = eh.cur(beg);
            int2 p = eh.at(cj);
            int qj = query(beg);
#pragma unroll 2   // two cells per trip: no loop-carried register copies, half the loop control (42 -> 36 per cell)
            for (j = beg; j < end; ++j) {
                const typename EH::Cur cn = eh.adv(cj);
                const int2 pn = eh.at(cn);
                const int qn = pre ? query(j + 1) : (j + 1 < end ? query(j + 1) : 0);
                int h, M = p.x, e = p.y;
                const int hx = h1;
                if (pre) M = M ? M + (int)__builtin_amdgcn_ubfe(prof, (uint32_t)qj, 4u) - 8 : 0;
                else M = M ? M + sc(tb, qj) : 0;
                h = M > e ? M : e;
                h = h > f ? h : f;
                h1 = h;
                mj = m > h ? mj : j;
                m = m > h ? m : h;
                t = M - oe_del; t = t > 0 ? t : 0;
                e -= e_del; e = e > t ? e : t;
                eh.put(cj, make_int2(hx, e));
                if ((hx | e) != 0) { nzl = j; nzf = nzf < j ? nzf : j; }
                t = M - oe_ins; t = t > 0 ? t : 0;
                f -= e_ins; f = f > t ? f : t;
                p = pn; qj = qn; cj = cn;
            }
        } else j = beg;
        eh.set(end, make_int2(h1, 0));
        if (h1 != 0) nzl = end;
        if (j == qlen) {
            max_ie = gscore > h1 ? max_ie : i;
            gscore = gscore > h1 ? gscore : h1;
        }
        if (m == 0) break;
        if (m > max) {
            max = m, max_i = i, max_j = mj;
            int d = mj - i; d = d < 0 ? -d : d;
            max_off = max_off > d ? max_off : d;
        } else if (zdrop > 0) {
            if (i - max_i > mj - max_j) {
                if (max - m - ((i - max_i) - (mj - max_j)) * e_del > zdrop) break;
            } else {
                if (max - m - ((mj - max_j) - (i - max_i)) * e_ins > zdrop) break;
            }
        }
        beg = nzf;
        j = end < beg ? end : (nzl >= 0 ? nzl : beg - 1);
        end = j + 2 < qlen ? j + 2 : qlen;
    }
    *_qle = max_j + 1;
    *_tle = max_i + 1;
    *_gtle = max_ie + 1;
    *_gscore = gscore;
    *_max_off = max_off;
    return max;
}

// global-memory variant (retry pass): an out-of-line call keeps the large-capacity kernel small
template <class EH, class QA>
DEVN int ksw_extend2(const DOpts &o, int qlen, QA query, int tlen, TAcc target, int o_del, int e_del, int o_ins,
                     int e_ins, int w, int end_bonus, int zdrop, int h0, int *_qle, int *_tle, int *_gtle,
                     int *_gscore, int *_max_off, EH eh, uint64_t &cells)
{
    return ksw_extend2_body(o, qlen, query, tlen, target, o_del, e_del, o_ins, e_ins, w, end_bonus, zdrop, h0, _qle,
                            _tle, _gtle, _gscore, _max_off, eh, cells);
}

#define MINUS_INF (-0x40000000)

// ksw_global2; z == nullptr -> score only.  Returns score; traceback pushed as libbwa push_cigar
// into cig[] (capacity cap, ops appended then reversed); *ncig = -1 on overflow.
DEVN int ksw_global2(const DOpts &o, int qlen, QAcc query, int tlen, TAcc target, int o_del, int e_del, int o_ins,
                     int e_ins, int w, int2 *eh, uint8_t *z, int64_t zcap, uint32_t *cig, int cap, int *ncig,
                     bool &ovf, uint64_t &cells)
{
    int i, j, k, oe_del = o_del + e_del, oe_ins = o_ins + e_ins, score, n_col;
    const Score sc = score_of(o);
    n_col = qlen < 2 * w + 1 ? qlen : 2 * w + 1;
    if (z && (int64_t)n_col * tlen > zcap) { ovf = true; return 0; }
    eh[0] = make_int2(0, MINUS_INF);
    for (j = 1; j <= qlen && j <= w; ++j) eh[j] = make_int2(-(o_ins + e_ins * j), MINUS_INF);
    for (; j <= qlen; ++j) eh[j] = make_int2(MINUS_INF, MINUS_INF);
    for (i = 0; i < tlen; ++i) {
        int32_t f = MINUS_INF, h1, beg, end, t;
        const int tb = target(i);
        beg = i > w ? i - w : 0;
        end = i + w + 1 < qlen ? i + w + 1 : qlen;
        h1 = beg == 0 ? -(o_del + e_del * (i + 1)) : MINUS_INF;
        uint8_t *zi = z ? z + (int64_t)i * n_col : nullptr;
        cells += (uint64_t)(end > beg ? end - beg : 0);
        for (j = beg; j < end; ++j) {
            int2 p = eh[j];
            int32_t h, m = p.x, e = p.y;
            uint8_t d;
            p.x = h1;
            m += sc(tb, query(j));
            d = m >= e ? 0 : 1;
            h = m >= e ? m : e;
            d = h >= f ? d : 2;
            h = h >= f ? h : f;
            h1 = h;
            t = m - oe_del;
            e -= e_del;
            d |= e > t ? 1 << 2 : 0;
            e = e > t ? e : t;
            p.y = e;
            eh[j] = p;
            t = m - oe_ins;
            f -= e_ins;
            d |= f > t ? 2 << 4 : 0;
            f = f > t ? f : t;
            if (zi) zi[j - beg] = d;
        }
        eh[end] = make_int2(h1, MINUS_INF);
    }
    score = eh[qlen].x;
    if (z) {
        int n = 0, which = 0;
        i = tlen - 1;
        k = (i + w + 1 < qlen ? i + w + 1 : qlen) - 1;
        auto push = [&](int op, int len) {
            if (n == 0 || op != (int)(cig[n - 1] & 0xf)) {
                if (n >= cap) { ovf = true; return; }
                cig[n++] = (uint32_t)len << 4 | (uint32_t)op;
            } else cig[n - 1] += (uint32_t)len << 4;
        };
        while (i >= 0 && k >= 0 && !ovf) {
            which = z[(int64_t)i * n_col + (k - (i > w ? i - w : 0))] >> (which << 1) & 3;
            if (which == 0) push(0, 1), --i, --k;
            else if (which == 1) push(2, 1), --i;
            else push(1, 1), --k;
        }
        if (i >= 0) push(2, i + 1);
        if (k >= 0) push(1, k + 1);
        for (i = 0; i < (n >> 1); ++i) { uint32_t t = cig[i]; cig[i] = cig[n - 1 - i]; cig[n - 1 - i] = t; }
        *ncig = ovf ? -1 : n;
    }
    return score;
}

// ksw_global2's score alone, inlined (mem_patch_reg's use in the extension stage): the same recurrences as
// ksw_global2 above without the traceback, so the extension kernel makes no out-of-line call and needs no
// private stack segment.
template <class EHP>
DEV int ksw_global2_score(const DOpts &o, int qlen, QAcc query, int tlen, TAcc target, int o_del, int e_del, int o_ins,
                          int e_ins, int w, EHP eh, uint64_t &cells)
{
    const int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
    const Score sc = score_of(o);
    eh[0] = make_int2(0, MINUS_INF);
    int j;
    for (j = 1; j <= qlen && j <= w; ++j) eh[j] = make_int2(-(o_ins + e_ins * j), MINUS_INF);
    for (; j <= qlen; ++j) eh[j] = make_int2(MINUS_INF, MINUS_INF);
    for (int i = 0; i < tlen; ++i) {
        int32_t f = MINUS_INF, h1, t;
        const int tb = target(i);
        const int beg = i > w ? i - w : 0;
        const int end = i + w + 1 < qlen ? i + w + 1 : qlen;
        h1 = beg == 0 ? -(o_del + e_del * (i + 1)) : MINUS_INF;
        cells += (uint64_t)(end > beg ? end - beg : 0);
        for (j = beg; j < end; ++j) {
            int2 p = eh[j];
            int32_t h, m = p.x, e = p.y;
            p.x = h1;
            m += sc(tb, query(j));
            h = m >= e ? m : e;
            h = h >= f ? h : f;
            h1 = h;
            t = m - oe_del;
            e -= e_del;
            e = e > t ? e : t;
            p.y = e;
            eh[j] = p;
            t = m - oe_ins;
            f -= e_ins;
            f = f > t ? f : t;
        }
        eh[end] = make_int2(h1, MINUS_INF);
    }
    return eh[qlen].x;
}

// bwa_gen_cigar2's score for mem_patch_reg (no CIGAR)
template <class EHP>
DEV int gen_cigar2_score(const DIndex &ix, const DOpts &o, int w_, const uint8_t *q, int qb, int l_query, int64_t rb,
                         int64_t re, int *score, EHP eh, uint64_t &cells, uint64_t &bases)
{
    if (l_query <= 0 || rb >= re || (rb < ix.l_pac && re > ix.l_pac)) return 0;
    const int64_t rlen = re - rb;
    if (re > (ix.l_pac << 1) || rb < 0) return 0;
    bases += (uint64_t)((rlen + 3) >> 2);
    const bool rev = rb >= ix.l_pac;
    QAcc qa{q, rev ? qb + l_query - 1 : qb, rev ? -1 : 1};
    TAcc ta{&ix, rev ? re - 1 : rb, rev ? -1 : 1};
    if (l_query == rlen && w_ == 0) {
        int s = 0;
        for (int i = 0; i < l_query; ++i) s += mat_sc(o, ta(i), qa(i));
        *score = s;
        return 1;
    }
    int max_ins = idiv_plus(((l_query + 1) >> 1) * o.mat_match - o.o_ins, o.e_ins, 1);
    int max_del = idiv_plus(((l_query + 1) >> 1) * o.mat_match - o.o_del, o.e_del, 1);
    int max_gap = max_ins > max_del ? max_ins : max_del;
    max_gap = max_gap > 1 ? max_gap : 1;
    int dl = (int)rlen - l_query; dl = dl < 0 ? -dl : dl;
    int w = (max_gap + dl + 1) >> 1;
    w = w < w_ ? w : w_;
    const int min_w = dl + 3;
    w = w > min_w ? w : min_w;
    *score = ksw_global2_score(o, l_query, qa, (int)rlen, ta, o.o_del, o.e_del, o.o_ins, o.e_ins, w, eh, cells);
    return 1;
}

// bwa_gen_cigar2 (score + CIGAR; MD/NM are not part of bioseqdb's output)
DEV int gen_cigar2(const DIndex &ix, const DOpts &o, int w_, const uint8_t *q, int qb, int l_query, int64_t rb,
                   int64_t re, int *score, int2 *eh, uint8_t *z, int64_t zcap, uint32_t *cig, int cap, int *ncig,
                   bool &ovf, uint64_t &cells, uint64_t &bases)
{
    *ncig = 0;
    if (l_query <= 0 || rb >= re || (rb < ix.l_pac && re > ix.l_pac)) return 0;
    int64_t rlen = re - rb;   // bns_get_seq never clamps here: [rb,re) lies inside [0, 2*l_pac)
    if (re > (ix.l_pac << 1) || rb < 0) return 0;
    bases += (uint64_t)((rlen + 3) >> 2);
    const bool rev = rb >= ix.l_pac;
    QAcc qa{q, rev ? qb + l_query - 1 : qb, rev ? -1 : 1};
    TAcc ta{&ix, rev ? re - 1 : rb, rev ? -1 : 1};
    if (l_query == rlen && w_ == 0) {
        if (z) {
            if (cap < 1) { ovf = true; return 0; }
            cig[0] = (uint32_t)l_query << 4;
            *ncig = 1;
        }
        int s = 0;
        for (int i = 0; i < l_query; ++i) s += mat_sc(o, ta(i), qa(i));
        *score = s;
    } else {
        int w, max_gap, max_ins, max_del, min_w;
        max_ins = idiv_plus(((l_query + 1) >> 1) * o.mat_match - o.o_ins, o.e_ins, 1);
        max_del = idiv_plus(((l_query + 1) >> 1) * o.mat_match - o.o_del, o.e_del, 1);
        max_gap = max_ins > max_del ? max_ins : max_del;
        max_gap = max_gap > 1 ? max_gap : 1;
        int dl = (int)rlen - l_query; dl = dl < 0 ? -dl : dl;
        w = (max_gap + dl + 1) >> 1;
        w = w < w_ ? w : w_;
        min_w = dl + 3;
        w = w > min_w ? w : min_w;
        *score = ksw_global2(o, l_query, qa, (int)rlen, ta, o.o_del, o.e_del, o.o_ins, o.e_ins, w, eh, z, zcap, cig,
                             cap, ncig, ovf, cells);
    }
    return 1;
}

// ------------------------------------------------------------------------------------------------
// k_flt_seeds: mem_flt_chained_seeds (bwamem.c) for reads long enough to trigger it (5.5 ln l <= 0.05 l,
// l >~ 700): seeds shorter than MEM_SHORT_LEN whose +-50-base neighbourhood scores below the HSP
// threshold under ksw_align2 (mem_seed_sw) leave their chain; kept seeds take that score (len*a when no
// SW ran), which orders them in mem_chain2aln.  Shorter reads keep score = len and skip all of this.
// ------------------------------------------------------------------------------------------------
#define KSW_P 8
DEV int sub0(int a, int b) { return a > b ? a - b : 0; }   // _mm_subs_epu16 on values >= 0

// r.score of ksw_align2(..., KSW_XSTART) -> ksw_i16: a lane-for-lane emulation of the striped SSE2 kernel
// (see oracle/bwa_oracle.c ksw_align2_score for why the striping shows in the result).  buf: 3*slen*8 int16.
DEV int ksw_i16_score(const Score sc, int qlen, const uint8_t *query, int tlen, const DIndex &ix, int64_t tbeg,
                      int o_del, int e_del, int o_ins, int e_ins, int16_t *buf, uint64_t &cells)
{
    const int slen = (qlen + KSW_P - 1) / KSW_P, oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
    int16_t *H0 = buf, *H1 = buf + slen * KSW_P, *E = buf + 2 * slen * KSW_P;
    for (int j = 0; j < slen * KSW_P; ++j) { H0[j] = 0; E[j] = 0; }
    int gmax = 0;
    for (int i = 0; i < tlen; ++i) {
        int f[KSW_P], mx[KSW_P], h[KSW_P];
        const int tb = ref_at(ix, tbeg + i);
        h[0] = 0;
#pragma unroll
        for (int k = 0; k < KSW_P; ++k) { f[k] = 0; mx[k] = 0; if (k) h[k] = H0[(slen - 1) * KSW_P + k - 1]; }
        for (int j = 0; j < slen; ++j) {
#pragma unroll
            for (int k = 0; k < KSW_P; ++k) {
                const int pos = j + k * slen;
                int v = h[k] + (pos < qlen ? sc(tb, query[pos]) : 0);
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
        cells += (uint64_t)slen * KSW_P;
        for (int kk = 0; kk < 16; ++kk) {   // lazy F: into H only, at most 16 sweeps
#pragma unroll
            for (int k = KSW_P - 1; k > 0; --k) f[k] = f[k - 1];
            f[0] = 0;
            bool more = true;
            for (int j = 0; j < slen && more; ++j) {
                more = false;
#pragma unroll
                for (int k = 0; k < KSW_P; ++k) {
                    int v = H1[j * KSW_P + k];
                    v = v > f[k] ? v : f[k];
                    H1[j * KSW_P + k] = (int16_t)v;
                    const int hv = sub0(v, oe_ins);
                    f[k] = sub0(f[k], e_ins);
                    more |= f[k] > hv;
                }
            }
            if (!more) break;
        }
        int imax = 0;
#pragma unroll
        for (int k = 0; k < KSW_P; ++k) imax = imax > mx[k] ? imax : mx[k];
        gmax = gmax > imax ? gmax : imax;
        int16_t *sw = H0; H0 = H1; H1 = sw;
    }
    return gmax;
}

// mem_seed_sw: -1 when the seed needs no SW
DEV int mem_seed_sw(const DIndex &ix, const DOpts &o, int l_query, const uint8_t *q, const Seed &sd, int16_t *buf,
                    uint64_t &cells, uint64_t &bases)
{
    const int64_t l_pac = ix.l_pac;
    if (sd.len >= 200) return -1;
    int qb = sd.qbeg, qe = sd.qbeg + sd.len;
    int64_t rb = sd.rbeg, re = sd.rbeg + sd.len;
    const int64_t mid = (rb + re) >> 1;
    qb -= 50; qb = qb > 0 ? qb : 0;
    qe += 50; qe = qe < l_query ? qe : l_query;
    rb -= 50; rb = rb > 0 ? rb : 0;
    re += 50; re = re < l_pac << 1 ? re : l_pac << 1;
    if (rb < l_pac && l_pac < re) {
        if (mid < l_pac) re = l_pac;
        else rb = l_pac;
    }
    if (qe - qb >= 200 || re - rb >= 200) return -1;
    {   // bns_fetch_seq: clamp to the row (strand-flipped) containing mid
        int is_rev;
        const int rid = pos2rid(ix, depos(ix, mid, is_rev));
        int64_t far_beg = ix.ann_off[rid], far_end = far_beg + ix.ann_len[rid];
        if (is_rev) { const int64_t t = far_beg; far_beg = (l_pac << 1) - far_end; far_end = (l_pac << 1) - t; }
        rb = rb > far_beg ? rb : far_beg;
        re = re < far_end ? re : far_end;
    }
    if (re <= rb) return 0;
    bases += (uint64_t)((re - rb + 3) >> 2);
    return ksw_i16_score(score_of(o), qe - qb, q + qb, (int)(re - rb), ix, rb, o.o_del, o.e_del, o.o_ins, o.e_ins, buf,
                         cells);
}

__global__ void __launch_bounds__(256) k_flt_seeds(DIndex ix, DOpts o, Caps cp, const uint8_t *codes,
                                                   const int64_t *offs, const int32_t *sel, int n, ChainDesc *chains,
                                                   Seed *seeds, const int32_t *n_chains, const uint32_t *status,
                                                   int32_t *sscore, uint8_t *scratch, Counters *ctr)
{
    const int nthr = gridDim.x * blockDim.x;
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    int16_t *buf = reinterpret_cast<int16_t *>(scratch + (size_t)tid * cp.scratch);
    uint64_t cells = 0, bases = 0;
    for (int li = tid; li < n; li += nthr) {
        if (status[li]) continue;
        const int r = read_of(sel, li);
        const int len = (int)(offs[r + 1] - offs[r]);
        const uint8_t *q = codes + offs[r];
        // the float/double mix of bwamem.c: MEM_MINSC_COEF 5.5f * log(), MEM_SEEDSW_COEF 0.05f * l_query
        const double min_l = o.min_chain_weight ? 1.1f * o.min_chain_weight : 5.5f * log((double)len);
        const bool active = !(min_l > (double)(0.05f * (float)len));
        const int min_hsp = (int)(o.a * min_l + .499);
        ChainDesc *cd = chains + (size_t)li * cp.chains;
        Seed *sd = seeds + (size_t)li * cp.seeds;
        int32_t *ss = sscore + (size_t)li * cp.seeds;
        const int nc = n_chains[li];
        for (int c = 0; c < nc; ++c) {
            Seed *cs = sd + cd[c].seed_off;
            int32_t *cscore = ss + cd[c].seed_off;
            int k = 0;
            for (int j = 0; j < cd[c].n; ++j) {
                const Seed t = cs[j];
                int score = t.len;   // mem_chain: s.score = s.len
                if (active) {
                    score = mem_seed_sw(ix, o, len, q, t, buf, cells, bases);
                    if (!(score < 0 || score >= min_hsp)) continue;
                    score = score < 0 ? t.len * o.a : score;
                }
                cs[k] = t;
                cscore[k] = score;
                ++k;
            }
            cd[c].n = k;
        }
    }
    wave_add(&ctr[STG_CHAIN].dp_cells, cells);
    wave_add(&ctr[STG_CHAIN].ref_bases, bases);
}

hipError_t launch_flt_seeds(int grid, hipStream_t st, const DIndex &ix, const DOpts &o, const Caps &cp,
                            const uint8_t *codes, const int64_t *offs, const int32_t *sel, int n, ChainDesc *chains,
                            Seed *seeds, const int32_t *n_chains, const uint32_t *status, int32_t *sscore,
                            uint8_t *scratch, Counters *ctr)
{
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_flt_seeds, dim3(grid), dim3(256), 0, st, ix, o, cp, codes, offs, sel, n, chains, seeds, n_chains,
                       status, sscore, scratch, ctr);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// k_extend: mem_chain2aln for every chain, mem_sort_dedup_patch, mem_mark_primary_se
// ------------------------------------------------------------------------------------------------
DEV int cal_max_gap(const DOpts &o, int qlen)
{
    int l_del = idiv_plus(qlen * o.a - o.o_del, o.e_del, 1);
    int l_ins = idiv_plus(qlen * o.a - o.o_ins, o.e_ins, 1);
    int l = l_del > l_ins ? l_del : l_ins;
    l = l > 1 ? l : 1;
    return l < o.w << 1 ? l : o.w << 1;
}

DEV uint64_t hash_64(uint64_t key)
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

// The extension's lane-private scratch: S = 64 lays each array out interleaved across the 64 lanes of a wave
// (element i of a lane at [i * 64 + lane] of the wave's region, SP), so a wave's same-index accesses share cache
// lines; S = 1 keeps a thread's arrays contiguous (the retry pass, whose workspace holds one read's scratch per
// thread).  Every array is typed SP<T, S>, so no code path can index it with the other layout.
template <int S>
struct ExtCtx {
    Reg *av; int n, cap;   // the read's regions: its own output slot (contiguous per read)
    SP<Reg, S> tmp;
    SP<int, S> idx;
    SP<uint64_t, S> srt;
    SP<int2, S> eh;
    SP<int, S> stk;        // introsort stack (192 ints)
    bool ovf;
    int guard = 0;         // ks_introsort scans stopped by the bound (Counters::sort_guard)
};

struct QMakeG {   // query accessors over the read in global memory
    const uint8_t *q;
    DEV QAcc at(int start, int dir) const { return QAcc{q, start, dir}; }
};
extern __shared__ uint8_t g_lds_q8[];   // same dynamic LDS as g_lds_eh; query bytes start at `off`
struct QLane {   // lane-interleaved query bytes in LDS: base j of this lane at off + j*64 + lane
    int off, start, dir;
    DEV int operator()(int j) const { return g_lds_q8[off + (start + dir * j) * 64]; }
};
struct QMakeL {
    int off;   // byte offset of this lane's column 0
    DEV QLane at(int start, int dir) const { return QLane{off, start, dir}; }
};
// k_extend<true> stages 4 * code; a window's one-past-the-end column (index -1 or len) lies inside the
// dynamic LDS allocation (the ring precedes the query rows, one spare row follows them)
template <> struct QPre<QLane> { static constexpr bool v = true; };

// Extension rows for k_extend<true>: the eh row is a 64-column LDS ring (EhRing); the read is staged
// in LDS once per read (QMakeL) after the ring columns.
struct EhSmall {
    int lane;       // LDS column (threadIdx.x of the 64-thread block)
    bool *ovf;      // ring overflow -> read re-run by the retry pass
};

template <class QA>
DEV int ext_call(const DOpts &o, int qlen, QA query, int tlen, TAcc target, int o_del, int e_del, int o_ins, int e_ins,
                 int w, int end_bonus, int zdrop, int h0, int *qle, int *tle, int *gtle, int *gscore, int *max_off,
                 EhSmall ehx, uint64_t &cells)
{
    // inlined: an out-of-line call spills the caller's live VGPRs to scratch around every extension
    return ksw_extend2_body(o, qlen, query, tlen, target, o_del, e_del, o_ins, e_ins, w, end_bonus, zdrop, h0, qle, tle,
                            gtle, gscore, max_off, EhRing{ehx.ovf, ehx.lane}, cells);
}
template <class QA, class EH>
DEV int ext_call(const DOpts &o, int qlen, QA query, int tlen, TAcc target, int o_del, int e_del, int o_ins, int e_ins,
                 int w, int end_bonus, int zdrop, int h0, int *qle, int *tle, int *gtle, int *gscore, int *max_off,
                 EH ehx, uint64_t &cells)
{
    return ksw_extend2(o, qlen, query, tlen, target, o_del, e_del, o_ins, e_ins, w, end_bonus, zdrop, h0, qle, tle, gtle,
                       gscore, max_off, ehx, cells);
}

// mem_chain2aln's reference window of a chain: [rmax0, rmax1) from every seed's maximal gaps, not crossing the
// forward/reverse junction and clamped to the row (strand-flipped) that holds seeds[0] (bns_fetch_seq)
DEV void chain_window(const DIndex &ix, const DOpts &o, int l_query, const Seed *seeds, int cn, int64_t &rmax0,
                      int64_t &rmax1, uint64_t &bases)
{
    const int64_t l_pac = ix.l_pac;
    rmax0 = l_pac << 1; rmax1 = 0;
    for (int i = 0; i < cn; ++i) {
        const Seed &t = seeds[i];
        int64_t b = t.rbeg - (t.qbeg + cal_max_gap(o, t.qbeg));
        int64_t e = t.rbeg + t.len + ((l_query - t.qbeg - t.len) + cal_max_gap(o, l_query - t.qbeg - t.len));
        rmax0 = rmax0 < b ? rmax0 : b;
        rmax1 = rmax1 > e ? rmax1 : e;
    }
    rmax0 = rmax0 > 0 ? rmax0 : 0;
    rmax1 = rmax1 < l_pac << 1 ? rmax1 : l_pac << 1;
    if (rmax0 < l_pac && l_pac < rmax1) {
        if (seeds[0].rbeg < l_pac) rmax1 = l_pac;
        else rmax0 = l_pac;
    }
    int is_rev;
    int rid = pos2rid(ix, depos(ix, seeds[0].rbeg, is_rev));
    int64_t far_beg = ix.ann_off[rid], far_end = far_beg + ix.ann_len[rid];
    if (is_rev) { int64_t t = far_beg; far_beg = (l_pac << 1) - far_end; far_end = (l_pac << 1) - t; }
    rmax0 = rmax0 > far_beg ? rmax0 : far_beg;
    rmax1 = rmax1 < far_end ? rmax1 : far_end;
    bases += (uint64_t)((rmax1 - rmax0 + 3) >> 2);
}

// the chain's seeds in ascending (score, index) order: mem_chain2aln visits srt[n-1] .. srt[0]; score = len
// (mem_chain), or mem_flt_chained_seeds' score for long reads
template <class SRT>
DEV void seed_order(SRT srt, const Seed *seeds, const int32_t *sscore, int cn)
{
    for (int i = 0; i < cn; ++i) srt[i] = (uint64_t)(uint32_t)(sscore ? sscore[i] : seeds[i].len) << 32 | (uint64_t)i;
    for (int i = 1; i < cn; ++i) {   // keys are unique: any correct sort equals ks_introsort_64
        uint64_t t = srt[i];
        int j = i;
        while (j > 0 && t < srt[j - 1]) { srt[j] = srt[j - 1]; --j; }
        srt[j] = t;
    }
}

// mem_chain2aln's test whether seed s (srt[k]) is skipped: contained in an existing region and not overlapping
// a longer seed of the chain, visited earlier, on a different diagonal
template <class SRT>
DEV bool seed_skipped(const DOpts &o, int l_query, const Reg *av, int n_av, SRT srt, int k, int cn, const Seed *seeds,
                      const Seed &s)
{
    int i;
    for (i = 0; i < n_av; ++i) {
        const Reg &p = av[i];
        if (s.rbeg < p.rb || s.rbeg + s.len > p.re || s.qbeg < p.qb || s.qbeg + s.len > p.qe) continue;
        if (s.len - p.seedlen0 > .1 * l_query) continue;
        int qd = s.qbeg - p.qb;
        int64_t rd = s.rbeg - p.rb;
        int max_gap = cal_max_gap(o, qd < rd ? qd : (int)rd);
        int w = max_gap < p.w ? max_gap : p.w;
        if (qd - rd < w && rd - qd < w) break;
        qd = p.qe - (s.qbeg + s.len);
        rd = p.re - (s.rbeg + s.len);
        max_gap = cal_max_gap(o, qd < rd ? qd : (int)rd);
        w = max_gap < p.w ? max_gap : p.w;
        if (qd - rd < w && rd - qd < w) break;
    }
    if (i == n_av) return false;
    for (i = k + 1; i < cn; ++i) {
        if (srt[i] == 0) continue;
        const Seed &t = seeds[(uint32_t)srt[i]];
        if (t.len < s.len * .95) continue;
        if (s.qbeg <= t.qbeg && s.qbeg + s.len - t.qbeg >= s.len >> 2 && t.qbeg - s.qbeg != t.rbeg - s.rbeg) break;
        if (t.qbeg <= s.qbeg && t.qbeg + t.len - s.qbeg >= s.len >> 2 && s.qbeg - t.qbeg != s.rbeg - t.rbeg) break;
    }
    return i == cn;
}

// the region's seed coverage and band once both extensions are done
DEV void seed_finish(Reg &a, const Seed *seeds, int cn, int aw0, int aw1, int slen)
{
    a.seedcov = 0;
    for (int i2 = 0; i2 < cn; ++i2) {
        const Seed &t = seeds[i2];
        if (t.qbeg >= a.qb && t.qbeg + t.len <= a.qe && t.rbeg >= a.rb && t.rbeg + t.len <= a.re) a.seedcov += t.len;
    }
    a.w = aw0 > aw1 ? aw0 : aw1;
    a.seedlen0 = slen;
}

template <class EH, class QM, int S>
DEV void chain2aln(const DIndex &ix, const DOpts &o, int l_query, const uint8_t *q, const ChainDesc &c, const Seed *seeds,
                   const int32_t *sscore, ExtCtx<S> &X, EH ehx, QM qm, uint64_t &cells, uint64_t &bases)
{
    int64_t rmax0, rmax1;
    if (c.n == 0) return;
    chain_window(ix, o, l_query, seeds, c.n, rmax0, rmax1, bases);
    const SP<uint64_t, S> srt = X.srt;
    seed_order(srt, seeds, sscore, c.n);
    for (int k = c.n - 1; k >= 0; --k) {
        const Seed s = seeds[(uint32_t)srt[k]];
        if (seed_skipped(o, l_query, X.av, X.n, srt, k, c.n, seeds, s)) { srt[k] = 0; continue; }
        if (X.n >= X.cap) { X.ovf = true; return; }
        Reg &a = X.av[X.n++];
        a = Reg{};
        int aw0, aw1, max_off0 = 0, max_off1 = 0;
        a.w = aw0 = aw1 = o.w;
        a.score = a.truesc = -1;
        a.rid = c.rid;
        if (s.qbeg) {
            int qle, tle, gtle, gscore;
            int64_t tmp = s.rbeg - rmax0;
            auto qa = qm.at(s.qbeg - 1, -1);
            TAcc ta{&ix, s.rbeg - 1, -1};
            for (int t = 0; t < 2; ++t) {
                int prev = a.score;
                aw0 = o.w << t;
                a.score = ext_call(o, s.qbeg, qa, (int)tmp, ta, o.o_del, o.e_del, o.o_ins, o.e_ins, aw0, o.pen_clip5,
                                      o.zdrop, s.len * o.a, &qle, &tle, &gtle, &gscore, &max_off0, ehx, cells);
                if (a.score == prev || max_off0 < (aw0 >> 1) + (aw0 >> 2)) break;
            }
            if (X.ovf) return;   // ring overflow: the retry pass redoes this read
            if (gscore <= 0 || gscore <= a.score - o.pen_clip5) {
                a.qb = s.qbeg - qle, a.rb = s.rbeg - tle;
                a.truesc = a.score;
            } else {
                a.qb = 0, a.rb = s.rbeg - gtle;
                a.truesc = gscore;
            }
        } else a.score = a.truesc = s.len * o.a, a.qb = 0, a.rb = s.rbeg;
        if (s.qbeg + s.len != l_query) {
            int qle, tle, gtle, gscore, sc0 = a.score;
            int qe = s.qbeg + s.len;
            int re = (int)(s.rbeg + s.len - rmax0);
            auto qa = qm.at(qe, 1);
            TAcc ta{&ix, rmax0 + re, 1};
            for (int t = 0; t < 2; ++t) {
                int prev = a.score;
                aw1 = o.w << t;
                a.score = ext_call(o, l_query - qe, qa, (int)(rmax1 - rmax0 - re), ta, o.o_del, o.e_del, o.o_ins,
                                      o.e_ins, aw1, o.pen_clip3, o.zdrop, sc0, &qle, &tle, &gtle, &gscore, &max_off1,
                                      ehx, cells);
                if (a.score == prev || max_off1 < (aw1 >> 1) + (aw1 >> 2)) break;
            }
            if (X.ovf) return;
            if (gscore <= 0 || gscore <= a.score - o.pen_clip3) {
                a.qe = qe + qle, a.re = rmax0 + re + tle;
                a.truesc += a.score - sc0;
            } else {
                a.qe = l_query, a.re = rmax0 + re + gtle;
                a.truesc += gscore - sc0;
            }
        } else a.qe = l_query, a.re = s.rbeg + s.len;
        seed_finish(a, seeds, c.n, aw0, aw1, s.len);
    }
}

template <class EHP>
DEV int patch_reg(const DIndex &ix, const DOpts &o, const uint8_t *q, const Reg &a, const Reg &b, int *_w, EHP eh,
                  uint64_t &cells, uint64_t &bases)
{
    int w, score = 0, q_s, r_s;
    double r;
    if (a.rb < ix.l_pac && b.rb >= ix.l_pac) return 0;
    if (a.qb >= b.qb || a.qe >= b.qe || a.re >= b.re) return 0;
    w = (int)((a.re - b.rb) - (a.qe - b.qb));
    w = w > 0 ? w : -w;
    r = (double)(a.re - b.rb) / (b.re - a.rb) - (double)(a.qe - b.qb) / (b.qe - a.qb);
    r = r > 0. ? r : -r;
    if (a.re < b.rb || a.qe < b.qb) {
        if (w > o.w << 1 || r >= 0.05f) return 0;
    } else if (w > o.w << 2 || r >= 0.05f * 2) return 0;
    w += a.w + b.w;
    w = w < o.w << 2 ? w : o.w << 2;
    gen_cigar2_score(ix, o, w, q, a.qb, b.qe - a.qb, a.rb, b.re, &score, eh, cells, bases);
    q_s = (int)((double)(b.qe - a.qb) / ((b.qe - b.qb) + (a.qe - a.qb)) * (b.score + a.score) + .499);
    r_s = (int)((double)(b.re - a.rb) / ((b.re - b.rb) + (a.re - a.rb)) * (b.score + a.score) + .499);
    if ((double)score / (q_s > r_s ? q_s : r_s) < 0.90f) return 0;
    *_w = w;
    return score;
}

template <int S>
DEV void permute(ExtCtx<S> &X, int n)
{
    bool ident = true;   // most region lists are already in order: skip the two copies through scratch
    for (int i = 0; i < n; ++i) ident = ident && X.idx[i] == i;
    if (ident) return;
    for (int i = 0; i < n; ++i) X.tmp[i] = X.av[X.idx[i]];
    for (int i = 0; i < n; ++i) X.av[i] = X.tmp[i];
}

template <int S>
DEV int sort_dedup_patch(const DIndex &ix, const DOpts &o, const uint8_t *q, ExtCtx<S> &X, uint64_t &cells, uint64_t &bases)
{
    int n = X.n, m, i, j;
    if (n <= 1) return n;
    Reg *a = X.av;
    for (i = 0; i < n; ++i) X.idx[i] = i;
    X.guard += ks_introsort(X.idx, n, [a](int x, int y) { return a[x].re < a[y].re; }, X.stk);
    permute(X, n);
    for (i = 0; i < n; ++i) a[i].n_comp = 1;
    for (i = 1; i < n; ++i) {
        Reg *p = &a[i];
        if (p->rid != a[i - 1].rid || p->rb >= a[i - 1].re + o.max_chain_gap) continue;
        for (j = i - 1; j >= 0 && p->rid == a[j].rid && p->rb < a[j].re + o.max_chain_gap; --j) {
            Reg *qq = &a[j];
            int64_t or_, oq, mr, mq;
            int score, w;
            if (qq->qe == qq->qb) continue;
            or_ = qq->re - p->rb;
            oq = qq->qb < p->qb ? qq->qe - p->qb : p->qe - qq->qb;
            mr = qq->re - qq->rb < p->re - p->rb ? qq->re - qq->rb : p->re - p->rb;
            mq = qq->qe - qq->qb < p->qe - p->qb ? qq->qe - qq->qb : p->qe - p->qb;
            if (or_ > o.mask_level_redun * mr && oq > o.mask_level_redun * mq) {
                if (p->score < qq->score) { p->qe = p->qb; break; }
                else qq->qe = qq->qb;
            } else if (qq->rb < p->rb && (score = patch_reg(ix, o, q, *qq, *p, &w, X.eh, cells, bases)) > 0) {
                p->n_comp += qq->n_comp + 1;
                p->seedcov = p->seedcov > qq->seedcov ? p->seedcov : qq->seedcov;
                p->sub = p->sub > qq->sub ? p->sub : qq->sub;
                p->csub = p->csub > qq->csub ? p->csub : qq->csub;
                p->qb = qq->qb, p->rb = qq->rb;
                p->truesc = p->score = score;
                p->w = w;
                qq->qb = qq->qe;
            }
        }
    }
    for (i = 0, m = 0; i < n; ++i)
        if (a[i].qe > a[i].qb) { if (m != i) a[m++] = a[i]; else ++m; }
    n = m;
    for (i = 0; i < n; ++i) X.idx[i] = i;
    X.guard += ks_introsort(X.idx, n, [a](int x, int y) {
        return a[x].score > a[y].score || (a[x].score == a[y].score && (a[x].rb < a[y].rb || (a[x].rb == a[y].rb && a[x].qb < a[y].qb)));
    }, X.stk);
    permute(X, n);
    for (i = 1; i < n; ++i)
        if (a[i].score == a[i - 1].score && a[i].rb == a[i - 1].rb && a[i].qb == a[i - 1].qb) a[i].qe = a[i].qb;
    for (i = 1, m = 1; i < n; ++i)
        if (a[i].qe > a[i].qb) { if (m != i) a[m++] = a[i]; else ++m; }
    return m;
}

template <int S>
DEV void mark_primary_se(const DOpts &o, ExtCtx<S> &X, int64_t id)
{
    int n = X.n;
    if (n == 0) return;
    Reg *a = X.av;
    for (int i = 0; i < n; ++i) {
        a[i].sub = 0; a[i].secondary = -1; a[i].hash = hash_64((uint64_t)(id + i));
        X.idx[i] = i;
    }
    X.guard += ks_introsort(X.idx, n, [a](int x, int y) {
        return a[x].score > a[y].score || (a[x].score == a[y].score && a[x].hash < a[y].hash);
    }, X.stk);
    permute(X, n);
    int tmp = o.a + o.b;
    tmp = o.o_del + o.e_del > tmp ? o.o_del + o.e_del : tmp;
    tmp = o.o_ins + o.e_ins > tmp ? o.o_ins + o.e_ins : tmp;
    const SP<int, S> z = X.idx;
    int nz = 0;
    z[nz++] = 0;
    for (int i = 1; i < n; ++i) {
        int k;
        for (k = 0; k < nz; ++k) {
            int j = z[k];
            int b_max = a[j].qb > a[i].qb ? a[j].qb : a[i].qb;
            int e_min = a[j].qe < a[i].qe ? a[j].qe : a[i].qe;
            if (e_min > b_max) {
                int min_l = a[i].qe - a[i].qb < a[j].qe - a[j].qb ? a[i].qe - a[i].qb : a[j].qe - a[j].qb;
                if (e_min - b_max >= min_l * o.mask_level) {
                    if (a[j].sub == 0) a[j].sub = a[i].score;
                    if (a[j].score - a[i].score <= tmp) ++a[j].sub_n;
                    break;
                }
            }
        }
        if (k == nz) z[nz++] = i;
        else a[i].secondary = z[k];
    }
}

template <bool LDS, int S>
__global__ void __launch_bounds__(LDS ? 64 : 256) k_extend(DIndex ix, DOpts o, Caps cp, const uint8_t *codes,
                                                           const int64_t *offs, const int32_t *sel, const int64_t *ids,
                                                           int n, const ChainDesc *chains, const Seed *seeds,
                                                           const int32_t *n_chains, Reg *regs_out, int32_t *n_regs,
                                                           uint32_t *status, uint8_t *scratch, Counters *ctr,
                                                           const int32_t *order, const int32_t *sscore, int32_t *work)
{
    const int nthr = gridDim.x * blockDim.x;
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t cells = 0, bases = 0;
    // S = 64: this wave's 64 * cp.scr_ext bytes, each array lane-interleaved; S = 1: the thread's own bytes
    const int lane = S == 1 ? 0 : (tid & 63);
    uint8_t *wb = scratch + (S == 1 ? (size_t)tid : (size_t)(tid >> 6) * 64) * (size_t)cp.scr_ext;
    ExtCtx<S> X;
    size_t off = 0;
    X.tmp = SP<Reg, S>{reinterpret_cast<Reg *>(wb) + lane};
    off += (size_t)cp.regs * S * sizeof(Reg);
    X.idx = SP<int, S>{reinterpret_cast<int *>(wb + off) + lane};
    off += (size_t)((cp.regs * 4 + 15) & ~15) * S;
    X.srt = SP<uint64_t, S>{reinterpret_cast<uint64_t *>(wb + off) + lane};
    off += (size_t)cp.seeds * S * 8;
    X.eh = SP<int2, S>{reinterpret_cast<int2 *>(wb + off) + lane};
    off += (size_t)(cp.max_len + 2) * S * sizeof(int2);
    X.stk = SP<int, S>{reinterpret_cast<int *>(wb + off) + lane};
    auto one = [&](int it) {
        const int li = order ? order[it] : it;   // reads ordered by estimated extension work (lane balance)
        n_regs[li] = 0;
        if (status[li]) return;
        const int r = read_of(sel, li);
        const uint8_t *q = codes + offs[r];
        const int len = (int)(offs[r + 1] - offs[r]);
        X.av = regs_out + (size_t)li * cp.regs;
        X.n = 0; X.cap = cp.regs; X.ovf = false;
        const ChainDesc *cd = chains + (size_t)li * cp.chains;
        const Seed *sd = seeds + (size_t)li * cp.seeds;
        const int32_t *ss = sscore ? sscore + (size_t)li * cp.seeds : nullptr;
        const int nc = n_chains[li];
        if (LDS) {
            EhSmall ehx{(int)threadIdx.x, &X.ovf};   // blockDim == 64: lane-interleaved LDS columns
            const int qoff = 64 * EXT_LDS_COLS * 4 + (int)threadIdx.x;
            for (int j = 0; j < len; ++j) g_lds_q8[qoff + j * 64] = (uint8_t)(q[j] << 2);   // stage 4 * code in LDS
            QMakeL qm{qoff};
            for (int c = 0; c < nc && !X.ovf; ++c)
                chain2aln(ix, o, len, q, cd[c], sd + cd[c].seed_off, ss ? ss + cd[c].seed_off : nullptr, X, ehx, qm, cells, bases);
        } else {
            EhG<SP<int2, S>> ehx{X.eh};
            QMakeG qm{q};
            for (int c = 0; c < nc && !X.ovf; ++c)
                chain2aln(ix, o, len, q, cd[c], sd + cd[c].seed_off, ss ? ss + cd[c].seed_off : nullptr, X, ehx, qm, cells, bases);
        }
        if (X.ovf) { status[li] |= ST_OVERFLOW; return; }
        X.n = sort_dedup_patch(ix, o, q, X, cells, bases);
        mark_primary_se(o, X, ids[r]);
        n_regs[li] = X.n;
    };
    // With a work counter each wave takes the next 64 reads of the order, heaviest first (the order is ascending in
    // estimated work): neighbouring reads carry similar work (lane balance), and the light chunks at the end fill in
    // behind the waves that drew heavy ones instead of leaving a tail.  Without one (the retry pass), a fixed stride.
    // One call site of the body either way.
    for (int it = tid;; it += nthr) {
        if (work) {
            int base = 0;
            if ((threadIdx.x & 63) == 0) base = atomicAdd(work, 64);   // one vector atomic per 64 reads
            base = __builtin_amdgcn_readfirstlane(base);
            if (base >= n) break;
            it = n - 1 - (base + (int)(threadIdx.x & 63));   // < 0 past the last read
        } else if (it >= n) break;
        if (it >= 0 && it < n) one(it);
    }
    wave_add(&ctr[STG_EXTEND].dp_cells, cells);
    wave_add(&ctr[STG_EXTEND].ref_bases, bases);
    wave_add(&ctr[STG_EXTEND].sort_guard, (unsigned long long)X.guard);
}

// ------------------------------------------------------------------------------------------------
// k_reg2aln: mem_reg2aln per region
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_reg2aln(DIndex ix, DOpts o, Caps cp, const uint8_t *codes, const int64_t *offs,
                                                 const int32_t *sel, int n, const Reg *regs, const int32_t *n_regs,
                                                 Hit *hits, uint32_t *cigars, int32_t *n_cig_read, uint32_t *status,
                                                 uint8_t *scratch, Counters *ctr)
{
    const int nthr = gridDim.x * blockDim.x;
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t cells = 0, bases = 0;
    uint8_t *sb = scratch + (size_t)tid * cp.scratch;
    int2 *eh = reinterpret_cast<int2 *>(sb);
    const size_t eh_bytes = ((size_t)(cp.max_len + 2) * sizeof(int2) + 63) & ~(size_t)63;
    uint8_t *z = sb + eh_bytes;
    const int64_t zcap = cp.scratch - (int64_t)eh_bytes;
    for (int li = tid; li < n; li += nthr) {
        n_cig_read[li] = 0;
        if (status[li]) continue;
        const int r = read_of(sel, li);
        const uint8_t *q = codes + offs[r];
        const int l_query = (int)(offs[r + 1] - offs[r]);
        const int nr = n_regs[li];
        bool ovf = false;
        int tot = 0;
        for (int g = 0; g < nr && !ovf; ++g) {
            const Reg &ar = regs[(size_t)li * cp.regs + g];
            Hit &h = hits[(size_t)li * cp.regs + g];
            uint32_t *cig = cigars + ((size_t)li * cp.regs + g) * cp.cigar;
            const int qb = ar.qb, qe = ar.qe;
            const int64_t rb = ar.rb, re = ar.re;
            int flag = ar.secondary >= 0 ? 0x100 : 0;
            int tmp = infer_bw(qe - qb, (int)(re - rb), ar.truesc, o.a, o.o_del, o.e_del);
            int w2 = infer_bw(qe - qb, (int)(re - rb), ar.truesc, o.a, o.o_ins, o.e_ins);
            w2 = w2 > tmp ? w2 : tmp;
            if (w2 > o.w) w2 = w2 < ar.w ? w2 : ar.w;
            int i = 0, score = 0, last_sc = -(1 << 30), ncig = 0;
            do {
                w2 = w2 < o.w << 2 ? w2 : o.w << 2;
                gen_cigar2(ix, o, w2, q, qb, qe - qb, rb, re, &score, eh, z, zcap, cig, cp.cigar - 2, &ncig, ovf, cells, bases);
                if (ovf) break;
                if (score == last_sc || w2 == o.w << 2) break;
                last_sc = score;
                w2 <<= 1;
            } while (++i < 3 && score < ar.truesc - o.a);
            if (ovf) break;
            int is_rev;
            int64_t pos = depos(ix, rb < ix.l_pac ? rb : re - 1, is_rev);
            (void)pos;
            if (ncig > 0) {
                if ((cig[0] & 0xf) == 2) {
                    --ncig;
                    for (int t = 0; t < ncig; ++t) cig[t] = cig[t + 1];
                } else if ((cig[ncig - 1] & 0xf) == 2) --ncig;
            }
            if (qb != 0 || qe != l_query) {
                int clip5 = is_rev ? l_query - qe : qb, clip3 = is_rev ? qb : l_query - qe;
                if (clip5) {
                    for (int t = ncig; t > 0; --t) cig[t] = cig[t - 1];
                    cig[0] = (uint32_t)clip5 << 4 | 3;
                    ++ncig;
                }
                if (clip3) cig[ncig++] = (uint32_t)clip3 << 4 | 3;
            }
            h.rb = rb; h.re = re; h.qb = qb; h.qe = qe; h.rid = ar.rid; h.score = ar.score; h.flag = flag;
            h.is_rev = is_rev; h.n_cigar = ncig; h.pad = 0;
            tot += ncig;
        }
        if (ovf) { status[li] |= ST_OVERFLOW; continue; }
        n_cig_read[li] = tot;
    }
    wave_add(&ctr[STG_REG2ALN].dp_cells, cells);
    wave_add(&ctr[STG_REG2ALN].ref_bases, bases);
}

// ------------------------------------------------------------------------------------------------
// packing: per-read counts from the main or the retry workspace, then scatter into bsq_hits
// ------------------------------------------------------------------------------------------------
struct SlotView {
    const Hit *hits; const uint32_t *cigars; const int32_t *n_regs; const int32_t *n_cig; Caps cp;
};

__global__ void k_counts(int n, SlotView mv, SlotView rv, const int32_t *retry_slot, const uint32_t *status,
                         int64_t *cnt_hits, int64_t *cnt_cig, unsigned long long *unresolved)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int rs = retry_slot ? retry_slot[i] : -1;
    if (rs >= 0) {
        cnt_hits[i] = rv.n_regs[rs];
        cnt_cig[i] = rv.n_cig[rs];
    } else {
        if (status[i]) atomicAdd(unresolved, 1ull);
        cnt_hits[i] = status[i] ? 0 : mv.n_regs[i];
        cnt_cig[i] = status[i] ? 0 : mv.n_cig[i];
    }
}

__global__ void k_pack(int n, SlotView mv, SlotView rv, const int32_t *retry_slot, const int64_t *off_hits,
                       const int64_t *off_cig, const int64_t *ann_off, const int64_t *ann_id, bsq_hit *out,
                       uint32_t *out_cig, int read_base, int64_t cig_base)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int rs = retry_slot ? retry_slot[i] : -1;
    const SlotView &v = rs >= 0 ? rv : mv;
    const int slot = rs >= 0 ? rs : i;
    const int nh = rs >= 0 ? rv.n_regs[rs] : (int)(off_hits[i + 1] - off_hits[i]);
    int64_t oc = off_cig[i];
    for (int g = 0; g < nh; ++g) {
        const Hit &h = v.hits[(size_t)slot * v.cp.regs + g];
        bsq_hit &b = out[off_hits[i] + g];
        const int64_t roff = ann_off[h.rid];
        b.ref_id = ann_id[h.rid];
        b.rb = h.rb; b.re = h.re;
        b.ref_match_start = (int32_t)(h.rb - roff);
        b.ref_match_end = (int32_t)(h.re - roff);
        b.ref_match_len = (int32_t)(h.re - h.rb);
        b.qb = h.qb; b.qe = h.qe; b.score = h.score; b.rid = h.rid;
        b.is_primary = (h.flag & 0x100) == 0; b.is_secondary = (h.flag & 0x100) != 0; b.is_reverse = h.is_rev != 0;
        b.pad0 = 0;
        b.read_index = read_base + i;   // batch-wide read and CIGAR-arena positions
        b.cigar_off = (uint32_t)(cig_base + oc); b.n_cigar = (uint32_t)h.n_cigar;
        static_assert(sizeof(bsq_hit) == 72, "bsq_hit layout");
        reinterpret_cast<uint32_t *>(&b)[17] = 0;   // trailing padding: records are compared byte for byte
        const uint32_t *src = v.cigars + ((size_t)slot * v.cp.regs + g) * v.cp.cigar;
        for (int t = 0; t < h.n_cigar; ++t) out_cig[oc + t] = src[t];
        oc += h.n_cigar;
    }
}

__global__ void k_collect_overflow(int n, const uint32_t *status, int32_t *list, int32_t *count)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (status[i] & ST_OVERFLOW) {
        int k = atomicAdd(count, 1);
        list[k] = i;
    }
}

}  // namespace bsq

// ------------------------------------------------------------------------------------------------
// host-side launchers (called from bsq_api.cpp)
// ------------------------------------------------------------------------------------------------
namespace bsq {

// seeding-only output (bsq_batch_intervals): per-read interval counts (0 for reads left to the retry pass)
// and compaction of the main-pass interval slots into one array
__global__ void k_intv_counts(int n, const int32_t *__restrict__ n_intv, const uint32_t *__restrict__ status,
                              int64_t *__restrict__ cnt)
{
    const int li = blockIdx.x * blockDim.x + threadIdx.x;
    if (li < n) cnt[li] = status[li] ? 0 : n_intv[li];
    if (li == n) cnt[n] = 0;
}

__global__ void k_intv_pack(int n, int cap, const Intv *__restrict__ slots, const int32_t *__restrict__ n_intv,
                            const uint32_t *__restrict__ status, const int64_t *__restrict__ off,
                            uint64_t *__restrict__ out)
{
    const int li = blockIdx.x * blockDim.x + threadIdx.x;
    if (li >= n || status[li]) return;
    const SP<const Intv> a{slots + intv_slot_at_d(li, 0, cap)};
    uint64_t *d = out + 4 * (size_t)off[li];
    for (int k = 0; k < n_intv[li]; ++k) {
        d[4 * k + 0] = a[k].x[0]; d[4 * k + 1] = a[k].x[1]; d[4 * k + 2] = a[k].x[2]; d[4 * k + 3] = a[k].info;
    }
}

hipError_t launch_intv_counts(hipStream_t st, int n, const int32_t *n_intv, const uint32_t *status, int64_t *cnt)
{
    hipLaunchKernelGGL(k_intv_counts, dim3((n + 1 + 255) / 256), dim3(256), 0, st, n, n_intv, status, cnt);
    return hipGetLastError();
}

hipError_t launch_intv_pack(hipStream_t st, int n, int cap, const Intv *slots, const int32_t *n_intv,
                            const uint32_t *status, const int64_t *off, uint64_t *out)
{
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_intv_pack, dim3((n + 255) / 256), dim3(256), 0, st, n, cap, slots, n_intv, status, off, out);
    return hipGetLastError();
}

hipError_t launch_smem(int grid, hipStream_t st, const DIndex &ix, const DOpts &o, const Caps &cp, const uint8_t *codes,
                       const int64_t *offs, const int32_t *sel, int n, Intv *intv, int32_t *n_intv, uint32_t *status,
                       uint8_t *scratch, Counters *ctr)
{
    hipLaunchKernelGGL(k_smem, dim3(grid), dim3(256), 0, st, ix, o, cp, codes, offs, sel, n, intv, n_intv, status, scratch, ctr);
    return hipGetLastError();
}

hipError_t launch_chain(int grid, hipStream_t st, const DIndex &ix, const DOpts &o, const Caps &cp, const int64_t *offs,
                        const int32_t *sel, int n, const Intv *intv, const int32_t *n_intv, ChainDesc *chains,
                        Seed *seeds, int32_t *n_chains, uint32_t *status, uint8_t *scratch, Counters *ctr)
{
    if (sel) {   // retry workspaces: a few reads per launch, contiguous per-thread scratch
        hipLaunchKernelGGL(k_chain<1>, dim3(grid), dim3(256), 0, st, ix, o, cp, offs, sel, n, intv, n_intv, chains, seeds,
                           n_chains, status, scratch, ctr, 0);
        return hipGetLastError();
    }
    // main pass: the reads whose chaining state fits the LDS share (nearly all), then k_chain<64> on the rest
    // (BSQ_CHAIN_SCRATCH=1: k_chain<64> on every read, for A/B runs and tests/test_gpu_chain.py)
    const char *cs_env = getenv("BSQ_CHAIN_SCRATCH");
    const bool scratch_only = cs_env && atoi(cs_env) == 1;
    if (!scratch_only && n > 0)
        hipLaunchKernelGGL(k_chain_s, dim3((n + 63) / 64), dim3(64), (size_t)CsLds::BYTES, st, ix, o, cp, offs, n, intv,
                           n_intv, chains, seeds, n_chains, status, ctr);
    hipLaunchKernelGGL(k_chain<64>, dim3(grid), dim3(256), 0, st, ix, o, cp, offs, sel, n, intv, n_intv, chains, seeds,
                       n_chains, status, scratch, ctr, scratch_only ? 0 : 1);
    return hipGetLastError();
}

// Sort key of a read for the extension stage: its number of chains, then the number of sides its first extended seed
// (the first chain's top seed in mem_chain2aln's order: largest score, then largest index) extends to, then that
// seed's left extent in 8-base buckets, then the estimated DP work (the query bases outside each chain's longest
// seed, summed over chains: ksw_extend2 runs ~one row per such base).
// Ordering by chain count first cut k_extend from 10.4 to 8.6 ms per 1M C3 reads (ordering by the DP estimate
// alone, or by chains, then seeds, then the estimate, left lanes of a wave in different seed loops).  The sides
// (round 5): mem_chain2aln's left and right extensions are two loops one after the other, each as long as its
// longest lane, so a wave mixing reads extended only to the left with reads extended only to the right (or on both
// sides) runs both loops at full length with half the lanes idle in each.  The left extent keeps left-only reads
// (extent >= 8) apart from right-only ones (0) and orders the two-sided reads' left calls; the estimate then orders
// the rest by rows.  tools/ext_model.py (the oracle's per-row trace of 4,096 C3 reads) puts this key at 0.72 of the
// previous one's lockstep time; lone 1M-read C3 launches measured extension 5.50 -> 4.70-4.82 ms, C4 76.1 -> 63.4 ms
// (profiles/r05/ext_key/).  Keyed instead by which sides (left only / right only / both) and the longer extent in
// 4-base buckets (model 0.67): 4.92-4.95 ms at C3, 62.2 ms at C4 -- not kept.
__global__ void k_ext_key(const Caps cp, const int64_t *__restrict__ offs, const int32_t *__restrict__ sel, int n,
                          const ChainDesc *__restrict__ chains, const Seed *__restrict__ seeds,
                          const int32_t *__restrict__ n_chains, const uint32_t *__restrict__ status,
                          const int32_t *__restrict__ sscore, uint32_t *__restrict__ key, int32_t *__restrict__ idx)
{
    const int li = blockIdx.x * blockDim.x + threadIdx.x;
    if (li >= n) return;
    uint32_t est = 0, sides = 0, lb = 0;
    if (!status[li]) {
        const int r = read_of(sel, li);
        const int len = (int)(offs[r + 1] - offs[r]);
        const ChainDesc *cd = chains + (size_t)li * cp.chains;
        const Seed *sd = seeds + (size_t)li * cp.seeds;
        const int32_t *ss = sscore ? sscore + (size_t)li * cp.seeds : nullptr;
        const int nc = n_chains[li];
        for (int c = 0; c < nc; ++c) {
            int best = 0;
            for (int k = 0; k < cd[c].n; ++k) best = best > sd[cd[c].seed_off + k].len ? best : sd[cd[c].seed_off + k].len;
            est += (uint32_t)(len > best ? len - best : 0) + 4u;
        }
        if (nc > 0 && cd[0].n > 0) {
            int top = 0, ts = -1;
            for (int k = 0; k < cd[0].n; ++k) {   // seed_order's last entry: (score, index) largest
                const int sc = ss ? ss[cd[0].seed_off + k] : sd[cd[0].seed_off + k].len;
                if (sc >= ts) { ts = sc; top = k; }
            }
            const Seed &s = sd[cd[0].seed_off + top];
            sides = (uint32_t)(s.qbeg > 0) + (uint32_t)(s.qbeg + s.len != len);
            lb = (uint32_t)(s.qbeg >> 3) < 63u ? (uint32_t)(s.qbeg >> 3) : 63u;
        }
    }
    const uint32_t nc2 = status[li] ? 0u : (uint32_t)(n_chains[li] < 63 ? n_chains[li] : 63);
    key[li] = nc2 << 24 | sides << 22 | lb << 16 | (est < 65535u ? est : 65535u);
    idx[li] = li;
}

hipError_t launch_ext_key(hipStream_t st, const Caps &cp, const int64_t *offs, const int32_t *sel, int n,
                          const ChainDesc *chains, const Seed *seeds, const int32_t *n_chains, const uint32_t *status,
                          const int32_t *sscore, uint32_t *key, int32_t *idx)
{
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_ext_key, dim3((n + 255) / 256), dim3(256), 0, st, cp, offs, sel, n, chains, seeds, n_chains,
                       status, sscore, key, idx);
    return hipGetLastError();
}

hipError_t launch_extend(int grid, hipStream_t st, const DIndex &ix, const DOpts &o, const Caps &cp, const uint8_t *codes,
                         const int64_t *offs, const int32_t *sel, const int64_t *ids, int n, const ChainDesc *chains,
                         const Seed *seeds, const int32_t *n_chains, Reg *regs, int32_t *n_regs, uint32_t *status,
                         uint8_t *scratch, Counters *ctr, const int32_t *order, const int32_t *sscore, int32_t *work)
{
    // LDS row storage when the u16 bound holds: h, e <= h0 + qlen*max with h0 <= len*a (+ a left score)
    // and the 64-column ring holds the band: ksw_extend2 clamps w to max_ins/max_del (ksw.c), which for
    // cheap gap extensions (e.g. e_del = 1) leaves bands up to 2w+1 = 201 columns wide.  The retry pass
    // (sel != nullptr) always takes the global-row kernel, so a read whose window outgrew the ring
    // completes there.
    const int end_bonus = o.pen_clip3 > o.pen_clip5 ? o.pen_clip3 : o.pen_clip5;
    const int mx = o.mat_max > 0 ? o.mat_max : 0;
    int wb = o.w;
    wb = std::min(wb, std::max(1, (int)((double)(cp.max_len * mx + end_bonus - o.o_ins) / o.e_ins + 1.)));
    wb = std::min(wb, std::max(1, (int)((double)(cp.max_len * mx + end_bonus - o.o_del) / o.e_del + 1.)));
    auto in4 = [](int v) { return v >= -8 && v <= 7; };   // the profile's 4-bit score fields
    const bool lds = !sel && cp.max_len <= 200 && 2 * wb + 2 < 63 && in4(o.mat_match) && in4(o.mat_mismatch) &&
                     in4(o.mat_amb) &&
                     (int64_t)cp.max_len * (2 * (int64_t)o.a + 2 * o.mat_max) + o.pen_clip3 + o.pen_clip5 < 60000;
    // Contiguous per-thread scratch (S = 1).  The lane-interleaved layout (S = 64, as k_chain's) measured slower
    // here: lone 1M-read launch 7.0 ms against 6.67 ms, PMC fetch + write 1.17 GB against 1.28 GB -- the kernel is
    // bound by VALU issue under divergence, not by its scratch traffic.
    if (work) {
        const hipError_t e = hipMemsetAsync(work, 0, sizeof(int32_t), st);
        if (e != hipSuccess) return e;
    }
    if (lds) {
        const size_t sh = (size_t)64 * EXT_LDS_COLS * 4 + (size_t)64 * (cp.max_len + 2);
        hipLaunchKernelGGL((k_extend<true, 1>), dim3(grid * 4), dim3(64), sh, st, ix, o, cp, codes, offs, sel, ids, n,
                           chains, seeds, n_chains, regs, n_regs, status, scratch, ctr, order, sscore, work);
    } else {
        hipLaunchKernelGGL((k_extend<false, 1>), dim3(grid), dim3(256), 0, st, ix, o, cp, codes, offs, sel, ids, n, chains,
                           seeds, n_chains, regs, n_regs, status, scratch, ctr, order, sscore, work);
    }
    return hipGetLastError();
}

hipError_t launch_reg2aln(int grid, hipStream_t st, const DIndex &ix, const DOpts &o, const Caps &cp, const uint8_t *codes,
                          const int64_t *offs, const int32_t *sel, int n, const Reg *regs, const int32_t *n_regs,
                          Hit *hits, uint32_t *cigars, int32_t *n_cig, uint32_t *status, uint8_t *scratch, Counters *ctr)
{
    hipLaunchKernelGGL(k_reg2aln, dim3(grid), dim3(256), 0, st, ix, o, cp, codes, offs, sel, n, regs, n_regs, hits, cigars,
                       n_cig, status, scratch, ctr);
    return hipGetLastError();
}

hipError_t launch_counts(hipStream_t st, int n, const SlotView &mv, const SlotView &rv, const int32_t *retry_slot,
                         const uint32_t *status, int64_t *cnt_hits, int64_t *cnt_cig, unsigned long long *unresolved)
{
    hipLaunchKernelGGL(k_counts, dim3((n + 255) / 256), dim3(256), 0, st, n, mv, rv, retry_slot, status, cnt_hits, cnt_cig,
                       unresolved);
    return hipGetLastError();
}

hipError_t launch_pack(hipStream_t st, int n, const SlotView &mv, const SlotView &rv, const int32_t *retry_slot,
                       const int64_t *off_hits, const int64_t *off_cig, const int64_t *ann_off, const int64_t *ann_id,
                       bsq_hit *out, uint32_t *out_cig, int read_base, int64_t cig_base)
{
    hipLaunchKernelGGL(k_pack, dim3((n + 255) / 256), dim3(256), 0, st, n, mv, rv, retry_slot, off_hits, off_cig, ann_off,
                       ann_id, out, out_cig, read_base, cig_base);
    return hipGetLastError();
}

// The exchange's wire form (bsq_internal.h WireHit): one thread per read writes its hit count and its hits' 32-B
// records; the read holding the batch's first hit writes the header {read_base, cig_base}.
__global__ void k_wire_pack(int32_t n_reads, const int64_t *off, const bsq_hit *hits, uint8_t *off_part, WireHit *wire)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_reads) return;
    const int64_t a = off[i], b = off[i + 1];
    reinterpret_cast<int32_t *>(off_part + kWireHead)[i] = (int32_t)(b - a);
    if (a == off[0] && b > a) {   // the first read with hits: its first hit is hits[0]
        const bsq_hit &h = hits[0];
        reinterpret_cast<int64_t *>(off_part)[0] = (int64_t)h.read_index - i;
        reinterpret_cast<int64_t *>(off_part)[1] = (int64_t)h.cigar_off;
    }
    for (int64_t g = a; g < b; ++g) {
        const bsq_hit &h = hits[g - off[0]];
        WireHit w;
        w.rb = h.rb; w.len = (int32_t)(h.re - h.rb); w.qb = h.qb; w.qe = h.qe; w.score = h.score; w.rid = h.rid;
        w.ncig = h.n_cigar | (uint32_t)(h.is_primary != 0) << 29 | (uint32_t)(h.is_secondary != 0) << 30 |
                 (uint32_t)(h.is_reverse != 0) << 31;
        wire[g - off[0]] = w;
    }
}

int launch_wire_pack(void *st, int32_t n_reads, const int64_t *off, const bsq_hit *hits, uint8_t *off_part, WireHit *wire)
{
    hipStream_t s = static_cast<hipStream_t>(st);
    if (hipMemsetAsync(off_part, 0, kWireHead, s) != hipSuccess) return BSQ_E_HIP;
    if (n_reads > 0)
        hipLaunchKernelGGL(k_wire_pack, dim3((n_reads + 255) / 256), dim3(256), 0, s, n_reads, off, hits, off_part, wire);
    return hipGetLastError() == hipSuccess ? BSQ_OK : BSQ_E_HIP;
}

__global__ void k_add_base(int64_t *v, int n, int64_t base)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] += base;
}

hipError_t launch_add_base(hipStream_t st, int64_t *v, int n, int64_t base)
{
    if (n <= 0 || base == 0) return hipSuccess;
    hipLaunchKernelGGL(k_add_base, dim3((n + 255) / 256), dim3(256), 0, st, v, n, base);
    return hipGetLastError();
}

hipError_t launch_collect_overflow(hipStream_t st, int n, const uint32_t *status, int32_t *list, int32_t *count)
{
    hipLaunchKernelGGL(k_collect_overflow, dim3((n + 255) / 256), dim3(256), 0, st, n, status, list, count);
    return hipGetLastError();
}

}  // namespace bsq

#ifdef BSQ_ISA_PROBE   // tools/hang_isa.sh: k_extend with lane-interleaved scratch, for the ISA comparison of DESIGN.md 3
template __global__ void bsq::k_extend<true, 64>(bsq::DIndex, bsq::DOpts, bsq::Caps, const uint8_t *, const int64_t *, const int32_t *,
                                            const int64_t *, int, const bsq::ChainDesc *, const bsq::Seed *, const int32_t *,
                                            bsq::Reg *, int32_t *, uint32_t *, uint8_t *, bsq::Counters *, const int32_t *,
                                            const int32_t *, int32_t *);
#endif
