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
// Restates algorithms of BWA (lh3/bwa, Apache-2.0) and klib (MIT) for bit-exact results; see NOTICE.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdlib>

#include "bsq_device.h"

namespace bsq {

#define DEV __device__ __forceinline__

template <typename X>
struct FM {
    const OccBlock *occ;
    const OccBlock32 *occ32;   // 64-base blocks (superblock-relative counts when X is u64)
    const SupBlock *sup;       // X = u64: superblock counts
    const uint4 *kt;   // k-mer interval table (bsq_device.h DIndex::kmer), depth K (0 = none)
    int K;
    // table entry idx: (x[0], x[2], x[1], 0) as 4 x u32 (16 B) or, for 64-bit rows, 4 x u64 (32 B); (x[0], x[2])
    // first, so the backward phase (which never reads x[1]) takes one 8-B (16-B) load per entry
    template <typename Z>
    DEV void kget(uint32_t idx, X &a0, X &a1, Z &a2) const
    {
        if constexpr (sizeof(X) == 4) {
            const uint4 e = kt[idx];
            a0 = e.x; a2 = (Z)e.y; a1 = e.z;
        } else {
            const ulonglong2 *p = reinterpret_cast<const ulonglong2 *>(kt) + 2 * (size_t)idx;
            const ulonglong2 u = p[0], v = p[1];
            a0 = u.x; a2 = (Z)u.y; a1 = v.x;
        }
    }
    template <typename Z>
    DEV void kget02(uint32_t idx, X &a0, Z &a2) const
    {
        if constexpr (sizeof(X) == 4) {
            const uint2 e = reinterpret_cast<const uint2 *>(kt)[2 * (size_t)idx];
            a0 = e.x; a2 = (Z)e.y;
        } else {
            const ulonglong2 u = reinterpret_cast<const ulonglong2 *>(kt)[2 * (size_t)idx];
            a0 = u.x; a2 = (Z)u.y;
        }
    }
    DEV X kget1(uint32_t idx) const
    {
        if constexpr (sizeof(X) == 4) return reinterpret_cast<const uint32_t *>(kt)[4 * (size_t)idx + 2];
        else return reinterpret_cast<const uint64_t *>(kt)[4 * (size_t)idx + 2];
    }
    X l2_0, l2_1, l2_2, l2_3, l2_4, primary;
    // the text T = pac || revcomp(pac) and its suffix array, for walking a unique interval along the text
    const uint8_t *pac;
    int64_t l_pac;
    const uint32_t *sa32;
    const uint64_t *sa64;
    DEV int64_t sa(X row) const { return sa64 ? (int64_t)sa64[row] : (int64_t)sa32[row]; }
    DEV int tbase(int64_t t) const
    {
        const int64_t f = t < l_pac ? t : (l_pac << 1) - 1 - t;
        const int b = (pac[f >> 2] >> ((~f & 3) << 1)) & 3;
        return t < l_pac ? b : 3 - b;
    }
    // branch-free select (a nested conditional compiles to divergent branches around every extension)
    DEV X L2(int c) const
    {
        const X a = (c & 1) ? l2_1 : l2_0, b = (c & 1) ? l2_3 : l2_2, r = (c & 2) ? b : a;
        return (c & 4) ? l2_4 : r;
    }
};

// rank of base c and of all bases > c in rows [0, k] (k = -1 -> 0), from a loaded occ block: the two
// sums bwt_extend needs for one base.  Selection is by bit masks so every word of the block is used
// unconditionally (a select chain lets the compiler narrow the block load and sink parts of it into
// branches, serialising the two blocks' round trips).
template <typename X>
DEV void occ_c(const uint4 (&w)[4], X k, bool none, int c, X &cc, X &cg)
{
    const uint32_t r = (uint32_t)(k & 127) + 1;
    const uint64_t h0 = (uint64_t)w[2].y << 32 | w[2].x, h1 = (uint64_t)w[2].w << 32 | w[2].z;
    const uint64_t l0 = (uint64_t)w[3].y << 32 | w[3].x, l1 = (uint64_t)w[3].w << 32 | w[3].z;
    const uint64_t m0 = r >= 64 ? ~0ull : ((1ull << r) - 1);
    const uint64_t m1 = r >= 128 ? ~0ull : (r > 64 ? ((1ull << (r - 64)) - 1) : 0ull);
    // base b is (h, l) = (b >> 1, b & 1): plane of c, and plane of bases > c
    const uint64_t fh = (c & 2) ? 0ull : ~0ull, fl = (c & 1) ? 0ull : ~0ull;
    const uint64_t any = c == 0 ? ~0ull : 0ull;
    const uint64_t ah0 = c < 2 ? ~0ull : (c == 2 ? l0 : 0ull), ah1 = c < 2 ? ~0ull : (c == 2 ? l1 : 0ull);
    const uint32_t nc = __popcll((h0 ^ fh) & (l0 ^ fl) & m0) + __popcll((h1 ^ fh) & (l1 ^ fl) & m1);
    const uint32_t ng = __popcll(((h0 & ah0) | (l0 & any)) & m0) + __popcll(((h1 & ah1) | (l1 & any)) & m1);
    X b0, b1, b2, b3;
    if (sizeof(X) == 4) {
        b0 = (X)w[0].x; b1 = (X)w[0].z; b2 = (X)w[1].x; b3 = (X)w[1].z;
    } else {
        b0 = (X)((uint64_t)w[0].y << 32 | w[0].x); b1 = (X)((uint64_t)w[0].w << 32 | w[0].z);
        b2 = (X)((uint64_t)w[1].y << 32 | w[1].x); b3 = (X)((uint64_t)w[1].w << 32 | w[1].z);
    }
    const X live = none ? (X)0 : ~(X)0;
    const X s0 = -(X)(c == 0), s1 = -(X)(c == 1), s2 = -(X)(c == 2), s3 = -(X)(c == 3);
    cc = (((b0 & s0) | (b1 & s1) | (b2 & s2) | (b3 & s3)) + nc) & live;
    cg = ((b1 & s0) + (b2 & (s0 | s1)) + (b3 & (s0 | s1 | s2)) + ng) & live;
}

// The same two sums from a 64-base OccBlock32 (w[0] = counts, w[1] = hi/lo planes): one word per plane.
// Rows [0, k & 63] of the block are the low (k & 63) + 1 bits: one 64-bit shift of ~0 by 63 - (k & 63) = ~k & 63
// (no r == 64 case: 3 instructions instead of 8 per block end, round 5).
DEV void occ_c32(const uint4 (&w)[2], uint32_t k, bool none, int c, uint32_t &cc, uint32_t &cg)
{
    const uint64_t h = (uint64_t)w[1].y << 32 | w[1].x, l = (uint64_t)w[1].w << 32 | w[1].z;
    const uint64_t m = ~0ull >> (~k & 63u);
    const uint64_t fh = (c & 2) ? 0ull : ~0ull, fl = (c & 1) ? 0ull : ~0ull;
    const uint64_t any = c == 0 ? ~0ull : 0ull;
    const uint64_t ah = c < 2 ? ~0ull : (c == 2 ? l : 0ull);
    const uint32_t nc = __popcll((h ^ fh) & (l ^ fl) & m);
    const uint32_t ng = __popcll(((h & ah) | (l & any)) & m);
    const uint32_t live = none ? 0u : ~0u;
    // (the count of c stays a mask-and-or: written as a select chain, the compiler turned it into a dynamically
    // indexed copy of the block in scratch memory -- 144 B per lane, seeding 2.8x slower)
    const uint32_t s0 = -(uint32_t)(c == 0), s1 = -(uint32_t)(c == 1), s2 = -(uint32_t)(c == 2), s3 = -(uint32_t)(c == 3);
    cc = (((w[0].x & s0) | (w[0].y & s1) | (w[0].z & s2) | (w[0].w & s3)) + nc) & live;
    cg = ((w[0].y & s0) + (w[0].z & (s0 | s1)) + (w[0].w & (s0 | s1 | s2)) + ng) & live;
}

// 64-bit rows: the same two sums from a superblock-relative 32-B block plus its superblock's counts (the
// superblock table is small and cache-resident; its two words load beside the block).  Half the block bytes
// and registers of the 128-base 64-B OccBlock, and one 64-bit plane word per popcount instead of two.
DEV void occ_c32w(const uint4 (&w)[2], uint64_t k, bool none, int c, const SupBlock *sb, uint64_t &cc, uint64_t &cg)
{
    uint32_t rc, rg;
    occ_c32(w, (uint32_t)k, false, c, rc, rg);
    const uint64_t live = none ? 0ull : ~0ull;
    cc = (sb->cnt[c] + rc) & live;
    cg = (sb->gt[c] + rg) & live;
}

// 64-bit rows: a rank block of the 3 GB table (random, outside every cache).  Plain loads: nontemporal ones (to keep
// the k-mer table cached) measured 21 % slower at C4.
DEV void ld_wblk(const uint4 *p, uint4 (&w)[2])
{
    w[0] = p[0]; w[1] = p[1];
}

// bwt_extend restricted to base c: returns (x_new_side, x_other_side, x2).  `a` is the interval end
// used for the rank queries (x[1] forward, x[0] backward), `o` the other one.
// Z: the type of interval sizes x[2] -- u32 also for 64-bit rows when l_pac < 2^32 (an interval size is at most
// the count of one base, <= l_pac), which takes a quarter of the u64 kernel's registers and list bytes off it.
template <typename X, typename Z>
DEV void extend1(const FM<X> &fm, X a, X o, Z x2, int c, X &na, X &no, Z &nx2, uint64_t &nblk)
{
    const X k = a - 1, l = a - 1 + (X)x2;
    const bool knone = k == (X)-1;
    const X kk = k - (k >= fm.primary), ll = l - (l >= fm.primary);
    X kc, kg, lc, lg;
    if constexpr (sizeof(X) == 4) {
        const uint4 *pk = reinterpret_cast<const uint4 *>(fm.occ32 + (knone ? 0 : (kk >> 6)));
        const uint4 *pl = reinterpret_cast<const uint4 *>(fm.occ32 + (ll >> 6));
        uint4 wk[2], wl[2];
        wk[0] = pk[0]; wk[1] = pk[1];
        wl[0] = pl[0]; wl[1] = pl[1];
        occ_c32(wk, kk, knone, c, kc, kg);
        occ_c32(wl, ll, false, c, lc, lg);
        nblk += (knone || (kk >> 6) == (ll >> 6)) ? 1 : 2;
    } else {
        // The two ends of an interval almost always share a superblock (2^22 rows): then the interval's size and
        // the rank difference of the bases > c are differences of the blocks' relative u32 counts, and only the
        // k end's cnt[c] (for the new x0) is read from the superblock table.
        const uint4 *pk = reinterpret_cast<const uint4 *>(fm.occ32 + (knone ? 0 : (kk >> 6)));
        const uint4 *pl = reinterpret_cast<const uint4 *>(fm.occ32 + (ll >> 6));
        constexpr int SS = 6 + SUP_SHIFT;
        const X sbk = knone ? 0 : (kk >> SS), sbl = ll >> SS;
        uint4 wk[2], wl[2];
        ld_wblk(pk, wk);
        ld_wblk(pl, wl);
        const X base_k = fm.sup[sbk].cnt[c];
        uint32_t rck, rgk, rcl, rgl;
        occ_c32(wk, (uint32_t)kk, knone, c, rck, rgk);
        occ_c32(wl, (uint32_t)ll, false, c, rcl, rgl);
        nblk += (knone || (kk >> 6) == (ll >> 6)) ? 1 : 2;
        const X kc0 = knone ? (X)0 : base_k + rck;
        X dgt;
        Z dx2;
        if (!knone && sbk == sbl) {
            dx2 = (Z)(rcl - rck);
            dgt = (X)(rgl - rgk);
        } else {
            const SupBlock *sl = fm.sup + sbl;
            const X lc1 = sl->cnt[c] + rcl, lg1 = sl->gt[c] + rgl;
            const X kg1 = knone ? (X)0 : fm.sup[sbk].gt[c] + rgk;
            dx2 = (Z)(lc1 - kc0);
            dgt = lg1 - kg1;
        }
        na = fm.L2(c) + 1 + kc0;
        nx2 = dx2;
        no = o + (X)(a <= fm.primary && a + (X)x2 - 1 >= fm.primary) + dgt;
        return;
    }
    na = fm.L2(c) + 1 + kc;
    nx2 = (Z)(lc - kc);
    no = o + (X)(a <= fm.primary && a + (X)x2 - 1 >= fm.primary) + (lg - kg);
}

// Two independent backward extensions by the same base (entries of one bwt_smem1 backward level);
// all four occ blocks are in flight together.  Backward extensions only need (x[0], x[2]).
template <typename X, typename Z>
DEV void ext_back2(const FM<X> &fm, X a0, Z a2, X b0, Z b2, bool da, bool hb, int c, X &ra0, Z &ra2, X &rb0, Z &rb2,
                   uint64_t &nblk)
{
    const X ka = a0 - 1, la = a0 - 1 + (X)a2;
    const X kb = hb ? b0 - 1 : ka, lb = hb ? b0 - 1 + (X)b2 : la;
    const bool kan = ka == (X)-1, kbn = kb == (X)-1;
    const X kka = ka - (ka >= fm.primary), lla = la - (la >= fm.primary);
    const X kkb = kb - (kb >= fm.primary), llb = lb - (lb >= fm.primary);
    X kc, kg, lc, lg;
    if constexpr (sizeof(X) == 4) {
        const uint4 *p0 = reinterpret_cast<const uint4 *>(fm.occ32 + (kan ? 0 : (kka >> 6)));
        const uint4 *p1 = reinterpret_cast<const uint4 *>(fm.occ32 + (lla >> 6));
        const uint4 *p2 = reinterpret_cast<const uint4 *>(fm.occ32 + (kbn ? 0 : (kkb >> 6)));
        const uint4 *p3 = reinterpret_cast<const uint4 *>(fm.occ32 + (llb >> 6));
        uint4 w0[2], w1[2], w2[2], w3[2];
        if (da) { w0[0] = p0[0]; w0[1] = p0[1]; w1[0] = p1[0]; w1[1] = p1[1]; }
        if (hb) { w2[0] = p2[0]; w2[1] = p2[1]; w3[0] = p3[0]; w3[1] = p3[1]; }
        occ_c32(w0, kka, kan, c, kc, kg);
        occ_c32(w1, lla, false, c, lc, lg);
        ra0 = fm.L2(c) + 1 + kc;
        ra2 = (Z)(lc - kc);
        occ_c32(w2, kkb, kbn, c, kc, kg);
        occ_c32(w3, llb, false, c, lc, lg);
        rb0 = fm.L2(c) + 1 + kc;
        rb2 = (Z)(lc - kc);
        if (da) nblk += (kan || (kka >> 6) == (lla >> 6)) ? 1 : 2;
        if (hb) nblk += (kbn || (kkb >> 6) == (llb >> 6)) ? 1 : 2;
    } else {
        const uint4 *p0 = reinterpret_cast<const uint4 *>(fm.occ32 + (kan ? 0 : (kka >> 6)));
        const uint4 *p1 = reinterpret_cast<const uint4 *>(fm.occ32 + (lla >> 6));
        const uint4 *p2 = reinterpret_cast<const uint4 *>(fm.occ32 + (kbn ? 0 : (kkb >> 6)));
        const uint4 *p3 = reinterpret_cast<const uint4 *>(fm.occ32 + (llb >> 6));
        constexpr int SS = 6 + SUP_SHIFT;
        // as in extend1: the size is a difference of relative counts when both ends share a superblock, and only
        // the k end's cnt[c] is read from the superblock table (backward extensions never need the gt sums)
        const X sa0 = kan ? 0 : (kka >> SS), sa1 = lla >> SS, sb0 = kbn ? 0 : (kkb >> SS), sb1 = llb >> SS;
        uint4 w0[2], w1[2], w2[2], w3[2];
        if (da) { ld_wblk(p0, w0); ld_wblk(p1, w1); }
        if (hb) { ld_wblk(p2, w2); ld_wblk(p3, w3); }
        const X base_a = fm.sup[sa0].cnt[c], base_b = fm.sup[sb0].cnt[c];
        uint32_t rk, rg_, rl;
        occ_c32(w0, (uint32_t)kka, kan, c, rk, rg_);
        occ_c32(w1, (uint32_t)lla, false, c, rl, rg_);
        const X ka0 = kan ? (X)0 : base_a + rk;
        ra0 = fm.L2(c) + 1 + ka0;
        ra2 = (!kan && sa0 == sa1) ? (Z)(rl - rk) : (Z)(fm.sup[sa1].cnt[c] + rl - ka0);
        occ_c32(w2, (uint32_t)kkb, kbn, c, rk, rg_);
        occ_c32(w3, (uint32_t)llb, false, c, rl, rg_);
        const X kb0 = kbn ? (X)0 : base_b + rk;
        rb0 = fm.L2(c) + 1 + kb0;
        rb2 = (!kbn && sb0 == sb1) ? (Z)(rl - rk) : (Z)(fm.sup[sb1].cnt[c] + rl - kb0);
        if (da) nblk += (kan || (kka >> 6) == (lla >> 6)) ? 1 : 2;
        if (hb) nblk += (kbn || (kkb >> 6) == (llb >> 6)) ? 1 : 2;
    }
}

// first entry of the k-mer table level for strings of length L: (4^L - 4) / 3
DEV uint32_t koff(int L) { return ((1u << (2 * L)) - 4u) / 3u; }

// The lane's list of (x0, x2, end) entries: entries e < cap in LDS (entry e at element offset e * stride,
// lane-interleaved), the next gcap in this read's global spill area (lists longer than the LDS share
// cost global accesses instead of a retry; the spill area is wave-interleaved too, entry g of a lane at
// [g * 64], so the lanes of a wave that spill the same entry share lines).  The LDS part is addressed by offsets into the
// dynamic LDS arrays and the spill part is read with (relaxed, wave-scope) atomic loads, so the compiler
// cannot merge the two branches' loads into one flat load through a selected pointer: flat loads of LDS
// go through the vector memory pipeline and make every wait cover both counters.
extern __shared__ uint32_t g_smem_u32[];
extern __shared__ uint64_t g_smem_u64[];
extern __shared__ uint16_t g_smem_u16[];
template <typename X> DEV X &lds_x(int i);
template <> DEV uint32_t &lds_x<uint32_t>(int i) { return g_smem_u32[i]; }
template <> DEV uint64_t &lds_x<uint64_t>(int i) { return g_smem_u64[i]; }
template <typename T> DEV T spill_load(const T *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT); }

template <typename X, typename Z>
struct LList {
    int x0, x2, end;   // element offsets of this lane's entry 0: x0 in X units, x2 in Z units, end in u16 units
    int stride, cap;
    X *gx0;
    Z *gx2;
    uint32_t *gend;
    int gcap;
    DEV int total() const { return cap + gcap; }
    DEV void set(int e, X a, Z b, int en)
    {
        if (e < cap) { lds_x<X>(x0 + e * stride) = a; lds_x<Z>(x2 + e * stride) = b; g_smem_u16[end + e * stride] = (uint16_t)en; }
        else { const int g = (e - cap) * 64; gx0[g] = a; gx2[g] = b; gend[g] = (uint32_t)en; }
    }
    DEV void get(int e, X &a, Z &b, int &en) const
    {
        if (e < cap) { a = lds_x<X>(x0 + e * stride); b = lds_x<Z>(x2 + e * stride); en = g_smem_u16[end + e * stride]; }
        else { const int g = (e - cap) * 64; a = spill_load(gx0 + g); b = spill_load(gx2 + g); en = (int)spill_load(gend + g); }
    }
};

struct OutSlot {   // the read's output intervals (global, wave-interleaved), mem grows from the front, mem1 from the back
    SP<Intv> a;
    int n, cap, n1;
};

template <typename X, typename Z, typename Q>
DEV int smem1_lds(const FM<X> &fm, int len, Q q, int x, int min_intv, LList<X, Z> &L, OutSlot &S,
                  bool &ovf, uint64_t &nblk, uint64_t &nkm)
{
    S.n1 = 0;
    if (q[x] > 3) return x + 1;
    if (min_intv < 1) min_intv = 1;
    int c0 = q[x];
    X ik0 = fm.L2(c0) + 1, ik1 = fm.L2(3 - c0) + 1;
    Z ik2 = (Z)(fm.L2(c0 + 1) - fm.L2(c0));
    int ikend = x + 1;
    int n = 0, i = x + 1;
    uint32_t fcode = (uint32_t)c0;   // code of q[x..i] while i - x + 1 <= K
    bool stop = false;               // the forward walk ended early (hole or interval below min_intv)
    {
        // Lengths 2..min(K, len - x) come from the k-mer table.  Their table rows depend only on the read's
        // bases, so every row is loaded before the first one is used (one round trip instead of K - 1);
        // the walk below then consumes them in order with the exact bookkeeping of the loop that follows.
        // (64-bit rows too: at 3 Gbp the table is a 179 MB array whose rows miss the caches as often as not,
        // and K - 1 dependent round trips per SMEM call were a fifth of the seeding kernel's time.)
        // rows preloaded: 11, or 13 for 64-bit rows (whose table is 13 deep: C4); a deeper table (kmer_depth up to
        // 15) serves lengths KM+1..K one per step below
        constexpr int KM = sizeof(X) == 8 ? 13 : 11;
        const int Kp = fm.K < KM ? fm.K : KM;
        const int Lt = Kp < len - x ? Kp : len - x;
        int cb[KM + 1];
#pragma unroll
        for (int t = 2; t <= KM; ++t) cb[t] = t <= Lt ? q[x + t - 1] : 4;
        X e0[KM + 1];
        Z e2[KM + 1];
        int nt = 1;   // bases from x covered without a hole (capped at Lt)
#pragma unroll
        for (int t = 2; t <= KM; ++t) {
            if (nt == t - 1 && cb[t] < 4) {
                fcode = fcode << 2 | (uint32_t)cb[t];
                fm.kget02(koff(t) + fcode, e0[t], e2[t]);
                nt = t;
            }
        }
        if (nt >= 2) {
            nkm += (uint64_t)(nt - 1);
            const X x1_last = fm.kget1(koff(nt) + fcode);
#pragma unroll
            for (int t = 2; t <= KM; ++t) {
                if (t <= nt && !stop) {
                    const X n0 = e0[t];
                    const Z n2 = e2[t];
                    if (n2 != ik2) {
                        if (n >= L.total()) { ovf = true; return len; }
                        L.set(n++, ik0, ik2, ikend);
                        if (n2 < (Z)min_intv) { stop = true; i = x + t - 1; }
                    }
                    if (!stop) { ik0 = n0; ik2 = n2; ikend = x + t; }
                }
            }
            ik1 = x1_last;
        }
        if (!stop) {
            i = x + nt;
            if (nt < Lt) {   // q[x + nt] is a hole: the walk stops there
                if (n >= L.total()) { ovf = true; return len; }
                L.set(n++, ik0, ik2, ikend);
                stop = true;
            }
        }
    }
    int qi = !stop && i < len ? q[i] : 0;
    for (; !stop && i < len; ++i) {
        if (ik2 == 1 && min_intv <= 1) {
            // A unique interval [x0, x0] stays [x0, x0] while the string extends along its one occurrence at
            // SA[x0] (the row of that suffix does not move) and becomes empty at the first base that differs
            // from the text (or at the text's end): walk the text instead of one rank query per base.  x[1]
            // is not read again by bwt_smem1 once the forward walk ends.
            const int64_t p = fm.sa(ik0) - x, nT = fm.l_pac << 1;
            int k = i;
            for (;;) {   // 8 bases per trip: all 16 loads issued before the first compare
                constexpr int W = 8;
                int qc[W], tc[W];
#pragma unroll
                for (int t = 0; t < W; ++t) {
                    const bool in = k + t < len && p + k + t < nT;
                    qc[t] = in ? q[k + t] : 5;
                    tc[t] = in ? fm.tbase(p + k + t) : 4;
                }
                int r = W;
#pragma unroll
                for (int t = W - 1; t >= 0; --t)
                    if (qc[t] != tc[t]) r = t;   // holes (> 3) never equal a text base; past the end 5 != 4
                k += r;
                if (r < W) break;
            }
            ikend = k;
            i = k;
            if (k < len) {   // a differing base or a hole: the interval is pushed and the walk stops
                if (n >= L.total()) { ovf = true; return len; }
                L.set(n++, ik0, ik2, ikend);
            }
            break;
        }
        const int cur = qi;
        qi = i + 1 < len ? q[i + 1] : 0;   // prefetch the next base
        if (cur < 4) {
            const int c = 3 - cur;
            X n1, n0;
            Z n2;
            fcode = fcode << 2 | (uint32_t)cur;
            if (i - x + 1 <= fm.K) {
                fm.kget(koff(i - x + 1) + fcode, n0, n1, n2);
                ++nkm;
            } else extend1(fm, ik1, ik0, ik2, c, n1, n0, n2, nblk);
            if (n2 != ik2) {
                if (n >= L.total()) { ovf = true; return len; }
                L.set(n++, ik0, ik2, ikend);
                if (n2 < (Z)min_intv) break;
            }
            ik0 = n0; ik1 = n1; ik2 = n2; ikend = i + 1;
        } else {
            if (n >= L.total()) { ovf = true; return len; }
            L.set(n++, ik0, ik2, ikend);
            break;
        }
    }
    if (i == len) {
        if (n >= L.total()) { ovf = true; return len; }
        L.set(n++, ik0, ik2, ikend);
    }
    for (int j = 0; j < (n >> 1); ++j) {   // reverse: longest match first
        X a0, b0;
        Z a2, b2;
        int ae, be;
        L.get(j, a0, a2, ae);
        L.get(n - 1 - j, b0, b2, be);
        L.set(j, b0, b2, be);
        L.set(n - 1 - j, a0, a2, ae);
    }
    int ret;
    { X d0; Z d2; L.get(0, d0, d2, ret); }
    int last_start = 0x7fffffff;
    const int K = fm.K;
    uint32_t wcode = 0;   // q[i .. i+K) packed, first base most significant (positions past the read: 0)
    for (int t = 0; t < K; ++t) wcode = wcode << 2 | (x + t < len ? (uint32_t)(q[x + t] & 3) : 0u);
    // One flat loop over (position i, entry pair j): a lane whose list at i is exhausted moves on to i - 1
    // in the same trip instead of waiting for the lane with the longest list (the nest's inner loop ran
    // to the wave's largest n at every i).  Per lane the order of work is the nest's.
    i = x - 1;
    int c = i < 0 ? -1 : (q[i] < 4 ? q[i] : -1);
    if (K > 0 && c >= 0) wcode = wcode >> 2 | (uint32_t)c << (2 * (K - 1));
    int nc = 0, j = 0;
    Z last_x2 = 0;
    for (;;) {
        {
            // entries j and j+1 are extended together (independent); bookkeeping stays in list order.
            // Compaction writes go to nc <= j, below both entries already read.
            const bool hb = j + 1 < n;
            X pa0, pb0;
            Z pa2, pb2;
            int pae, pbe;
            L.get(j, pa0, pa2, pae);
            L.get(hb ? j + 1 : j, pb0, pb2, pbe);
            X oa0 = 0, ob0 = 0;
            Z oa2 = 0, ob2 = 0;
            if (c >= 0) {
                // strings q[i .. end) of at most K bases come from the k-mer table
                const int La = pae - i, Lb = pbe - i;
                const bool ta = La <= K, tb = hb && Lb <= K;
                X ea0 = 0, eb0 = 0;
                Z ea2 = 0, eb2 = 0;
                if (ta) fm.kget02(koff(La) + (wcode >> (2 * (K - La))), ea0, ea2);
                if (tb) fm.kget02(koff(Lb) + (wcode >> (2 * (K - Lb))), eb0, eb2);
                nkm += (uint64_t)ta + (uint64_t)tb;
                if (!ta || (hb && !tb)) ext_back2(fm, pa0, pa2, pb0, pb2, !ta, hb && !tb, c, oa0, oa2, ob0, ob2, nblk);
                if (ta) { oa0 = ea0; oa2 = ea2; }
                if (tb) { ob0 = eb0; ob2 = eb2; }
            }
            for (int h = 0; h < 2; ++h) {
                if (h == 1 && !hb) break;
                const X p0 = h ? pb0 : pa0, o0 = h ? ob0 : oa0;
                const Z p2 = h ? pb2 : pa2, o2 = h ? ob2 : oa2;
                const int pe = h ? pbe : pae;
                const bool keep_hit = c < 0 || o2 < (Z)min_intv;
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
        }
        j += 2;
        if (j >= n) {   // position i done (at i = -1 every entry is a hit, so nc == 0 ends the loop there)
            if (nc == 0) break;
            n = nc; nc = 0; j = 0; last_x2 = 0;
            --i;
            c = i < 0 ? -1 : (q[i] < 4 ? q[i] : -1);
            if (K > 0 && c >= 0) wcode = wcode >> 2 | (uint32_t)c << (2 * (K - 1));
        }
    }
    return ret;
}

template <typename X, typename Z, typename Q>
DEV int smem1_merged(const FM<X> &fm, int len, Q q, int x, int min_intv, LList<X, Z> &L, OutSlot &S,
                  bool &ovf, uint64_t &nblk, uint64_t &nkm)
{
    S.n1 = 0;
    if (q[x] > 3) return x + 1;
    if (min_intv < 1) min_intv = 1;
    int c0 = q[x];
    X ik0 = fm.L2(c0) + 1, ik1 = fm.L2(3 - c0) + 1;
    Z ik2 = (Z)(fm.L2(c0 + 1) - fm.L2(c0));
    int ikend = x + 1;
    int n = 0, i = x + 1;
    uint32_t fcode = (uint32_t)c0;   // code of q[x..i] while i - x + 1 <= K
    bool stop = false;               // the forward walk ended early (hole or interval below min_intv)
    {
        // Lengths 2..min(K, len - x) come from the k-mer table.  Their table rows depend only on the read's
        // bases, so every row is loaded before the first one is used (one round trip instead of K - 1);
        // the walk below then consumes them in order with the exact bookkeeping of the loop that follows.
        // (64-bit rows too: at 3 Gbp the table is a 179 MB array whose rows miss the caches as often as not,
        // and K - 1 dependent round trips per SMEM call were a fifth of the seeding kernel's time.)
        // rows preloaded: 11, or 13 for 64-bit rows (whose table is 13 deep: C4); a deeper table (kmer_depth up to
        // 15) serves lengths KM+1..K one per step below
        constexpr int KM = sizeof(X) == 8 ? 13 : 11;
        const int Kp = fm.K < KM ? fm.K : KM;
        const int Lt = Kp < len - x ? Kp : len - x;
        int cb[KM + 1];
#pragma unroll
        for (int t = 2; t <= KM; ++t) cb[t] = t <= Lt ? q[x + t - 1] : 4;
        X e0[KM + 1];
        Z e2[KM + 1];
        int nt = 1;   // bases from x covered without a hole (capped at Lt)
#pragma unroll
        for (int t = 2; t <= KM; ++t) {
            if (nt == t - 1 && cb[t] < 4) {
                fcode = fcode << 2 | (uint32_t)cb[t];
                fm.kget02(koff(t) + fcode, e0[t], e2[t]);
                nt = t;
            }
        }
        if (nt >= 2) {
            nkm += (uint64_t)(nt - 1);
            const X x1_last = fm.kget1(koff(nt) + fcode);
#pragma unroll
            for (int t = 2; t <= KM; ++t) {
                if (t <= nt && !stop) {
                    const X n0 = e0[t];
                    const Z n2 = e2[t];
                    if (n2 != ik2) {
                        if (n >= L.total()) { ovf = true; return len; }
                        L.set(n++, ik0, ik2, ikend);
                        if (n2 < (Z)min_intv) { stop = true; i = x + t - 1; }
                    }
                    if (!stop) { ik0 = n0; ik2 = n2; ikend = x + t; }
                }
            }
            ik1 = x1_last;
        }
        if (!stop) {
            i = x + nt;
            if (nt < Lt) {   // q[x + nt] is a hole: the walk stops there
                if (n >= L.total()) { ovf = true; return len; }
                L.set(n++, ik0, ik2, ikend);
                stop = true;
            }
        }
    }
    int qi = !stop && i < len ? q[i] : 0;
    // One loop for both phases of bwt_smem1: a lane that has finished its forward walk (reversed its list and set up
    // the backward pass) takes its backward pairs in the same trips in which other lanes of the wave still extend
    // forward, instead of waiting at the forward loop's exit for the wave's longest forward walk.  Per lane every
    // step, and the order of the steps, is smem1_lds's.
    const int K = fm.K;
    int phase = 0;   // 0 forward, 1 backward, 2 done
    int ret = 0, last_start = 0x7fffffff, c = -1, nc = 0, j = 0;
    uint32_t wcode = 0;
    Z last_x2 = 0;
    for (;;) {
        if (phase == 0) {
            bool fend = stop || i >= len;
            if (!fend) {
                if (ik2 == 1 && min_intv <= 1) {   // the unique-interval text walk (smem1_lds)
                    const int64_t p = fm.sa(ik0) - x, nT = fm.l_pac << 1;
                    int k = i;
                    for (;;) {
                        constexpr int W = 8;
                        int qc[W], tc[W];
#pragma unroll
                        for (int t = 0; t < W; ++t) {
                            const bool in = k + t < len && p + k + t < nT;
                            qc[t] = in ? q[k + t] : 5;
                            tc[t] = in ? fm.tbase(p + k + t) : 4;
                        }
                        int r = W;
#pragma unroll
                        for (int t = W - 1; t >= 0; --t)
                            if (qc[t] != tc[t]) r = t;
                        k += r;
                        if (r < W) break;
                    }
                    ikend = k;
                    i = k;
                    if (k < len) {
                        if (n >= L.total()) { ovf = true; return len; }
                        L.set(n++, ik0, ik2, ikend);
                    }
                    fend = true;
                } else {
                    const int cur = qi;
                    qi = i + 1 < len ? q[i + 1] : 0;
                    if (cur < 4) {
                        const int cc = 3 - cur;
                        X n1, n0;
                        Z n2;
                        fcode = fcode << 2 | (uint32_t)cur;
                        if (i - x + 1 <= fm.K) {
                            fm.kget(koff(i - x + 1) + fcode, n0, n1, n2);
                            ++nkm;
                        } else extend1(fm, ik1, ik0, ik2, cc, n1, n0, n2, nblk);
                        if (n2 != ik2) {
                            if (n >= L.total()) { ovf = true; return len; }
                            L.set(n++, ik0, ik2, ikend);
                            if (n2 < (Z)min_intv) fend = true;
                        }
                        if (!fend) {
                            ik0 = n0; ik1 = n1; ik2 = n2; ikend = i + 1;
                            if (++i >= len) fend = true;
                        }
                    } else {
                        if (n >= L.total()) { ovf = true; return len; }
                        L.set(n++, ik0, ik2, ikend);
                        fend = true;
                    }
                }
            }
            if (fend) {   // the forward walk is over: last push, reversal, backward set-up
                if (i == len) {
                    if (n >= L.total()) { ovf = true; return len; }
                    L.set(n++, ik0, ik2, ikend);
                }
                for (int jj = 0; jj < (n >> 1); ++jj) {
                    X a0, b0;
                    Z a2, b2;
                    int ae, be;
                    L.get(jj, a0, a2, ae);
                    L.get(n - 1 - jj, b0, b2, be);
                    L.set(jj, b0, b2, be);
                    L.set(n - 1 - jj, a0, a2, ae);
                }
                { X d0; Z d2; L.get(0, d0, d2, ret); }
                for (int t = 0; t < K; ++t) wcode = wcode << 2 | (x + t < len ? (uint32_t)(q[x + t] & 3) : 0u);
                i = x - 1;
                c = i < 0 ? -1 : (q[i] < 4 ? q[i] : -1);
                if (K > 0 && c >= 0) wcode = wcode >> 2 | (uint32_t)c << (2 * (K - 1));
                phase = 1;
            }
        }
        if (phase == 1) {   // one pair of the flat backward loop (smem1_lds)
            const bool hb = j + 1 < n;
            X pa0, pb0;
            Z pa2, pb2;
            int pae, pbe;
            L.get(j, pa0, pa2, pae);
            L.get(hb ? j + 1 : j, pb0, pb2, pbe);
            X oa0 = 0, ob0 = 0;
            Z oa2 = 0, ob2 = 0;
            if (c >= 0) {
                const int La = pae - i, Lb = pbe - i;
                const bool ta = La <= K, tb = hb && Lb <= K;
                X ea0 = 0, eb0 = 0;
                Z ea2 = 0, eb2 = 0;
                if (ta) fm.kget02(koff(La) + (wcode >> (2 * (K - La))), ea0, ea2);
                if (tb) fm.kget02(koff(Lb) + (wcode >> (2 * (K - Lb))), eb0, eb2);
                nkm += (uint64_t)ta + (uint64_t)tb;
                if (!ta || (hb && !tb)) ext_back2(fm, pa0, pa2, pb0, pb2, !ta, hb && !tb, c, oa0, oa2, ob0, ob2, nblk);
                if (ta) { oa0 = ea0; oa2 = ea2; }
                if (tb) { ob0 = eb0; ob2 = eb2; }
            }
            for (int h = 0; h < 2; ++h) {
                if (h == 1 && !hb) break;
                const X p0 = h ? pb0 : pa0, o0 = h ? ob0 : oa0;
                const Z p2 = h ? pb2 : pa2, o2 = h ? ob2 : oa2;
                const int pe = h ? pbe : pae;
                const bool keep_hit = c < 0 || o2 < (Z)min_intv;
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
            j += 2;
            if (j >= n) {
                if (nc == 0) phase = 2;
                else {
                    n = nc; nc = 0; j = 0; last_x2 = 0;
                    --i;
                    c = i < 0 ? -1 : (q[i] < 4 ? q[i] : -1);
                    if (K > 0 && c >= 0) wcode = wcode >> 2 | (uint32_t)c << (2 * (K - 1));
                }
            }
        }
        if (phase == 2) break;
    }
    return ret;
}

// smem1_lds (M = false) or smem1_merged (M = true), chosen at compile time per kernel instantiation
template <bool M, typename X, typename Z, typename Q>
DEV int smem1_call(const FM<X> &fm, int len, Q q, int x, int min_intv, LList<X, Z> &L, OutSlot &S, bool &ovf,
                   uint64_t &nblk, uint64_t &nkm)
{
    if constexpr (M) return smem1_merged(fm, len, q, x, min_intv, L, S, ovf, nblk, nkm);
    else return smem1_lds(fm, len, q, x, min_intv, L, S, ovf, nblk, nkm);
}

template <typename X, typename Z, typename Q>
DEV int seed_strategy1_x(const FM<X> &fm, int len, Q q, int x, int min_len, int max_intv, Intv &mem,
                         uint64_t &nblk, uint64_t &nkm, bool walk)
{
    mem.x[0] = mem.x[1] = mem.x[2] = mem.info = 0;
    if (q[x] > 3) return x + 1;
    const int c0 = q[x];
    X ik0 = fm.L2(c0) + 1, ik1 = fm.L2(3 - c0) + 1;
    Z ik2 = (Z)(fm.L2(c0 + 1) - fm.L2(c0));
    uint32_t fcode = (uint32_t)c0;
    int i0 = x + 1;
    if (fm.K > 1 && min_len >= fm.K) {
        // No string of at most K bases can be returned (that needs i - x >= min_len), so the steps through
        // lengths 2..L (L = min(K, len - x)) only carry the interval forward: one k-mer table read at length L
        // gives it, unless a hole base ends the walk first (the loop returns just past it).
        const int L = fm.K < len - x ? fm.K : len - x;
        int t = 1;
        for (; t < L; ++t) {
            const int c = q[x + t];
            if (c > 3) return x + t + 1;
            fcode = fcode << 2 | (uint32_t)c;
        }
        if (L > 1) {
            fm.kget(koff(L) + fcode, ik0, ik1, ik2);
            ++nkm;
        }
        i0 = x + L;
    }
    int qi = i0 < len ? q[i0] : 0;
    for (int i = i0; i < len; ++i) {
        if (ik2 == 1 && max_intv > 1 && walk) {
            // A unique interval stays [x0, x0] while the string follows its one occurrence (at SA[x0] in T) and
            // is empty from the first differing base on; an empty one stays empty.  Sizes stay below max_intv, so
            // the loop returns at the first step j >= x + min_len (or at a hole, or runs off the read): decide that
            // step from the text instead of one bwt_extend per base.  The seed's x[1] is not tracked on this path
            // (mem_chain reads x[0], x[2] and info only -- the same convention as the SMEM list entries).
            const int js = i > x + min_len ? i : x + min_len;
            const int jend = js < len ? js : len - 1;
            int h = i;
            while (h <= jend && q[h] < 4) ++h;
            if (h <= jend) return h + 1;          // a hole ends the call
            if (js >= len) return len;            // the read ends first: no seed
            const int64_t p = fm.sa(ik0) - x, nT = fm.l_pac << 1;
            bool match = true;
            for (int j = i; j <= js && match; ++j) match = p + j < nT && q[j] == fm.tbase(p + j);
            if (match) {
                mem.x[0] = ik0; mem.x[1] = 0; mem.x[2] = 1;
                mem.info = (uint64_t)x << 32 | (uint64_t)(js + 1);
            }
            return js + 1;
        }
        const int cur = qi;
        qi = i + 1 < len ? q[i + 1] : 0;
        if (cur < 4) {
            const int c = 3 - cur;
            X n1, n0;
            Z n2;
            fcode = fcode << 2 | (uint32_t)cur;
            if (i - x + 1 <= fm.K) {
                fm.kget(koff(i - x + 1) + fcode, n0, n1, n2);
                ++nkm;
            } else extend1(fm, ik1, ik0, ik2, c, n1, n0, n2, nblk);
            if (n2 < (Z)max_intv && i - x >= min_len) {
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

// A read's bases in the wave-transposed copy (k_codes_wave): base i at p[i * 64], so the lanes of a wave
// reading base i of their reads load one contiguous 64-B line instead of 64 lines.
struct QT {
    const uint8_t *p;
    DEV int operator[](int i) const { return p[(size_t)i * 64]; }
};

// codes_t[(li / 64) * 64 * L + i * 64 + li % 64] = base i of read li (i < its length; L = the batch's
// read-length cap).  One block per 64 reads: the wave's reads are contiguous in `codes`, so they are staged in
// LDS with coalesced loads, then written out transposed (64 lanes store one 64-B line per base index).
extern __shared__ uint8_t g_codes_stage[];
__global__ void __launch_bounds__(256) k_codes_wave(const uint8_t *codes, const int64_t *offs, int n, int L,
                                                    uint8_t *codes_t)
{
    const int r0 = blockIdx.x * 64, r1 = r0 + 64 < n ? r0 + 64 : n;
    const int64_t b0 = offs[r0], nb = offs[r1] - b0;   // <= 64 * L bytes
    for (int64_t i = threadIdx.x; i < nb; i += blockDim.x) g_codes_stage[i] = codes[b0 + i];
    __syncthreads();
    const int lane = threadIdx.x & 63, li = r0 + lane;
    if (li >= r1) return;
    const int s = (int)(offs[li] - b0), len = (int)(offs[li + 1] - offs[li]);
    uint8_t *d = codes_t + (size_t)blockIdx.x * 64 * (size_t)L + lane;
    for (int i = (int)(threadIdx.x >> 6); i < len; i += 4) d[(size_t)i * 64] = g_codes_stage[s + i];
}

// 4 waves per SIMD for u32 rows (16 one-wave blocks per CU, the LDS limit), 3 for 64-bit rows
template <typename X, typename Z, typename Q, bool M>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(sizeof(X) == 4 ? 4 : 3))) k_smem_lds(DIndex ix, DOpts o, Caps cp, const uint8_t *codes, const int64_t *offs,
                                                  int n, Intv *intv_out, int32_t *n_intv, uint32_t *status,
                                                  Counters *ctr, int lcap, uint8_t *spill, int gcap, int qcap)
{
    const int T = blockDim.x, t = threadIdx.x;
    LList<X, Z> L;   // LDS: [x0: T*lcap X][x2: T*lcap Z][end: T*lcap u16]
    L.x0 = t;
    L.x2 = (int)((size_t)T * lcap * sizeof(X) / sizeof(Z)) + t;
    L.end = (int)((size_t)T * lcap * (sizeof(X) + sizeof(Z)) / 2) + t;
    L.stride = T;
    L.cap = lcap;
    {   // spill area: [x0: N*gcap X][x2: N*gcap Z][end: N*gcap u32] (N = n in whole waves), each array holding a
        // wave's gcap entries per lane lane-interleaved (entry g of lane l at [g * 64 + l] of the wave's block)
        const size_t li0 = (size_t)blockIdx.x * T + t;
        const size_t me = (li0 >> 6) * 64 * (size_t)gcap + (li0 & 63), tot = (size_t)(n + 63) / 64 * 64 * (size_t)gcap;
        L.gx0 = reinterpret_cast<X *>(spill) + me;
        L.gx2 = reinterpret_cast<Z *>(spill + tot * sizeof(X)) + me;
        L.gend = reinterpret_cast<uint32_t *>(spill + tot * (sizeof(X) + sizeof(Z))) + me;
        L.gcap = spill ? gcap : 0;
    }
    FM<X> fm;
    fm.occ = ix.occ;
    fm.occ32 = ix.occ32;
    fm.sup = ix.sup;
    fm.l2_0 = (X)ix.L2[0]; fm.l2_1 = (X)ix.L2[1]; fm.l2_2 = (X)ix.L2[2]; fm.l2_3 = (X)ix.L2[3]; fm.l2_4 = (X)ix.L2[4];
    fm.primary = (X)ix.primary;
    fm.kt = reinterpret_cast<const uint4 *>(ix.kmer);
    fm.K = ix.kmer_k;   // the table is built in the index's row width
    fm.pac = ix.pac; fm.l_pac = ix.l_pac; fm.sa32 = ix.sa32; fm.sa64 = ix.sa64;
    uint64_t nblk = 0, nkm = 0;
    // one read per lane; a grid smaller than the batch (BSQ_SMEM_GRID, the co-residency experiment) loops its waves
    // over the rest (the loop condition is wave-uniform)
    for (int li = blockIdx.x * T + t; li - t < n; li += gridDim.x * T) {
    if (li < n) {
        {
            const size_t me = ((size_t)li >> 6) * 64 * (size_t)gcap + ((size_t)li & 63), tot = (size_t)(n + 63) / 64 * 64 * (size_t)gcap;
            L.gx0 = reinterpret_cast<X *>(spill) + me;
            L.gx2 = reinterpret_cast<Z *>(spill + tot * sizeof(X)) + me;
            L.gend = reinterpret_cast<uint32_t *>(spill + tot * (sizeof(X) + sizeof(Z))) + me;
        }
        Q q;
        if constexpr (__is_same(Q, QT)) q = QT{codes + (size_t)(li >> 6) * 64 * (size_t)qcap + (li & 63)};   // codes_t
        else q = codes + offs[li];
        const int len = (int)(offs[li + 1] - offs[li]);
        bool ovf = false;
        OutSlot S{SP<Intv>{intv_out + intv_slot_at_d(li, 0, cp.intv)}, 0, cp.intv, 0};
        const int split_len = (int)(o.min_seed_len * o.split_factor + .499);
        auto take_mem1 = [&](bool pass2) {
            // mem1 (reversed emission order) sits at S.a[cap-n1 .. cap); filter-append in order
            for (int k = 0; k < S.n1; ++k) {
                const Intv &m = S.a[S.cap - S.n1 + k];
                const uint64_t m0 = m.x[0], m2 = m.x[2], mi = m.info;
                uint32_t st = (uint32_t)(mi >> 32), en = (uint32_t)mi;
                bool keep = pass2 ? (uint64_t)(en - st) >= (uint64_t)o.min_seed_len : (int)(en - st) >= o.min_seed_len;
                if (keep) { Intv &d = S.a[S.n++]; d.x[0] = m0; d.x[1] = 0; d.x[2] = m2; d.info = mi; }
            }
            S.n1 = 0;
        };
        int x = 0;
        while (x < len && !ovf) {
            if (q[x] < 4) {
                x = smem1_call<M>(fm, len, q, x, 1, L, S, ovf, nblk, nkm);
                if (!ovf) take_mem1(false);
            } else ++x;
        }
        const int old_n = S.n;
        for (int k = 0; k < old_n && !ovf; ++k) {
            const Intv p = S.a[k];
            const int start = (int)(p.info >> 32), end = (int)(uint32_t)p.info;
            if (end - start < split_len || p.x[2] > (uint64_t)o.split_width) continue;
            smem1_call<M>(fm, len, q, (start + end) >> 1, (int)p.x[2] + 1, L, S, ovf, nblk, nkm);
            if (!ovf) take_mem1(true);
        }
        if (o.max_mem_intv > 0) {
            x = 0;
            while (x < len && !ovf) {
                if (q[x] < 4) {
                    Intv m;
                    x = seed_strategy1_x<X, Z>(fm, len, q, x, o.min_seed_len, o.max_mem_intv, m, nblk, nkm, o.ss_walk != 0);
                    if (m.x[2] > 0) {
                        if (S.n >= S.cap) { ovf = true; break; }
                        Intv &d = S.a[S.n++];
                        d.x[0] = m.x[0]; d.x[1] = m.x[1]; d.x[2] = m.x[2]; d.info = m.info;
                    }
                } else ++x;
            }
        }
        if (ovf) {
            status[li] |= ST_OVERFLOW;
            n_intv[li] = 0;
        } else {
            const SP<Intv> out = S.a;
            for (int a = 1; a < S.n; ++a) {   // equal keys are identical intervals: any correct sort is exact
                const uint64_t t0 = out[a].x[0], t1 = out[a].x[1], t2 = out[a].x[2], ti = out[a].info;
                int b = a;
                for (; b > 0; --b) {
                    const uint64_t pi = out[b - 1].info;
                    if (!(ti < pi)) break;
                    out[b].x[0] = out[b - 1].x[0]; out[b].x[1] = out[b - 1].x[1];
                    out[b].x[2] = out[b - 1].x[2]; out[b].info = pi;
                }
                out[b].x[0] = t0; out[b].x[1] = t1; out[b].x[2] = t2; out[b].info = ti;
            }
            n_intv[li] = S.n;
        }
    }
    }
    wave_add2(&ctr[STG_SMEM].occ_blocks, nblk);
    wave_add2(&ctr[STG_SMEM].kmer_hits, nkm);
}

// k_smem_lanes: k_smem_lds with persistent lanes that step through their reads one CALL at a time.
// In k_smem_lds a lane owns one read, and the wave runs pass 1 (bwt_smem1 over x), pass 2 (re-seeding) and pass 3
// (bwt_seed_strategy1) as three loops: a lane whose read needs 2 bwt_smem1 calls idles while another lane of the wave
// makes 10 (the 2 % random reads make ~10 short SMEMs), and the wave ends with its slowest read.  Here each trip of
// the outer loop makes at most one call per lane -- one bwt_smem1 (pass 1 or 2: both lanes' kinds share the one call
// site) or one bwt_seed_strategy1 -- after an ALU-only step that moves each lane to its next call (holes skipped,
// pass-2 entries that do not qualify skipped, pass changes); a lane that has finished its read sorts its intervals
// and takes the next read (li += the grid's lanes; lane = li % 64, so the wave-transposed codes and the per-wave
// slots keep their layouts).  Per read the calls, their order and their arguments are k_smem_lds's: identical intervals.
template <typename X, typename Z, typename Q, bool M>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(sizeof(X) == 4 ? 4 : 3))) k_smem_lanes(DIndex ix, DOpts o, Caps cp, const uint8_t *codes, const int64_t *offs,
                                                   int n, Intv *intv_out, int32_t *n_intv, uint32_t *status,
                                                   Counters *ctr, int lcap, uint8_t *spill, int gcap, int qcap)
{
    const int t = threadIdx.x;
    LList<X, Z> L;   // LDS: [x0: 64*lcap X][x2: 64*lcap Z][end: 64*lcap u16]
    L.x0 = t;
    L.x2 = (int)((size_t)64 * lcap * sizeof(X) / sizeof(Z)) + t;
    L.end = (int)((size_t)64 * lcap * (sizeof(X) + sizeof(Z)) / 2) + t;
    L.stride = 64;
    L.cap = lcap;
    L.gcap = spill ? gcap : 0;
    const size_t spill_tot = (size_t)(n + 63) / 64 * 64 * (size_t)gcap;
    FM<X> fm;
    fm.occ = ix.occ;
    fm.occ32 = ix.occ32;
    fm.sup = ix.sup;
    fm.l2_0 = (X)ix.L2[0]; fm.l2_1 = (X)ix.L2[1]; fm.l2_2 = (X)ix.L2[2]; fm.l2_3 = (X)ix.L2[3]; fm.l2_4 = (X)ix.L2[4];
    fm.primary = (X)ix.primary;
    fm.kt = reinterpret_cast<const uint4 *>(ix.kmer);
    fm.K = ix.kmer_k;
    fm.pac = ix.pac; fm.l_pac = ix.l_pac; fm.sa32 = ix.sa32; fm.sa64 = ix.sa64;
    const int split_len = (int)(o.min_seed_len * o.split_factor + .499);
    const int lstride = gridDim.x * 64;
    uint64_t nblk = 0, nkm = 0;
    enum { NEXT, P1, P2, P3, FIN, DONE };
    int st = NEXT, li = blockIdx.x * 64 + t - lstride, len = 0, x = 0, k2 = 0, old_n = 0;
    bool ovf = false;
    Q q{};
    OutSlot S{SP<Intv>{intv_out}, 0, cp.intv, 0};
    for (;;) {
        if (st == NEXT) {   // the lane's next read
            li += lstride;
            if (li >= n) st = DONE;
            else {
                const size_t me = ((size_t)li >> 6) * 64 * (size_t)gcap + ((size_t)li & 63);
                L.gx0 = reinterpret_cast<X *>(spill) + me;
                L.gx2 = reinterpret_cast<Z *>(spill + spill_tot * sizeof(X)) + me;
                L.gend = reinterpret_cast<uint32_t *>(spill + spill_tot * (sizeof(X) + sizeof(Z))) + me;
                if constexpr (__is_same(Q, QT)) q = QT{codes + (size_t)(li >> 6) * 64 * (size_t)qcap + (li & 63)};
                else q = codes + offs[li];
                len = (int)(offs[li + 1] - offs[li]);
                ovf = false;
                S = OutSlot{SP<Intv>{intv_out + intv_slot_at_d(li, 0, cp.intv)}, 0, cp.intv, 0};
                x = 0;
                st = P1;
            }
        }
        if (__ballot(st != DONE) == 0) break;
        // to the lane's next call (ALU and the read's bases only)
        int sx = 0, mi = 1;
        bool call_smem = false, call_ss = false;
        for (bool adv = st == P1 || st == P2 || st == P3; adv;) {
            adv = false;
            if (st == P1) {
                while (x < len && q[x] > 3) ++x;
                if (x < len && !ovf) { call_smem = true; sx = x; mi = 1; }
                else { old_n = S.n; k2 = 0; st = P2; adv = true; }
            } else if (st == P2) {
                if (ovf || k2 >= old_n) { st = P3; x = 0; adv = true; }
                else {
                    const Intv p = S.a[k2];
                    const int start = (int)(p.info >> 32), end = (int)(uint32_t)p.info;
                    if (end - start < split_len || p.x[2] > (uint64_t)o.split_width) { ++k2; adv = true; }
                    else { call_smem = true; sx = (start + end) >> 1; mi = (int)p.x[2] + 1; }
                }
            } else if (st == P3) {
                if (o.max_mem_intv <= 0 || ovf) st = FIN;
                else {
                    while (x < len && q[x] > 3) ++x;
                    if (x < len) call_ss = true;
                    else st = FIN;
                }
            }
        }
        if (call_smem) {   // pass 1 and pass 2 share this call site
            const int r = smem1_call<M>(fm, len, q, sx, mi, L, S, ovf, nblk, nkm);
            if (!ovf) {   // take_mem1
                const bool pass2 = st == P2;
                for (int k = 0; k < S.n1; ++k) {
                    const Intv &m = S.a[S.cap - S.n1 + k];
                    const uint64_t m0 = m.x[0], m2 = m.x[2], mn = m.info;
                    const uint32_t s0 = (uint32_t)(mn >> 32), en = (uint32_t)mn;
                    const bool keep = pass2 ? (uint64_t)(en - s0) >= (uint64_t)o.min_seed_len : (int)(en - s0) >= o.min_seed_len;
                    if (keep) { Intv &d = S.a[S.n++]; d.x[0] = m0; d.x[1] = 0; d.x[2] = m2; d.info = mn; }
                }
                S.n1 = 0;
            }
            if (st == P1) x = r;
            else ++k2;
        }
        if (call_ss) {
            Intv m;
            x = seed_strategy1_x<X, Z>(fm, len, q, x, o.min_seed_len, o.max_mem_intv, m, nblk, nkm, o.ss_walk != 0);
            if (m.x[2] > 0) {
                if (S.n >= S.cap) ovf = true;
                else { Intv &d = S.a[S.n++]; d.x[0] = m.x[0]; d.x[1] = m.x[1]; d.x[2] = m.x[2]; d.info = m.info; }
            }
        }
        if (st == FIN) {
            if (ovf) {
                status[li] |= ST_OVERFLOW;
                n_intv[li] = 0;
            } else {
                const SP<Intv> out = S.a;
                for (int a = 1; a < S.n; ++a) {   // equal keys are identical intervals: any correct sort is exact
                    const uint64_t t0 = out[a].x[0], t1 = out[a].x[1], t2 = out[a].x[2], ti = out[a].info;
                    int b = a;
                    for (; b > 0; --b) {
                        const uint64_t pi = out[b - 1].info;
                        if (!(ti < pi)) break;
                        out[b].x[0] = out[b - 1].x[0]; out[b].x[1] = out[b - 1].x[1];
                        out[b].x[2] = out[b - 1].x[2]; out[b].info = pi;
                    }
                    out[b].x[0] = t0; out[b].x[1] = t1; out[b].x[2] = t2; out[b].info = ti;
                }
                n_intv[li] = S.n;
            }
            st = NEXT;
        }
    }
    wave_add2(&ctr[STG_SMEM].occ_blocks, nblk);
    wave_add2(&ctr[STG_SMEM].kmer_hits, nkm);
}

// LDS bytes per thread for `lcap` list entries
template <typename X, typename Z>
static size_t lds_bytes(int threads, int lcap) { return (size_t)threads * lcap * (sizeof(X) + sizeof(Z) + 2); }

// 64-bit rows whose interval sizes fit u32 (every x[2] is at most one base's count, <= l_pac); BSQ_FORCE_WIDE=2
// (tests) takes the all-u64 kernel on any index
bool wide_z32(const DIndex &ix)
{
    const char *fw = getenv("BSQ_FORCE_WIDE");
    return !(fw && *fw == '2') && ix.l_pac < ((int64_t)1 << 32);
}

// codes_t: a workspace buffer of ceil(n / 64) * 64 * cp.max_len bytes for the wave-transposed copy of the
// reads (nullptr: the kernel reads the packed codes)
hipError_t launch_smem_lds(hipStream_t st, const DIndex &ix, const DOpts &o, const Caps &cp, const uint8_t *codes,
                           const int64_t *offs, int n, Intv *intv, int32_t *n_intv, uint32_t *status, Counters *ctr,
                           int lcap, uint8_t *spill, int gcap, uint8_t *codes_t)
{
    // one-wave blocks: a block's LDS lists are released when its wave ends, not when the slowest of four
    // waves does (C2 +2.7 %, C3 +1.4 % against 256-lane blocks at the same 16 waves per CU)
    const int T = 64;
    int grid = (n + T - 1) / T;
    if (grid == 0) return hipSuccess;
    // persistent lanes (k_smem_lanes, BSQ_SMEM_LANES=1; default k_smem_lds): each lane steps through rpl reads call by call
    const char *le = getenv("BSQ_SMEM_LANES");
    const bool lanes = le && *le == '1';
    if (lanes) {
        const char *r = getenv("BSQ_SMEM_RPL");
        const int rpl = r && atoi(r) > 0 ? atoi(r) : 4;
        grid = (grid + rpl - 1) / rpl;
    }
    if (const char *g = getenv("BSQ_SMEM_GRID")) { const int c = atoi(g); if (c > 0 && c < grid) grid = c; }
    const int L = cp.max_len;
    if (codes_t)
        hipLaunchKernelGGL(k_codes_wave, dim3((n + 63) / 64), dim3(256), (size_t)64 * L, st, codes, offs, n, L, codes_t);
    // the merged forward/backward loop of bwt_smem1 (smem1_merged, BSQ_SMEM_MERGE=1; default smem1_lds)
    const char *me = getenv("BSQ_SMEM_MERGE");
    const bool merge = me && *me == '1';
#define BSQ_SMEM_LAUNCH2(X_, Z_, M_)                                                                                   \
    do {                                                                                                               \
        const size_t sh = lds_bytes<X_, Z_>(T, lcap);                                                                  \
        if (lanes) {                                                                                                   \
            if (codes_t)                                                                                               \
                hipLaunchKernelGGL((k_smem_lanes<X_, Z_, QT, M_>), dim3(grid), dim3(T), sh, st, ix, o, cp, codes_t,     \
                                   offs, n, intv, n_intv, status, ctr, lcap, spill, gcap, L);                          \
            else                                                                                                       \
                hipLaunchKernelGGL((k_smem_lanes<X_, Z_, const uint8_t *, M_>), dim3(grid), dim3(T), sh, st, ix, o, cp, \
                                   codes, offs, n, intv, n_intv, status, ctr, lcap, spill, gcap, L);                   \
        } else {                                                                                                       \
            if (codes_t)                                                                                               \
                hipLaunchKernelGGL((k_smem_lds<X_, Z_, QT, M_>), dim3(grid), dim3(T), sh, st, ix, o, cp, codes_t, offs,  \
                                   n, intv, n_intv, status, ctr, lcap, spill, gcap, L);                                 \
            else                                                                                                       \
                hipLaunchKernelGGL((k_smem_lds<X_, Z_, const uint8_t *, M_>), dim3(grid), dim3(T), sh, st, ix, o, cp,   \
                                   codes, offs, n, intv, n_intv, status, ctr, lcap, spill, gcap, L);                   \
        }                                                                                                              \
    } while (0)
#define BSQ_SMEM_LAUNCH(X_, Z_)                                                                                         \
    do {                                                                                                               \
        if (merge) BSQ_SMEM_LAUNCH2(X_, Z_, true);                                                                     \
        else BSQ_SMEM_LAUNCH2(X_, Z_, false);                                                                          \
    } while (0)
    if (!ix.wide) BSQ_SMEM_LAUNCH(uint32_t, uint32_t);
    else if (wide_z32(ix)) BSQ_SMEM_LAUNCH(uint64_t, uint32_t);   // 64-bit rows, interval sizes in u32 (l_pac < 2^32)
    else BSQ_SMEM_LAUNCH(uint64_t, uint64_t);
#undef BSQ_SMEM_LAUNCH2
#undef BSQ_SMEM_LAUNCH
    return hipGetLastError();
}

// =============================================================================================
// k_smem_sm: the same mem_collect_intv (bwt_smem1 x2 passes + bwt_seed_strategy1), restructured as a per-lane state
// machine so the wave issues its memory at once (u32 rows, reads of <= SM_MAXLEN bases).
//
// k_smem_lds runs each lane's read as nested structured loops (forward walk, backward loop, seed strategy): a wave
// executes a loop body only for the lanes inside it, and waits at every loop exit for its slowest lane, so its
// rank-block loads go out with ~10 of 64 lanes active (SQ_INSTS_VMEM_RD) and the memory system sees
// a fraction of the requests the wave could have in flight.  Here every lane is a resumable state machine:
//   advance: each lane consumes the data its last request loaded, runs its control (divergent, ALU + LDS only)
//            until it needs memory again, and writes up to 8 16-B load addresses into its request slots;
//   issue:   one uniform block of 8 predicated 16-B loads for all lanes -- every lane that needs a rank block,
//            a k-mer table row or an interval slot gets it in the same instructions.
// A lane that finishes its read takes the next one (persistent lanes, reads li = wave + k * waves, lane = li % 64),
// so lanes never wait for each other's reads.  The read is staged in LDS as 2-bit codes + a hole bitmap
// (k_pack_reads), the SMEM list stays in LDS as in k_smem_lds (same LList and spill area), mem1 entries are read
// back through the request slots (TAKE), and the final per-read sort of the intervals is k_intv_sort.  The
// arithmetic of every step is k_smem_lds's (extend1 / ext_back2 / occ_c32 / the k-mer rows), in the same order per
// lane, so the intervals are identical; the unique-interval text walk is not used (the extension steps it replaces
// give the same list, one rank block per step).
// =============================================================================================
constexpr int SM_SLOTS = 8;
constexpr int SM_MAXLEN = 320;   // 20 + 10 + 1 packed words <= 32 (8 slots of 16 B)

enum SmState : int {
    SMS_LOAD_REQ = 0, SMS_LOAD, SMS_P1, SMS_START, SMS_PRE, SMS_FWD_NEXT, SMS_FWD_EXT, SMS_FWD_KM, SMS_FWD_END,
    SMS_BWD_REQ, SMS_BWD, SMS_RET, SMS_TAKE_REQ, SMS_TAKE, SMS_P2_REQ, SMS_P2, SMS_P3, SMS_SS_LOOP, SMS_SS_KM,
    SMS_SS_NEXT, SMS_SS_EXT, SMS_FIN, SMS_DONE
};

// reads as 2-bit codes (code & 3, 16 per word, base i at bits 2(i & 15) of word i >> 4), then a hole bitmap (code > 3,
// 32 per word), then the length; nwp words per read (a multiple of 4: whole 16-B slots)
__global__ void __launch_bounds__(256) k_pack_reads(const uint8_t *codes, const int64_t *offs, int n, int nwp, int nw2,
                                                    int nwh, uint32_t *qpack)
{
    const int li = blockIdx.x * blockDim.x + threadIdx.x;
    if (li >= n) return;
    const uint8_t *q = codes + offs[li];
    const int len = (int)(offs[li + 1] - offs[li]);
    uint32_t *o = qpack + (size_t)li * nwp;
    for (int w = 0; w < nw2; ++w) {
        uint32_t v = 0;
        for (int t = 0; t < 16; ++t) { const int i = w * 16 + t; if (i < len) v |= (uint32_t)(q[i] & 3) << (2 * t); }
        o[w] = v;
    }
    for (int w = 0; w < nwh; ++w) {
        uint32_t v = 0;
        for (int t = 0; t < 32; ++t) { const int i = w * 32 + t; if (i < len && q[i] > 3) v |= 1u << t; }
        o[nw2 + w] = v;
    }
    o[nw2 + nwh] = (uint32_t)len;
    for (int w = nw2 + nwh + 1; w < nwp; ++w) o[w] = 0;
}

// the per-read interval sort that ends k_smem_lds (mem_collect_intv's ks_introsort by info: equal keys are identical
// intervals, so any correct sort is exact), one lane per read over its wave-interleaved slots
__global__ void __launch_bounds__(256) k_intv_sort(int n, Intv *intv_out, const int32_t *n_intv, int cap)
{
    const int li = blockIdx.x * blockDim.x + threadIdx.x;
    if (li >= n) return;
    const int m = n_intv[li];
    const SP<Intv> out{intv_out + intv_slot_at_d(li, 0, cap)};
    for (int a = 1; a < m; ++a) {
        const uint64_t t0 = out[a].x[0], t1 = out[a].x[1], t2 = out[a].x[2], ti = out[a].info;
        int b = a;
        for (; b > 0; --b) {
            const uint64_t pi = out[b - 1].info;
            if (!(ti < pi)) break;
            out[b].x[0] = out[b - 1].x[0]; out[b].x[1] = out[b - 1].x[1];
            out[b].x[2] = out[b - 1].x[2]; out[b].info = pi;
        }
        out[b].x[0] = t0; out[b].x[1] = t1; out[b].x[2] = t2; out[b].info = ti;
    }
}

// rank sums of base c at both ends of the interval [a - 1, a - 1 + x2] from the blocks loaded into slots s0..s0+3
// (k end: s0, s0+1; l end: s0+2, s0+3, or the k end's block again when both ends share it)
template <int S0>
DEV void sm_sums(const FM<uint32_t> &fm, const uint4 (&D)[SM_SLOTS], uint32_t a, uint32_t x2, int c, uint32_t &kc,
                 uint32_t &kg, uint32_t &lc, uint32_t &lg, uint64_t &nblk)
{
    const uint32_t k = a - 1, l = k + x2;
    const bool knone = k == 0xffffffffu;
    const uint32_t kk = k - (k >= fm.primary), ll = l - (l >= fm.primary);
    const bool same = !knone && (kk >> 6) == (ll >> 6);
    const uint4 wk[2] = {D[S0], D[S0 + 1]};
    const uint4 wl[2] = {same ? D[S0] : D[S0 + 2], same ? D[S0 + 1] : D[S0 + 3]};
    occ_c32(wk, kk, knone, c, kc, kg);
    occ_c32(wl, ll, false, c, lc, lg);
    nblk += (knone || same) ? 1 : 2;
}

// the request for sm_sums<S0>: the k end's block unless k = -1, the l end's unless it is the same block
template <int S0>
DEV void sm_req_blocks(const FM<uint32_t> &fm, uint32_t a, uint32_t x2, const uint4 *(&ad)[SM_SLOTS], uint32_t &vm)
{
    const uint32_t k = a - 1, l = k + x2;
    const bool knone = k == 0xffffffffu;
    const uint32_t kk = k - (k >= fm.primary), ll = l - (l >= fm.primary);
    if (!knone) { ad[S0] = reinterpret_cast<const uint4 *>(fm.occ32 + (kk >> 6)); ad[S0 + 1] = ad[S0] + 1; vm |= 3u << S0; }
    if (knone || (kk >> 6) != (ll >> 6)) {
        ad[S0 + 2] = reinterpret_cast<const uint4 *>(fm.occ32 + (ll >> 6)); ad[S0 + 3] = ad[S0 + 2] + 1; vm |= 12u << S0;
    }
}

DEV uint64_t u64_of(uint32_t lo, uint32_t hi) { return (uint64_t)hi << 32 | lo; }

__global__ void __launch_bounds__(64) k_smem_sm(DIndex ix, DOpts o, Caps cp, const uint32_t *qpack, int nwp, int nw2,
                                                int nwh, int n, Intv *intv_out, int32_t *n_intv, uint32_t *status,
                                                Counters *ctr, int lcap, uint8_t *spill, int gcap)
{
    const int lane = threadIdx.x;
    FM<uint32_t> fm;
    fm.occ = ix.occ;
    fm.occ32 = ix.occ32;
    fm.sup = ix.sup;
    fm.l2_0 = (uint32_t)ix.L2[0]; fm.l2_1 = (uint32_t)ix.L2[1]; fm.l2_2 = (uint32_t)ix.L2[2];
    fm.l2_3 = (uint32_t)ix.L2[3]; fm.l2_4 = (uint32_t)ix.L2[4];
    fm.primary = (uint32_t)ix.primary;
    fm.kt = reinterpret_cast<const uint4 *>(ix.kmer);
    fm.K = ix.kmer_k < 11 ? ix.kmer_k : 11;   // this kernel uses levels <= 11 of a deeper table
    fm.pac = ix.pac; fm.l_pac = ix.l_pac; fm.sa32 = ix.sa32; fm.sa64 = ix.sa64;
    const int K = fm.K;
    // LDS (u32 units): the read's nwp words lane-interleaved, then the list [x0: 64*lcap][x2: 64*lcap][end: 64*lcap u16]
    LList<uint32_t, uint32_t> L;
    const int lbase = nwp * 64;
    L.x0 = lbase + lane;
    L.x2 = lbase + 64 * lcap + lane;
    L.end = 2 * (lbase + 128 * lcap) + lane;
    L.stride = 64;
    L.cap = lcap;
    L.gcap = spill ? gcap : 0;
    const size_t spill_tot = (size_t)(n + 63) / 64 * 64 * (size_t)gcap;
    auto qw = [&](int w) -> uint32_t { return g_smem_u32[w * 64 + lane]; };
    auto q2 = [&](int i) -> int { return (int)(qw(i >> 4) >> ((i & 15) << 1) & 3u); };
    auto qv = [&](int i) -> int { return (qw(nw2 + (i >> 5)) >> (i & 31) & 1u) ? 4 : q2(i); };
    const int split_len = (int)(o.min_seed_len * o.split_factor + .499);
    const int cap = cp.intv;

    uint64_t nblk = 0, nkm = 0;
    int st = SMS_LOAD_REQ;
    int li = blockIdx.x * 64 + lane;
    const int lstride = gridDim.x * 64;
    SP<Intv> Sa{nullptr};
    int len = 0, Sn = 0, Sn1 = 0, x = 0, k2 = 0, old_n = 0, ret_to = 0, tk = 0;
    bool ovf = false;
    // bwt_smem1 / bwt_seed_strategy1 state
    int sx = 0, min_intv = 1, ikend = 0, n_l = 0, i = 0, nt = 0, Lt = 0, pt = 0, ret = 0, last_start = 0, c = 0, nc = 0,
        j = 0;
    uint32_t ik0 = 0, ik1 = 0, ik2 = 0, fcode = 0, wcode = 0, last_x2 = 0;
    bool stop = false, ta = false, tb = false, hb = false, kmreq = false;
    uint32_t pa0 = 0, pa2 = 0, pb0 = 0, pb2 = 0;
    int pae = 0, pbe = 0;
    uint4 D[SM_SLOTS];
#pragma unroll
    for (int s = 0; s < SM_SLOTS; ++s) D[s] = make_uint4(0, 0, 0, 0);
    // termination guard: no read needs 2^20 trips (a 320-base read takes a few thousand); should a lane ever cycle,
    // the wave stops and hands every read it still owns to the retry pass instead of spinning on the device
    const int64_t trip_cap = (int64_t)((n - 1 - (int)blockIdx.x * 64) / lstride + 1) << 20;
    int64_t trips = 0;
    bool stuck = false;

    for (;;) {
        const uint4 *ad[SM_SLOTS];
        uint32_t vm = 0;
        int spins = 0;
        for (bool go = true; go;) {
            if (++spins > (1 << 16)) { stuck = true; break; }
            switch (st) {
            case SMS_LOAD_REQ: {
                if (li >= n) { st = SMS_DONE; go = false; break; }
                const uint4 *p = reinterpret_cast<const uint4 *>(qpack + (size_t)li * nwp);
#pragma unroll
                for (int s = 0; s < SM_SLOTS; ++s)
                    if (4 * s < nwp) { ad[s] = p + s; vm |= 1u << s; }
                st = SMS_LOAD; go = false;
                break;
            }
            case SMS_LOAD: {
#pragma unroll
                for (int s = 0; s < SM_SLOTS; ++s)
                    if (4 * s < nwp) {
                        g_smem_u32[(4 * s) * 64 + lane] = D[s].x; g_smem_u32[(4 * s + 1) * 64 + lane] = D[s].y;
                        g_smem_u32[(4 * s + 2) * 64 + lane] = D[s].z; g_smem_u32[(4 * s + 3) * 64 + lane] = D[s].w;
                    }
                len = (int)qw(nw2 + nwh);
                Sa = SP<Intv>{intv_out + intv_slot_at_d(li, 0, cap)};
                {
                    const size_t me = ((size_t)li >> 6) * 64 * (size_t)gcap + ((size_t)li & 63);
                    L.gx0 = reinterpret_cast<uint32_t *>(spill) + me;
                    L.gx2 = reinterpret_cast<uint32_t *>(spill + spill_tot * 4) + me;
                    L.gend = reinterpret_cast<uint32_t *>(spill + spill_tot * 8) + me;
                }
                Sn = 0; Sn1 = 0; ovf = false; x = 0;
                st = SMS_P1;
                break;
            }
            case SMS_P1: {   // while (x < len) { if (q[x] < 4) x = smem1(x, 1), take_mem1; else ++x; }
                while (x < len && qv(x) > 3) ++x;
                if (x >= len) { old_n = Sn; k2 = 0; st = SMS_P2_REQ; break; }
                sx = x; min_intv = 1; ret_to = 0;
                st = SMS_START;
                break;
            }
            case SMS_START: {   // bwt_smem1 entry and its forward k-mer prefix (smem1_lds lines 316-347)
                Sn1 = 0;
                const int c0 = qv(sx);
                if (c0 > 3) { ret = sx + 1; st = SMS_RET; break; }
                if (min_intv < 1) min_intv = 1;
                ik0 = fm.L2(c0) + 1; ik1 = fm.L2(3 - c0) + 1; ik2 = fm.L2(c0 + 1) - fm.L2(c0);
                ikend = sx + 1; n_l = 0; i = sx + 1; fcode = (uint32_t)c0; stop = false;
                Lt = K < len - sx ? K : len - sx;
                nt = 1;
                while (nt < Lt && qv(sx + nt) < 4) ++nt;
                pt = 2;
                if (nt >= 2) {
#pragma unroll
                    for (int s = 0; s < SM_SLOTS; ++s) {
                        const int t = pt + s;
                        if (t <= nt) {
                            fcode = fcode << 2 | (uint32_t)q2(sx + t - 1);
                            ad[s] = fm.kt + koff(t) + fcode; vm |= 1u << s;
                        }
                    }
                    st = SMS_PRE; go = false;
                    break;
                }
                // no prefix rows: the post-prefix bookkeeping below
                if (!stop) {
                    i = sx + nt;
                    if (nt < Lt) {
                        if (n_l >= L.total()) { ovf = true; st = SMS_FIN; break; }
                        L.set(n_l++, ik0, ik2, ikend);
                        stop = true;
                    }
                }
                st = stop ? SMS_FWD_END : SMS_FWD_NEXT;
                break;
            }
            case SMS_PRE: {   // consume prefix rows pt .. min(nt, pt + 7)
                const int last = nt < pt + SM_SLOTS - 1 ? nt : pt + SM_SLOTS - 1;
                nkm += (uint64_t)(last - pt + 1);
#pragma unroll
                for (int s = 0; s < SM_SLOTS; ++s) {
                    const int t = pt + s;
                    if (t <= last && !stop && !ovf) {
                        const uint32_t n0 = D[s].x, n2 = D[s].y;
                        if (n2 != ik2) {
                            if (n_l >= L.total()) ovf = true;
                            else {
                                L.set(n_l++, ik0, ik2, ikend);
                                if (n2 < (uint32_t)min_intv) { stop = true; i = sx + t - 1; }
                            }
                        }
                        if (!stop && !ovf) { ik0 = n0; ik2 = n2; ikend = sx + t; }
                    }
                }
                if (ovf) { st = SMS_FIN; break; }
                if (!stop && last == nt) {
#pragma unroll
                    for (int s = 0; s < SM_SLOTS; ++s) if (s == nt - pt) ik1 = D[s].z;   // x[1] of row nt
                }
                pt = last + 1;
                if (!stop && pt <= nt) {   // the next rows
#pragma unroll
                    for (int s = 0; s < SM_SLOTS; ++s) {
                        const int t = pt + s;
                        if (t <= nt) {
                            fcode = fcode << 2 | (uint32_t)q2(sx + t - 1);
                            ad[s] = fm.kt + koff(t) + fcode; vm |= 1u << s;
                        }
                    }
                    go = false;
                    break;
                }
                if (!stop) {
                    i = sx + nt;
                    if (nt < Lt) {
                        if (n_l >= L.total()) { ovf = true; st = SMS_FIN; break; }
                        L.set(n_l++, ik0, ik2, ikend);
                        stop = true;
                    }
                }
                st = stop ? SMS_FWD_END : SMS_FWD_NEXT;
                break;
            }
            case SMS_FWD_NEXT: {   // one forward extension (smem1_lds lines 376-430, without the text walk)
                if (stop || i >= len) { st = SMS_FWD_END; break; }
                const int cur = qv(i);
                if (cur < 4) {
                    c = 3 - cur;
                    fcode = fcode << 2 | (uint32_t)cur;
                    if (i - sx + 1 <= K) { ad[0] = fm.kt + koff(i - sx + 1) + fcode; vm |= 1u; st = SMS_FWD_KM; }
                    else { sm_req_blocks<0>(fm, ik1, ik2, ad, vm); st = SMS_FWD_EXT; }
                    go = false;
                } else {
                    if (n_l >= L.total()) { ovf = true; st = SMS_FIN; break; }
                    L.set(n_l++, ik0, ik2, ikend);
                    st = SMS_FWD_END;
                }
                break;
            }
            case SMS_FWD_EXT:
            case SMS_FWD_KM: {
                uint32_t n0, n1, n2;
                if (st == SMS_FWD_KM) { n0 = D[0].x; n2 = D[0].y; n1 = D[0].z; ++nkm; }
                else {   // extend1(fm, ik1, ik0, ik2, c): a = ik1, o = ik0
                    uint32_t kc, kg, lc, lg;
                    sm_sums<0>(fm, D, ik1, ik2, c, kc, kg, lc, lg, nblk);
                    n1 = fm.L2(c) + 1 + kc;
                    n2 = lc - kc;
                    n0 = ik0 + (uint32_t)(ik1 <= fm.primary && ik1 + ik2 - 1 >= fm.primary) + (lg - kg);
                }
                if (n2 != ik2) {
                    if (n_l >= L.total()) { ovf = true; st = SMS_FIN; break; }
                    L.set(n_l++, ik0, ik2, ikend);
                    if (n2 < (uint32_t)min_intv) { st = SMS_FWD_END; break; }
                }
                ik0 = n0; ik1 = n1; ik2 = n2; ikend = i + 1; ++i;
                st = SMS_FWD_NEXT;
                break;
            }
            case SMS_FWD_END: {   // final push, reversal, backward-loop setup (smem1_lds lines 431-457)
                if (i == len) {
                    if (n_l >= L.total()) { ovf = true; st = SMS_FIN; break; }
                    L.set(n_l++, ik0, ik2, ikend);
                }
                for (int jj = 0; jj < (n_l >> 1); ++jj) {
                    uint32_t a0, b0, a2, b2;
                    int ae, be;
                    L.get(jj, a0, a2, ae);
                    L.get(n_l - 1 - jj, b0, b2, be);
                    L.set(jj, b0, b2, be);
                    L.set(n_l - 1 - jj, a0, a2, ae);
                }
                { uint32_t d0, d2; L.get(0, d0, d2, ret); }
                last_start = 0x7fffffff;
                wcode = 0;
                for (int t = 0; t < K; ++t) wcode = wcode << 2 | (sx + t < len ? (uint32_t)q2(sx + t) : 0u);
                i = sx - 1;
                c = i < 0 ? -1 : (qv(i) < 4 ? qv(i) : -1);
                if (K > 0 && c >= 0) wcode = wcode >> 2 | (uint32_t)c << (2 * (K - 1));
                nc = 0; j = 0; last_x2 = 0;
                st = SMS_BWD_REQ;
                break;
            }
            case SMS_BWD_REQ: {   // entries j, j+1 of position i: their k-mer rows or rank blocks
                hb = j + 1 < n_l;
                L.get(j, pa0, pa2, pae);
                L.get(hb ? j + 1 : j, pb0, pb2, pbe);
                if (c >= 0) {
                    const int La = pae - i, Lb = pbe - i;
                    ta = La <= K; tb = hb && Lb <= K;
                    if (ta) { ad[0] = fm.kt + koff(La) + (wcode >> (2 * (K - La))); vm |= 1u; }
                    else sm_req_blocks<0>(fm, pa0, pa2, ad, vm);
                    if (hb) {
                        if (tb) { ad[4] = fm.kt + koff(Lb) + (wcode >> (2 * (K - Lb))); vm |= 16u; }
                        else sm_req_blocks<4>(fm, pb0, pb2, ad, vm);
                    }
                    st = SMS_BWD; go = false;
                } else st = SMS_BWD;
                break;
            }
            case SMS_BWD: {   // smem1_lds lines 470-511
                uint32_t oa0 = 0, ob0 = 0, oa2 = 0, ob2 = 0;
                if (c >= 0) {
                    uint32_t kc, kg, lc, lg;
                    if (ta) { oa0 = D[0].x; oa2 = D[0].y; }
                    else { sm_sums<0>(fm, D, pa0, pa2, c, kc, kg, lc, lg, nblk); oa0 = fm.L2(c) + 1 + kc; oa2 = lc - kc; }
                    if (hb) {
                        if (tb) { ob0 = D[4].x; ob2 = D[4].y; }
                        else { sm_sums<4>(fm, D, pb0, pb2, c, kc, kg, lc, lg, nblk); ob0 = fm.L2(c) + 1 + kc; ob2 = lc - kc; }
                    }
                    nkm += (uint64_t)ta + (uint64_t)(hb && tb);
                }
                for (int h = 0; h < 2; ++h) {
                    if (h == 1 && !hb) break;
                    const uint32_t p0 = h ? pb0 : pa0, o0 = h ? ob0 : oa0, p2 = h ? pb2 : pa2, o2 = h ? ob2 : oa2;
                    const int pe = h ? pbe : pae;
                    const bool keep_hit = c < 0 || o2 < (uint32_t)min_intv;
                    if (keep_hit) {
                        if (nc == 0 && (Sn1 == 0 || i + 1 < last_start)) {
                            if (Sn + Sn1 >= cap) { ovf = true; break; }
                            Intv &m = Sa[cap - 1 - Sn1];
                            m.x[0] = p0; m.x[1] = 0; m.x[2] = p2;
                            m.info = (uint64_t)(uint32_t)(i + 1) << 32 | (uint32_t)pe;
                            ++Sn1;
                            last_start = i + 1;
                        }
                    } else if (nc == 0 || o2 != last_x2) {
                        L.set(nc++, o0, o2, pe);
                        last_x2 = o2;
                    }
                }
                if (ovf) { st = SMS_FIN; break; }
                j += 2;
                st = SMS_BWD_REQ;
                if (j >= n_l) {
                    if (nc == 0) { st = SMS_RET; break; }
                    n_l = nc; nc = 0; j = 0; last_x2 = 0;
                    --i;
                    c = i < 0 ? -1 : (qv(i) < 4 ? qv(i) : -1);
                    if (K > 0 && c >= 0) wcode = wcode >> 2 | (uint32_t)c << (2 * (K - 1));
                }
                break;
            }
            case SMS_RET: {   // back in the caller: pass 1 continues at x = ret; both passes take mem1 first
                if (ret_to == 0) x = ret;
                tk = 0;
                st = SMS_TAKE_REQ;
                break;
            }
            case SMS_TAKE_REQ: {   // take_mem1: mem1 (reversed emission order) sits at Sa[cap - Sn1 .. cap)
                if (tk >= Sn1) {
                    Sn1 = 0;
                    if (ret_to == 0) st = SMS_P1;
                    else { ++k2; st = SMS_P2_REQ; }
                    break;
                }
#pragma unroll
                for (int s = 0; s < 4; ++s)
                    if (tk + s < Sn1) {
                        const uint4 *e = reinterpret_cast<const uint4 *>(&Sa[cap - Sn1 + tk + s]);
                        ad[2 * s] = e; ad[2 * s + 1] = e + 1; vm |= 3u << (2 * s);
                    }
                st = SMS_TAKE; go = false;
                break;
            }
            case SMS_TAKE: {
#pragma unroll
                for (int s = 0; s < 4; ++s)
                    if (tk + s < Sn1) {
                        const uint64_t m0 = u64_of(D[2 * s].x, D[2 * s].y), m2 = u64_of(D[2 * s + 1].x, D[2 * s + 1].y);
                        const uint64_t mi = u64_of(D[2 * s + 1].z, D[2 * s + 1].w);
                        const uint32_t s0 = (uint32_t)(mi >> 32), en = (uint32_t)mi;
                        const bool keep = ret_to ? (uint64_t)(en - s0) >= (uint64_t)o.min_seed_len : (int)(en - s0) >= o.min_seed_len;
                        if (keep) { Intv &d = Sa[Sn++]; d.x[0] = m0; d.x[1] = 0; d.x[2] = m2; d.info = mi; }
                    }
                tk += 4;
                st = SMS_TAKE_REQ;
                break;
            }
            case SMS_P2_REQ: {   // pass 2: re-seed long SMEMs of few occurrences from their middle
                if (k2 >= old_n) { st = SMS_P3; break; }
                const uint4 *e = reinterpret_cast<const uint4 *>(&Sa[k2]);
                ad[0] = e; ad[1] = e + 1; vm |= 3u;
                st = SMS_P2; go = false;
                break;
            }
            case SMS_P2: {
                const uint64_t px2 = u64_of(D[1].x, D[1].y), pinfo = u64_of(D[1].z, D[1].w);
                const int start = (int)(pinfo >> 32), end = (int)(uint32_t)pinfo;
                if (end - start < split_len || px2 > (uint64_t)o.split_width) { ++k2; st = SMS_P2_REQ; break; }
                sx = (start + end) >> 1; min_intv = (int)px2 + 1; ret_to = 1;
                st = SMS_START;
                break;
            }
            case SMS_P3: {
                if (o.max_mem_intv > 0) { x = 0; st = SMS_SS_LOOP; } else st = SMS_FIN;
                break;
            }
            case SMS_SS_LOOP: {   // bwt_seed_strategy1 over x (seed_strategy1_x)
                while (x < len && qv(x) > 3) ++x;
                if (x >= len) { st = SMS_FIN; break; }
                const int c0 = qv(x);
                ik0 = fm.L2(c0) + 1; ik1 = fm.L2(3 - c0) + 1; ik2 = fm.L2(c0 + 1) - fm.L2(c0);
                fcode = (uint32_t)c0;
                i = x + 1;
                st = SMS_SS_NEXT;
                if (K > 1 && o.min_seed_len >= K) {
                    const int Ls = K < len - x ? K : len - x;
                    int t = 1;
                    for (; t < Ls; ++t) {
                        const int cc = qv(x + t);
                        if (cc > 3) break;
                        fcode = fcode << 2 | (uint32_t)cc;
                    }
                    if (t < Ls) { x = x + t + 1; st = SMS_SS_LOOP; break; }
                    i = x + Ls;
                    if (Ls > 1) { ad[0] = fm.kt + koff(Ls) + fcode; vm |= 1u; st = SMS_SS_KM; go = false; }
                }
                break;
            }
            case SMS_SS_KM: {
                ik0 = D[0].x; ik2 = D[0].y; ik1 = D[0].z; ++nkm;
                st = SMS_SS_NEXT;
                break;
            }
            case SMS_SS_NEXT: {
                if (i >= len) { x = len; st = SMS_SS_LOOP; break; }
                const int cur = qv(i);
                if (cur > 3) { x = i + 1; st = SMS_SS_LOOP; break; }
                c = 3 - cur;
                fcode = fcode << 2 | (uint32_t)cur;
                kmreq = i - x + 1 <= K;
                if (kmreq) { ad[0] = fm.kt + koff(i - x + 1) + fcode; vm |= 1u; }
                else sm_req_blocks<0>(fm, ik1, ik2, ad, vm);
                st = SMS_SS_EXT; go = false;
                break;
            }
            case SMS_SS_EXT: {
                uint32_t n0, n1, n2;
                if (kmreq) { n0 = D[0].x; n2 = D[0].y; n1 = D[0].z; ++nkm; }
                else {
                    uint32_t kc, kg, lc, lg;
                    sm_sums<0>(fm, D, ik1, ik2, c, kc, kg, lc, lg, nblk);
                    n1 = fm.L2(c) + 1 + kc;
                    n2 = lc - kc;
                    n0 = ik0 + (uint32_t)(ik1 <= fm.primary && ik1 + ik2 - 1 >= fm.primary) + (lg - kg);
                }
                if (n2 < (uint32_t)o.max_mem_intv && i - x >= o.min_seed_len) {
                    if (n2 > 0) {
                        if (Sn >= cap) { ovf = true; st = SMS_FIN; break; }
                        Intv &d = Sa[Sn++];
                        d.x[0] = n0; d.x[1] = n1; d.x[2] = n2; d.info = (uint64_t)x << 32 | (uint64_t)(i + 1);
                    }
                    x = i + 1;
                    st = SMS_SS_LOOP;
                } else {
                    ik0 = n0; ik1 = n1; ik2 = n2; ++i;
                    st = SMS_SS_NEXT;
                }
                break;
            }
            case SMS_FIN: {
                if (ovf) { atomicOr(&status[li], ST_OVERFLOW); n_intv[li] = 0; }
                else n_intv[li] = Sn;
                li += lstride;
                st = SMS_LOAD_REQ;
                break;
            }
            default:   // SMS_DONE
                go = false;
                break;
            }
        }
        if (__ballot(stuck) != 0 || ++trips > trip_cap) {
            for (; li < n; li += lstride) { atomicOr(&status[li], ST_OVERFLOW); n_intv[li] = 0; }
            break;
        }
        if (__ballot(st != SMS_DONE) == 0) break;
#pragma unroll
        for (int s = 0; s < SM_SLOTS; ++s)
            if (vm & (1u << s)) D[s] = *ad[s];
    }
    wave_add2(&ctr[STG_SMEM].occ_blocks, nblk);
    wave_add2(&ctr[STG_SMEM].kmer_hits, nkm);
}

// Main-pass seeding through k_smem_sm (u32 rows, max_len <= SM_MAXLEN): pack the reads, run the lanes, sort the
// intervals of each read.  qpack: a workspace buffer of n * sm_words(max_len) u32.
int sm_words(int max_len) { return ((max_len + 15) / 16 + (max_len + 31) / 32 + 1 + 3) & ~3; }
bool sm_applies(const DIndex &ix, int max_len) { return !ix.wide && max_len <= SM_MAXLEN; }

hipError_t launch_smem_sm(hipStream_t st, const DIndex &ix, const DOpts &o, const Caps &cp, const uint8_t *codes,
                          const int64_t *offs, int n, Intv *intv, int32_t *n_intv, uint32_t *status, Counters *ctr,
                          int lcap, uint8_t *spill, int gcap, uint32_t *qpack, int reads_per_lane)
{
    if (n <= 0) return hipSuccess;
    const int nw2 = (cp.max_len + 15) / 16, nwh = (cp.max_len + 31) / 32, nwp = sm_words(cp.max_len);
    hipLaunchKernelGGL(k_pack_reads, dim3((n + 255) / 256), dim3(256), 0, st, codes, offs, n, nwp, nw2, nwh, qpack);
    const int waves = (n + 63) / 64;
    const int rpl = reads_per_lane > 0 ? reads_per_lane : 1;
    const int grid = (waves + rpl - 1) / rpl;
    const size_t sh = (size_t)nwp * 64 * 4 + lds_bytes<uint32_t, uint32_t>(64, lcap);
    hipLaunchKernelGGL(k_smem_sm, dim3(grid), dim3(64), sh, st, ix, o, cp, (const uint32_t *)qpack, nwp, nw2, nwh, n, intv,
                       n_intv, status, ctr, lcap, spill, gcap);
    hipLaunchKernelGGL(k_intv_sort, dim3((n + 255) / 256), dim3(256), 0, st, n, intv, (const int32_t *)n_intv, cp.intv);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// k-mer interval table build (index upload): level 1 from L2, level L+1 from level L by one full
// backward bwt_extend per parent (prepending base c to S gives code c * 4^L + code(S)).  The
// bidirectional interval of a string does not depend on the extension path that reached it, so a
// table entry equals what the kernels' forward or backward extend chains compute for that string
// (only non-empty intervals are ever consumed; empty ones are only compared against x[2] bounds).
template <typename X>
__global__ void k_kmer_level(DIndex ix, void *tabv, int L)
{
    const uint64_t n = 1ull << (2 * L);
    const uint64_t P = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    auto put = [&](uint64_t idx, X a0, X a1, X a2) {
        if constexpr (sizeof(X) == 4) {
            reinterpret_cast<uint4 *>(tabv)[idx] = make_uint4(a0, a2, a1, 0u);
        } else {
            ulonglong2 *p = reinterpret_cast<ulonglong2 *>(tabv) + 2 * idx;
            p[0] = make_ulonglong2(a0, a2);
            p[1] = make_ulonglong2(a1, 0ull);
        }
    };
    if (L == 0) {
        if (P < 4) {
            const int c = (int)P;
            put(P, (X)ix.L2[c] + 1, (X)ix.L2[3 - c] + 1, (X)(ix.L2[c + 1] - ix.L2[c]));
        }
        return;
    }
    if (P >= n) return;
    FM<X> fm;
    fm.occ = ix.occ;
    fm.occ32 = ix.occ32;
    fm.sup = ix.sup;
    fm.kt = reinterpret_cast<const uint4 *>(tabv);
    fm.K = 0;
    fm.l2_0 = (X)ix.L2[0]; fm.l2_1 = (X)ix.L2[1]; fm.l2_2 = (X)ix.L2[2];
    fm.l2_3 = (X)ix.L2[3]; fm.l2_4 = (X)ix.L2[4];
    fm.primary = (X)ix.primary;
    X x0, x1, x2;
    fm.kget((uint32_t)(koff(L) + P), x0, x1, x2);
    X o0[4], o2[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        X na, no, nx2;
        uint64_t nb = 0;
        extend1(fm, x0, (X)0, x2, c, na, no, nx2, nb);
        o0[c] = na; o2[c] = nx2;
    }
    const X x1_3 = x1 + (X)(x0 <= fm.primary && x0 + x2 - 1 >= fm.primary);
    const X x1_2 = x1_3 + o2[3], x1_1 = x1_2 + o2[2], x1_0 = x1_1 + o2[1];
    const uint64_t d = koff(L + 1) + P;
    put(d + 0 * n, o0[0], x1_0, o2[0]);
    put(d + 1 * n, o0[1], x1_1, o2[1]);
    put(d + 2 * n, o0[2], x1_2, o2[2]);
    put(d + 3 * n, o0[3], x1_3, o2[3]);
}

// entry bytes: 16 (u32 rows) or 32 (64-bit rows)
hipError_t launch_kmer_build(hipStream_t st, const DIndex &ix, uint32_t *tab, int K)
{
    for (int L = 0; L < K; ++L) {
        const uint64_t n = L == 0 ? 4 : 1ull << (2 * L);
        const dim3 g((unsigned)((n + 255) / 256)), bl(256);
        if (ix.wide) hipLaunchKernelGGL(k_kmer_level<uint64_t>, g, bl, 0, st, ix, (void *)tab, L);
        else hipLaunchKernelGGL(k_kmer_level<uint32_t>, g, bl, 0, st, ix, (void *)tab, L);
    }
    return hipGetLastError();
}

}  // namespace bsq
