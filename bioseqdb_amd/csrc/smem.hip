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
        // rows preloaded: 11, or 15 for 64-bit rows (whose table is 15 deep: C4; 162 VGPRs as with 13, and the C4
        // step 31.7 -> 32.5 M reads/s against 13 levels); a table deeper than KM
        // (BSQ_KMER_K up to 15 for u32 rows) serves lengths KM+1..K one per step below
        constexpr int KM = sizeof(X) == 8 ? 15 : 11;
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
DEV int seed_strategy1_x(const FM<X> &fm, int len, Q q, int x, int min_len, int max_intv, Intv &mem,
                         uint64_t &nblk, uint64_t &nkm)
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
template <typename X, typename Z, typename Q>
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
                x = smem1_lds(fm, len, q, x, 1, L, S, ovf, nblk, nkm);
                if (!ovf) take_mem1(false);
            } else ++x;
        }
        const int old_n = S.n;
        for (int k = 0; k < old_n && !ovf; ++k) {
            const Intv p = S.a[k];
            const int start = (int)(p.info >> 32), end = (int)(uint32_t)p.info;
            if (end - start < split_len || p.x[2] > (uint64_t)o.split_width) continue;
            smem1_lds(fm, len, q, (start + end) >> 1, (int)p.x[2] + 1, L, S, ovf, nblk, nkm);
            if (!ovf) take_mem1(true);
        }
        if (o.max_mem_intv > 0) {
            x = 0;
            while (x < len && !ovf) {
                if (q[x] < 4) {
                    Intv m;
                    x = seed_strategy1_x<X, Z>(fm, len, q, x, o.min_seed_len, o.max_mem_intv, m, nblk, nkm);
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
    if (const char *g = getenv("BSQ_SMEM_GRID")) { const int c = atoi(g); if (c > 0 && c < grid) grid = c; }
    const int L = cp.max_len;
    if (codes_t)
        hipLaunchKernelGGL(k_codes_wave, dim3((n + 63) / 64), dim3(256), (size_t)64 * L, st, codes, offs, n, L, codes_t);
#define BSQ_SMEM_LAUNCH(X_, Z_)                                                                                         \
    do {                                                                                                               \
        const size_t sh = lds_bytes<X_, Z_>(T, lcap);                                                                  \
        if (codes_t)                                                                                                   \
            hipLaunchKernelGGL((k_smem_lds<X_, Z_, QT>), dim3(grid), dim3(T), sh, st, ix, o, cp, codes_t, offs, n,      \
                               intv, n_intv, status, ctr, lcap, spill, gcap, L);                                       \
        else                                                                                                           \
            hipLaunchKernelGGL((k_smem_lds<X_, Z_, const uint8_t *>), dim3(grid), dim3(T), sh, st, ix, o, cp, codes,    \
                               offs, n, intv, n_intv, status, ctr, lcap, spill, gcap, L);                              \
    } while (0)
    if (!ix.wide) BSQ_SMEM_LAUNCH(uint32_t, uint32_t);
    else if (wide_z32(ix)) BSQ_SMEM_LAUNCH(uint64_t, uint32_t);   // 64-bit rows, interval sizes in u32 (l_pac < 2^32)
    else BSQ_SMEM_LAUNCH(uint64_t, uint64_t);
#undef BSQ_SMEM_LAUNCH
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
