// dp_wave.hip -- wave-cooperative banded DP for mem_reg2aln (libbwa bwa_gen_cigar2 / ksw_global2).
//
// One 64-lane wave per read; the read's regions are processed in order with wave-uniform control
// (every lane computes the same scalars) and lane-parallel DP rows:
//   * lane l owns query column beg + 64*chunk + l of the current target row;
//   * the ksw_global2 row state eh[0..qlen] (H(i-1,j-1), E(i,j)) lives in LDS, so cells outside the
//     band keep exactly the values the serial kernel would leave there;
//   * the F (insertion) recurrence F(j+1) = max(F(j) - e_ins, M(j) - oe_ins) is evaluated as an
//     exclusive max-plus prefix scan across lanes, F(j) = max(F0 - (j-c0)e, max_{k<j}(t_k - (j-1-k)e));
//   * the traceback matrix z (one byte per cell, same bits as ksw) is written row by row into LDS,
//     coalesced, and walked back uniformly.
// Integer arithmetic only; results equal the serial ksw_global2 cell for cell.
// Restates algorithms of BWA (lh3/bwa, Apache-2.0) and klib (MIT) for bit-exact results; see NOTICE.
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <stdint.h>

#include "bsq_device.h"
#include "dev_common.h"
#include "../../include/bsq.h"

namespace bsq {

#define NEG_SCAN (-0x3fffffff - 0x3fffffff)   // scan identity far below any reachable value
#define MINUS_INF_W (-0x40000000)

DEV void lds_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

DEV int lane_id() { return threadIdx.x & 63; }

// wave64 exclusive max-scan with DPP (row_shr 1/2/4/8, row_bcast 15/31, wave_shr 1): gfx9-family
#define DPP_STEP(v, ctrl, rmask) { int u_ = __builtin_amdgcn_update_dpp(NEG_SCAN, v, ctrl, rmask, 0xf, false); v = v > u_ ? v : u_; }
DEV int wave_excl_max(int v)
{
    DPP_STEP(v, 0x111, 0xf);
    DPP_STEP(v, 0x112, 0xf);
    DPP_STEP(v, 0x114, 0xf);
    DPP_STEP(v, 0x118, 0xf);
    DPP_STEP(v, 0x142, 0xa);
    DPP_STEP(v, 0x143, 0xc);
    return __builtin_amdgcn_update_dpp(NEG_SCAN, v, 0x138, 0xf, 0xf, false);   // wave_shr:1
}

// lane l receives v of lane l-1; lane 0 receives `first`
DEV int wave_shr1(int v, int first) { return __builtin_amdgcn_update_dpp(first, v, 0x138, 0xf, 0xf, false); }

// Scans and reductions over G consecutive lanes (a group; G = 64: the wave) with DPP: row_shr 1/2/4/8 within
// each 16-lane row, row_bcast 15/31 across rows; lanes whose source is outside the group keep the identity.
// (Cross-lane shuffles compile to ds_bpermute, an LDS round trip per step.)
#define DPP_ID(op, v, id, ctrl, rmask) { const int u_ = __builtin_amdgcn_update_dpp(id, v, ctrl, rmask, 0xf, false); v = op(v, u_); }
DEV int op_add(int a, int b) { return a + b; }
DEV int op_min(int a, int b) { return a < b ? a : b; }
DEV int op_max(int a, int b) { return a > b ? a : b; }
template <int G, int (*OP)(int, int)> DEV int grp_scan(int v, int id)
{
    DPP_ID(OP, v, id, 0x111, 0xf);
    DPP_ID(OP, v, id, 0x112, 0xf);
    DPP_ID(OP, v, id, 0x114, 0xf);
    DPP_ID(OP, v, id, 0x118, 0xf);
    if (G >= 32) DPP_ID(OP, v, id, 0x142, 0xa);   // row_bcast:15 into rows 1 and 3
    if (G == 64) DPP_ID(OP, v, id, 0x143, 0xc);   // row_bcast:31 into rows 2 and 3
    return v;
}
// every lane of the group receives the group's last lane
template <int G> DEV int grp_last(int v)
{
    if (G == 16) return __builtin_amdgcn_update_dpp(0, v, 0x15f, 0xf, 0xf, false);   // row_newbcast:15
    if (G == 32) {
        const int a = __builtin_amdgcn_readlane(v, 31), b = __builtin_amdgcn_readlane(v, 63);
        return (threadIdx.x & 32) ? b : a;
    }
    return __builtin_amdgcn_readlane(v, 63);
}
template <int G> DEV int grp_incl_sum(int v, int) { return grp_scan<G, op_add>(v, 0); }
template <int G> DEV int grp_incl_min(int v, int) { return grp_scan<G, op_min>(v, 0x7fffffff); }
template <int G> DEV int grp_max_all(int v) { return grp_last<G>(grp_scan<G, op_max>(v, NEG_SCAN)); }
template <int G> DEV int grp_sum(int v) { return grp_last<G>(grp_scan<G, op_add>(v, 0)); }
DEV int wave_sum(int v) { return grp_sum<64>(v); }

// The exact form of diagonal_wins (dev_common.h) for the diagonals it cannot decide: with diagonal score S,
// every path through ksw_global2's n x n matrix other than the diagonal has either
//   * g >= 2 insertions and as many deletions: at most (n-2)*mat_max - (o_ins + o_del + 2*(e_ins + e_del)), or
//   * one insertion and one deletion: it leaves the diagonal at a, runs along diagonal +1 (insertion first:
//     cells (i, i+1)) or -1 (deletion first: cells (i+1, i)) for i in [a, b), and rejoins at b+1, skipping
//     diagonal cells a..b: S - oe_ins - oe_del - s0[b] + C[b] - C[a], C the prefix sums of
//     delta[i] = (shifted cell's score) - s0[i]; the best such path is
//     S - oe_ins - oe_del + max_b (C[b] - min_{a<=b} C[a] - s0[b]), computed exactly here with scans.
// When S beats both, the diagonal is the unique optimum and (as in diagonal_wins) the DP's answer is "nM" / S.
// G lanes cooperate (gl = lane in the group); tq(j, t, q) gives the target and query bases at j.
template <int G, class TQ>
DEV bool detour_free(const DOpts &o, const Score sc, int n, int S, TQ tq, int gl)
{
    const int64_t bound2 = (int64_t)(n - 2) * o.mat_max - (o.o_ins + o.o_del + 2 * (o.e_ins + o.e_del));
    if ((int64_t)S <= bound2) return false;
    const int NEG = -0x3fffffff;
    int c1 = 0, cm = 0, m1 = 0, mm = 0, x = NEG;   // prefix sums and minima carried across chunks
    for (int c0 = 0; c0 < n; c0 += G) {
        const int j = c0 + gl;
        const bool act = j < n, nx = j + 1 < n;
        int tj = 0, qj = 0, tn = 0, qn = 0;
        if (act) tq(j, tj, qj);
        if (nx) tq(j + 1, tn, qn);
        const int s0 = act ? sc(tj, qj) : 0;
        const int d1 = nx ? sc(tj, qn) - s0 : 0, dm = nx ? sc(tn, qj) - s0 : 0;
        const int i1 = grp_incl_sum<G>(d1, gl), im = grp_incl_sum<G>(dm, gl);
        const int C1 = c1 + i1 - d1, Cm = cm + im - dm;   // C[j] = sum of delta[i], i < j
        int n1 = grp_incl_min<G>(act ? C1 : 0x3fffffff, gl), nm = grp_incl_min<G>(act ? Cm : 0x3fffffff, gl);
        n1 = n1 < m1 ? n1 : m1;
        nm = nm < mm ? nm : mm;
        if (act) {
            const int a1 = C1 - n1 - s0, am = Cm - nm - s0;
            x = x > a1 ? x : a1;
            x = x > am ? x : am;
        }
        c1 += grp_last<G>(i1);
        cm += grp_last<G>(im);
        m1 = grp_last<G>(n1);
        mm = grp_last<G>(nm);
    }
    x = grp_max_all<G>(x);
    return (int64_t)x < (int64_t)(o.o_ins + o.e_ins + o.o_del + o.e_del);
}

// ksw_global2 over accessor-defined sequences.  eh: LDS, qlen+1 entries.  z: LDS (n_col*tlen bytes)
// or nullptr (score only).  CIGAR (traceback) written to cig[] with libbwa push_cigar semantics.
extern __shared__ uint8_t g_lds_dp[];   // dynamic LDS of k_reg2aln_w
struct QW {   // query bases staged in this wave's LDS: base j at off + start + dir*j
    int off, start, dir;
    DEV int operator()(int j) const { return g_lds_dp[off + start + dir * j]; }
};

template <class QA>
DEV int ksw_global2_w(const DOpts &o, int qlen, QA query, int tlen, TAcc target, int o_del, int e_del, int o_ins,
                      int e_ins, int w, int2 *eh, uint8_t *z, int zcap, uint32_t *cig, int cap, int *ncig, bool &ovf,
                      uint64_t &cells)
{
    const int l = lane_id();
    const Score sc = score_of(o);
    const int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
    const int n_col = qlen < 2 * w + 1 ? qlen : 2 * w + 1;
    if (z && (int64_t)n_col * tlen > zcap) { ovf = true; return 0; }
    for (int j = l; j <= qlen; j += 64)
        eh[j] = j == 0 ? make_int2(0, MINUS_INF_W) : (j <= w ? make_int2(-(o_ins + e_ins * j), MINUS_INF_W)
                                                             : make_int2(MINUS_INF_W, MINUS_INF_W));
    lds_fence();
    TStream ts;
    if (tlen > 0) ts.init(*target.ix, target.start, target.dir);
    for (int i = 0; i < tlen; ++i) {
        const int tb = ts.next();   // uniform; next pac word prefetched
        const int beg = i > w ? i - w : 0;
        const int end = i + w + 1 < qlen ? i + w + 1 : qlen;
        int h_carry = beg == 0 ? -(o_del + e_del * (i + 1)) : MINUS_INF_W;
        int f_carry = MINUS_INF_W;
        cells += (uint64_t)(end > beg ? end - beg : 0);
        for (int c0 = beg; c0 < end; c0 += 64) {
            const int j = c0 + l;
            const bool act = j < end;
            int2 p = act ? eh[j] : make_int2(0, 0);
            const int m = p.x + (act ? sc(tb, query(j)) : 0);
            const int e = p.y;
            const int tf = m - oe_ins;
            const int g = act ? tf + l * e_ins : NEG_SCAN;
            const int ex = wave_excl_max(g);
            int f = f_carry - l * e_ins;
            if (l > 0) {
                const int fs = ex - (l - 1) * e_ins;
                f = f > fs ? f : fs;
            }
            int d = m >= e ? 0 : 1;
            int h = m >= e ? m : e;
            d = h >= f ? d : 2;
            h = h >= f ? h : f;
            const int te = m - oe_del, e2 = e - e_del;
            d |= e2 > te ? 1 << 2 : 0;
            const int enew = e2 > te ? e2 : te;
            const int f2 = f - e_ins;
            d |= f2 > tf ? 2 << 4 : 0;
            const int fnext = f2 > tf ? f2 : tf;
            const int hprev = wave_shr1(h, h_carry);
            if (act) {
                eh[j] = make_int2(hprev, enew);
                if (z) z[i * n_col + (j - beg)] = (uint8_t)d;
            }
            const int last = (end - 1 - c0) < 63 ? (end - 1 - c0) : 63;
            h_carry = __builtin_amdgcn_readlane(h, last);
            f_carry = __builtin_amdgcn_readlane(fnext, last);
        }
        if (l == 0) eh[end] = make_int2(h_carry, MINUS_INF_W);
        lds_fence();
    }
    const int score = eh[qlen].x;
    if (z) {
        int n = 0, which = 0, i = tlen - 1;
        int k = (i + w + 1 < qlen ? i + w + 1 : qlen) - 1;
        uint32_t cur = 0;   // pending op (len<<4|op), flushed on op change
        auto push = [&](int op, int len) {
            if (n > 0 && (int)(cur & 0xf) == op) { cur += (uint32_t)len << 4; return; }
            if (n > 0) {
                if (n - 1 >= cap) { ovf = true; return; }
                cig[n - 1] = cur;
            }
            cur = (uint32_t)len << 4 | (uint32_t)op;
            ++n;
        };
        while (i >= 0 && k >= 0 && !ovf) {
            which = z[i * n_col + (k - (i > w ? i - w : 0))] >> (which << 1) & 3;
            if (which == 0) push(0, 1), --i, --k;
            else if (which == 1) push(2, 1), --i;
            else push(1, 1), --k;
        }
        if (i >= 0) push(2, i + 1);
        if (k >= 0) push(1, k + 1);
        if (n > cap) ovf = true;
        if (!ovf && n > 0) cig[n - 1] = cur;
        if (!ovf)
            for (int a = 0; a < (n >> 1); ++a) { uint32_t t = cig[a]; cig[a] = cig[n - 1 - a]; cig[n - 1 - a] = t; }
        *ncig = ovf ? -1 : n;
    }
    return score;
}

// lane l receives v of lane l+1; the last lane receives `last`
DEV int wave_shl1(int v, int last) { return __builtin_amdgcn_update_dpp(last, v, 0x130, 0xf, 0xf, false); }

// ksw_global2 for bands of at most 64 columns with the row state held in registers.  In global mode the
// band is [max(0,i-w), min(i+w+1,qlen)): it slides by s = 0 or 1 column per row and grows by one at the
// right, and the column entering at the right reads (H(i-1,end-1), -inf), so the next row's state is
//   s == 0: Hd' = h of lane l-1 (lane 0: the column-0 boundary value), E' = e_new of lane l
//   s == 1: Hd' = h of lane l,                                        E' = e_new of lane l+1
// (-inf for the new column's E) -- exactly the eh[] values the serial kernel would read.
template <bool ZL>
DEV int ksw_global2_reg(const Score sc, int qlen, int q_off, int q_start, int q_dir, const DIndex &ix, int64_t t_start,
                        int t_dir, int tlen, int o_del, int e_del, int o_ins, int e_ins, int w, int n_col, int z_off,
                        uint8_t *zg, uint64_t &cells)
{
    const int l = lane_id();
    const int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
    // both sequences in registers, so the row loop has no memory wait: the target 2 bits per base, 16
    // per lane (row i's base = a scalar readlane); the query 4 bits per base, 8 per lane, plus qv =
    // q[beg + l], the band's columns, shifted along with the band
    uint32_t tw = 0;
    for (int k = 0; k < 16; ++k) {
        const int i = l * 16 + k;
        if (i < tlen) tw |= (uint32_t)ref_at(ix, t_start + (int64_t)t_dir * i) << (2 * k);
    }
    uint32_t qpk = 0;
    for (int k = 0; k < 8; ++k) {
        const int j = l * 8 + k;
        const uint32_t v = j < qlen ? (uint32_t)g_lds_dp[q_off + q_start + q_dir * j] : 4u;
        qpk |= v << (4 * k);
    }
    int qv = l < qlen ? g_lds_dp[q_off + q_start + q_dir * l] : 4;
    int Hd = l == 0 ? 0 : (l <= w ? -(o_ins + e_ins * l) : MINUS_INF_W);
    int E = MINUS_INF_W;
    int beg = 0, last_end = 0, width = 0, h = 0;
    for (int i = 0; i < tlen; ++i) {
        const int tb = (int)((uint32_t)__builtin_amdgcn_readlane((int)tw, i >> 4) >> (2 * (i & 15))) & 3;
        const int end = i + w + 1 < qlen ? i + w + 1 : qlen;
        width = end - beg;
        const bool act = l < width;
        const int m = Hd + sc(tb, qv);
        const int tf = m - oe_ins;
        const int ex = wave_excl_max(act ? tf + l * e_ins : NEG_SCAN);
        int f = MINUS_INF_W - l * e_ins;
        if (l > 0) { const int fs = ex - (l - 1) * e_ins; f = f > fs ? f : fs; }
        int d = m >= E ? 0 : 1;
        h = m >= E ? m : E;
        d = h >= f ? d : 2;
        h = h >= f ? h : f;
        const int te = m - oe_del, e2 = E - e_del;
        d |= e2 > te ? 1 << 2 : 0;
        const int enew = e2 > te ? e2 : te;
        const int f2 = f - e_ins;
        d |= f2 > tf ? 2 << 4 : 0;
        if (act) {
            if (ZL) g_lds_dp[z_off + i * n_col + l] = (uint8_t)d;
            else zg[i * n_col + l] = (uint8_t)d;
        }
        cells += (uint64_t)width;
        last_end = end;
        const int beg_next = i + 1 > w ? i + 1 - w : 0;
        if (beg_next == beg) {
            Hd = wave_shr1(h, -(o_del + e_del * (i + 1)));
            E = l < width ? enew : MINUS_INF_W;
        } else {
            Hd = h;
            const int es = wave_shl1(enew, MINUS_INF_W);
            E = l + 1 < width ? es : MINUS_INF_W;
            const int jn = beg_next + 63;   // column entering lane 63
            const int qn = jn < qlen ? (int)((uint32_t)__builtin_amdgcn_readlane((int)qpk, jn >> 3) >> (4 * (jn & 7))) & 15 : 4;
            qv = wave_shl1(qv, qn);
        }
        beg = beg_next;
    }
    if (tlen > 0 && last_end == qlen) return __builtin_amdgcn_readlane(h, width - 1);
    return qlen == 0 ? 0 : (qlen <= w ? -(o_ins + e_ins * qlen) : MINUS_INF_W);
}

// ksw_global2 for bands of 65..128 columns, row state in registers with TWO columns per lane (lane l owns band columns
// c0 = 2l and c1 = 2l + 1).  The rows are ksw_global2_reg's: the F recurrence is one wave scan over the lanes' pair
// maxima, F(c0) = max(F0 - c0*e, max_{c<c0} (tf_c - (c0-1-c)e)) and F(c1) = max(F(c0) - e, tf(c0)); a band slide by
// s = 0 moves H one column right (c1 of lane l-1 into c0 of lane l), s = 1 moves E and the query one column left.
// It replaces ksw_global2_w's LDS row (two 64-column chunks per row for these bands, an LDS round trip per chunk and a
// workgroup fence per row).  Same cells, same traceback bytes.
template <bool ZL>
DEV int ksw_global2_reg2(const Score sc, int qlen, int q_off, int q_start, int q_dir, const DIndex &ix, int64_t t_start,
                         int t_dir, int tlen, int o_del, int e_del, int o_ins, int e_ins, int w, int n_col, int z_off,
                         uint8_t *zg, uint64_t &cells)
{
    const int l = lane_id(), c0 = 2 * l, c1 = c0 + 1;
    const int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
    uint32_t tw = 0;   // target, 16 bases per lane (tlen <= 1024)
    for (int k = 0; k < 16; ++k) {
        const int i = l * 16 + k;
        if (i < tlen) tw |= (uint32_t)ref_at(ix, t_start + (int64_t)t_dir * i) << (2 * k);
    }
    uint32_t qpk = 0;   // query, 8 bases per lane (qlen <= 512)
    for (int k = 0; k < 8; ++k) {
        const int j = l * 8 + k;
        const uint32_t v = j < qlen ? (uint32_t)g_lds_dp[q_off + q_start + q_dir * j] : 4u;
        qpk |= v << (4 * k);
    }
    int qv0 = c0 < qlen ? g_lds_dp[q_off + q_start + q_dir * c0] : 4;
    int qv1 = c1 < qlen ? g_lds_dp[q_off + q_start + q_dir * c1] : 4;
    int Hd0 = c0 == 0 ? 0 : (c0 <= w ? -(o_ins + e_ins * c0) : MINUS_INF_W);
    int Hd1 = c1 <= w ? -(o_ins + e_ins * c1) : MINUS_INF_W;
    int E0 = MINUS_INF_W, E1 = MINUS_INF_W;
    int beg = 0, last_end = 0, width = 0, h0 = 0, h1 = 0;
    for (int i = 0; i < tlen; ++i) {
        const int tb = (int)((uint32_t)__builtin_amdgcn_readlane((int)tw, i >> 4) >> (2 * (i & 15))) & 3;
        const int end = i + w + 1 < qlen ? i + w + 1 : qlen;
        width = end - beg;
        const bool a0 = c0 < width, a1 = c1 < width;
        const int m0 = Hd0 + sc(tb, qv0), m1 = Hd1 + sc(tb, qv1);
        const int tf0 = m0 - oe_ins, tf1 = m1 - oe_ins;
        const int g0 = a0 ? tf0 + c0 * e_ins : NEG_SCAN, g1 = a1 ? tf1 + c1 * e_ins : NEG_SCAN;
        const int ex = wave_excl_max(g0 > g1 ? g0 : g1);
        int f0 = MINUS_INF_W - c0 * e_ins;
        if (l > 0) { const int fs = ex - (c0 - 1) * e_ins; f0 = f0 > fs ? f0 : fs; }
        int f1 = f0 - e_ins;
        f1 = f1 > tf0 ? f1 : tf0;
        int d0 = m0 >= E0 ? 0 : 1, d1 = m1 >= E1 ? 0 : 1;
        h0 = m0 >= E0 ? m0 : E0;
        h1 = m1 >= E1 ? m1 : E1;
        d0 = h0 >= f0 ? d0 : 2;
        d1 = h1 >= f1 ? d1 : 2;
        h0 = h0 >= f0 ? h0 : f0;
        h1 = h1 >= f1 ? h1 : f1;
        const int te0 = m0 - oe_del, e20 = E0 - e_del, te1 = m1 - oe_del, e21 = E1 - e_del;
        d0 |= e20 > te0 ? 1 << 2 : 0;
        d1 |= e21 > te1 ? 1 << 2 : 0;
        const int en0 = e20 > te0 ? e20 : te0, en1 = e21 > te1 ? e21 : te1;
        d0 |= f0 - e_ins > tf0 ? 2 << 4 : 0;
        d1 |= f1 - e_ins > tf1 ? 2 << 4 : 0;
        if (a0) {
            if (ZL) g_lds_dp[z_off + i * n_col + c0] = (uint8_t)d0;
            else zg[i * n_col + c0] = (uint8_t)d0;
        }
        if (a1) {
            if (ZL) g_lds_dp[z_off + i * n_col + c1] = (uint8_t)d1;
            else zg[i * n_col + c1] = (uint8_t)d1;
        }
        cells += (uint64_t)width;
        last_end = end;
        const int beg_next = i + 1 > w ? i + 1 - w : 0;
        if (beg_next == beg) {   // (only while beg == 0: column -1 is the boundary)
            Hd0 = wave_shr1(h1, -(o_del + e_del * (i + 1)));
            Hd1 = h0;
            E0 = a0 ? en0 : MINUS_INF_W;
            E1 = a1 ? en1 : MINUS_INF_W;
        } else {
            Hd0 = h0;
            Hd1 = h1;
            const int es = wave_shl1(en0, MINUS_INF_W);
            E0 = a1 ? en1 : MINUS_INF_W;
            E1 = c1 + 1 < width ? es : MINUS_INF_W;
            const int jn = beg_next + 127;   // column entering lane 63's second slot
            const int qn = jn < qlen ? (int)((uint32_t)__builtin_amdgcn_readlane((int)qpk, jn >> 3) >> (4 * (jn & 7))) & 15 : 4;
            const int qs = wave_shl1(qv0, qn);
            qv0 = qv1;
            qv1 = qs;
        }
        beg = beg_next;
    }
    if (tlen > 0 && last_end == qlen) {
        const int cw = width - 1;
        return __builtin_amdgcn_readlane((cw & 1) ? h1 : h0, cw >> 1);
    }
    return qlen == 0 ? 0 : (qlen <= w ? -(o_ins + e_ins * qlen) : MINUS_INF_W);
}

// traceback of a z matrix held in LDS (offset) or global memory; libbwa push_cigar semantics.
// G lanes cooperate (a DPP row, a 32-lane segment or the wave; gl = lane in the group, gbase = the
// group's first lane): in the match state the next G cells of the diagonal are read at once and a
// ballot finds the first one whose state-0 transition leaves the diagonal, so a diagonal run of r
// cells (mismatches included) is one push of r M's; other steps follow the serial loop exactly.
template <bool ZL, int G>
DEV void traceback_w(int qlen, int tlen, int w, int n_col, int z_off, const uint8_t *zg, uint32_t *cig, int cap,
                     int *ncig, bool &ovf, int gl = 0, int gbase = 0)
{
    if (G == 64) gl = lane_id();
    int n = 0, which = 0, i = tlen - 1;
    int k = (i + w + 1 < qlen ? i + w + 1 : qlen) - 1;
    uint32_t cur = 0;
    auto push = [&](int op, int len) {
        if (n > 0 && (int)(cur & 0xf) == op) { cur += (uint32_t)len << 4; return; }
        if (n > 0) {
            if (n - 1 >= cap) { ovf = true; return; }
            cig[n - 1] = cur;
        }
        cur = (uint32_t)len << 4 | (uint32_t)op;
        ++n;
    };
    auto zat = [&](int ii, int kk) -> int {
        const int idx = ii * n_col + (kk - (ii > w ? ii - w : 0));
        return ZL ? g_lds_dp[z_off + idx] : zg[idx];
    };
    while (i >= 0 && k >= 0 && !ovf) {
        if (which == 0) {
            const int ii = i - gl, kk = k - gl;
            const bool stop = ii < 0 || kk < 0 || (zat(ii, kk) & 3) != 0;
            const uint64_t bal = __ballot(stop);
            const uint64_t gm = G == 64 ? bal : (bal >> gbase) & ((1ull << G) - 1);
            const int r = gm ? (int)__builtin_ctzll(gm) : G;
            if (r > 0) {
                push(0, r);
                i -= r; k -= r;
                continue;
            }
        }
        which = zat(i, k) >> (which << 1) & 3;
        if (which == 0) push(0, 1), --i, --k;
        else if (which == 1) push(2, 1), --i;
        else push(1, 1), --k;
    }
    if (i >= 0) push(2, i + 1);
    if (k >= 0) push(1, k + 1);
    if (n > cap) ovf = true;
    if (!ovf && n > 0) cig[n - 1] = cur;
    if (!ovf)
        for (int a = 0; a < (n >> 1); ++a) { uint32_t t = cig[a]; cig[a] = cig[n - 1 - a]; cig[n - 1 - a] = t; }
    *ncig = ovf ? -1 : n;
}

// bwa_gen_cigar2, wave version
DEV int gen_cigar2_w(const DIndex &ix, const DOpts &o, int w_, int q_off, int qb, int l_query, int64_t rb,
                     int64_t re, int *score, int2 *eh, uint8_t *z, int z_off, int zcap, uint32_t *cig, int cap,
                     int *ncig, bool &ovf, uint64_t &cells, uint64_t &bases)
{
    *ncig = 0;
    if (l_query <= 0 || rb >= re || (rb < ix.l_pac && re > ix.l_pac)) return 0;
    const int64_t rlen = re - rb;
    if (re > (ix.l_pac << 1) || rb < 0) return 0;
    bases += (uint64_t)((rlen + 3) >> 2);
    const bool rev = rb >= ix.l_pac;
    QW qa{q_off, rev ? qb + l_query - 1 : qb, rev ? -1 : 1};
    TAcc ta{&ix, rev ? re - 1 : rb, rev ? -1 : 1};
    int s = 0;
    if (l_query == rlen) {
        const Score sc = score_of(o);
        for (int i = lane_id(); i < l_query; i += 64) s += sc(ta(i), qa(i));
        s = wave_sum(s);
    }
    const bool diag = l_query == rlen &&
                      (w_ == 0 || diagonal_wins(o, l_query, s) ||
                       detour_free<64>(o, score_of(o), l_query, s, [&](int j, int &t, int &q) { t = ta(j); q = qa(j); },
                                       lane_id()));
    if (diag) {
        if (cap < 1) { ovf = true; return 0; }
        cig[0] = (uint32_t)l_query << 4;
        *ncig = 1;
        *score = s;
    } else {
        int max_ins = idiv_plus(((l_query + 1) >> 1) * o.mat_match - o.o_ins, o.e_ins, 1);
        int max_del = idiv_plus(((l_query + 1) >> 1) * o.mat_match - o.o_del, o.e_del, 1);
        int max_gap = max_ins > max_del ? max_ins : max_del;
        max_gap = max_gap > 1 ? max_gap : 1;
        int dl = (int)rlen - l_query; dl = dl < 0 ? -dl : dl;
        int w = (max_gap + dl + 1) >> 1;
        w = w < w_ ? w : w_;
        const int min_w = dl + 3;
        w = w > min_w ? w : min_w;
        const int n_col = l_query < 2 * w + 1 ? l_query : 2 * w + 1;
        if (n_col <= 64 && rlen < (int64_t)l_query + w && rlen <= 1024 && l_query <= 512) {
            // register-resident rows and sequences; traceback matrix in LDS (z_off >= 0) or the global slab
            if ((int64_t)n_col * rlen > zcap) { ovf = true; return 0; }
            const bool zl = z_off >= 0;
            *score = zl ? ksw_global2_reg<true>(score_of(o), l_query, q_off, qa.start, qa.dir, ix, ta.start, ta.dir,
                                                (int)rlen, o.o_del, o.e_del, o.o_ins, o.e_ins, w, n_col, z_off,
                                                nullptr, cells)
                        : ksw_global2_reg<false>(score_of(o), l_query, q_off, qa.start, qa.dir, ix, ta.start, ta.dir,
                                                 (int)rlen, o.o_del, o.e_del, o.o_ins, o.e_ins, w, n_col, 0, z, cells);
            if (zl) traceback_w<true, 64>(l_query, (int)rlen, w, n_col, z_off, nullptr, cig, cap, ncig, ovf);
            else traceback_w<false, 64>(l_query, (int)rlen, w, n_col, 0, z, cig, cap, ncig, ovf);
        } else if (n_col <= 128 && rlen < (int64_t)l_query + w && rlen <= 1024 && l_query <= 512) {
            // two columns per lane (the bands of 65..128 columns the group kernels defer here)
            if ((int64_t)n_col * rlen > zcap) { ovf = true; return 0; }
            const bool zl = z_off >= 0;
            *score = zl ? ksw_global2_reg2<true>(score_of(o), l_query, q_off, qa.start, qa.dir, ix, ta.start, ta.dir,
                                                 (int)rlen, o.o_del, o.e_del, o.o_ins, o.e_ins, w, n_col, z_off,
                                                 nullptr, cells)
                        : ksw_global2_reg2<false>(score_of(o), l_query, q_off, qa.start, qa.dir, ix, ta.start, ta.dir,
                                                  (int)rlen, o.o_del, o.e_del, o.o_ins, o.e_ins, w, n_col, 0, z, cells);
            if (zl) traceback_w<true, 64>(l_query, (int)rlen, w, n_col, z_off, nullptr, cig, cap, ncig, ovf);
            else traceback_w<false, 64>(l_query, (int)rlen, w, n_col, 0, z, cig, cap, ncig, ovf);
        } else {
            *score = ksw_global2_w(o, l_query, qa, (int)rlen, ta, o.o_del, o.e_del, o.o_ins, o.e_ins, w, eh, z, zcap,
                                   cig, cap, ncig, ovf, cells);
        }
    }
    return 1;
}

// mem_reg2aln per region, one wave per read.  LDS per wave: eh (max_len+2 int2) + z (zcap bytes).
__global__ void __launch_bounds__(256) k_reg2aln_w(DIndex ix, DOpts o, Caps cp, const uint8_t *__restrict__ codes,
                                                   const int64_t *__restrict__ offs, int n,
                                                   const Reg *__restrict__ regs, const int32_t *__restrict__ n_regs,
                                                   Hit *__restrict__ hits, uint32_t *__restrict__ cigars,
                                                   int32_t *__restrict__ n_cig_read, uint32_t *__restrict__ status,
                                                   Counters *ctr, int zcap, uint8_t *__restrict__ zslab,
                                                   int64_t zslab_bytes, const int32_t *__restrict__ list,
                                                   const int32_t *__restrict__ list_n, int32_t *__restrict__ work)
{
    // the control below is wave-uniform: make that visible so it lives in SGPRs / scalar loads
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const size_t eh_bytes = ((size_t)(cp.max_len + 2) * sizeof(int2) + 15) & ~(size_t)15;
    const size_t q_bytes = ((size_t)cp.max_len + 16) & ~(size_t)15;
    const size_t per_wave = eh_bytes + (size_t)zcap + q_bytes;
    uint8_t *mine = g_lds_dp + (size_t)wave * per_wave;
    int2 *eh = reinterpret_cast<int2 *>(mine);
    uint8_t *z_lds = mine + eh_bytes;
    const int q_off = (int)((size_t)wave * per_wave + eh_bytes + (size_t)zcap);
    const int gw = blockIdx.x * (blockDim.x >> 6) + wave, nw = gridDim.x * (blockDim.x >> 6);
    uint8_t *z_glob = zslab + (size_t)gw * (size_t)zslab_bytes;   // this wave's spill slab
    uint64_t cells = 0, bases = 0;
    const int n_items = list ? *list_n : n;   // reads deferred by the group kernels, or all reads
    // Reads are taken from a work counter, one per wave at a time: their cost varies by 10x and more (bands of 33-77
    // columns, one to three band doublings, one or two regions), so a fixed stride left the launch waiting on the waves
    // that drew the expensive ones.  (work == nullptr: fixed stride.)
    auto next = [&](int cur) -> int {
        if (!work) return cur + nw;
        int v = 0;
        if (lane_id() == 0) v = atomicAdd(work, 1);   // one vector atomic per read
        return __builtin_amdgcn_readfirstlane(v);
    };
    for (int it_ = work ? next(0) : gw; it_ < n_items; it_ = next(it_)) {
    const int li = list ? list[it_] : it_;
    if (status[li]) { n_cig_read[li] = 0; continue; }
    {
        const uint8_t *q = codes + offs[li];
        const int l_query = (int)(offs[li + 1] - offs[li]);
        const int nr = n_regs[li];
        for (int j = lane_id(); j < l_query; j += 64) g_lds_dp[q_off + j] = q[j];   // stage the read
        lds_fence();
        bool ovf = false;
        int tot = 0;
        for (int g = 0; g < nr && !ovf; ++g) {
            const Reg ar = regs[(size_t)li * cp.regs + g];
            uint32_t *cig = cigars + ((size_t)li * cp.regs + g) * cp.cigar;
            const int qb = ar.qb, qe = ar.qe;
            const int64_t rb = ar.rb, re = ar.re;
            const int flag = ar.secondary >= 0 ? 0x100 : 0;
            int tmp = infer_bw(qe - qb, (int)(re - rb), ar.truesc, o.a, o.o_del, o.e_del);
            int w2 = infer_bw(qe - qb, (int)(re - rb), ar.truesc, o.a, o.o_ins, o.e_ins);
            w2 = w2 > tmp ? w2 : tmp;
            if (w2 > o.w) w2 = w2 < ar.w ? w2 : ar.w;
            int i = 0, score = 0, last_sc = -(1 << 30), ncig = 0;
            do {
                w2 = w2 < o.w << 2 ? w2 : o.w << 2;
                {   // traceback matrix in LDS when it fits, else in the wave's global slab
                    const int lq = qe - qb;
                    int64_t rl = re - rb;
                    int mg = idiv_plus(((lq + 1) >> 1) * o.mat_match - o.o_ins, o.e_ins, 1);
                    int md = idiv_plus(((lq + 1) >> 1) * o.mat_match - o.o_del, o.e_del, 1);
                    mg = mg > md ? mg : md; mg = mg > 1 ? mg : 1;
                    int dl = (int)rl - lq; dl = dl < 0 ? -dl : dl;
                    int ww = (mg + dl + 1) >> 1; ww = ww < w2 ? ww : w2; ww = ww > dl + 3 ? ww : dl + 3;
                    const int64_t need = (int64_t)(lq < 2 * ww + 1 ? lq : 2 * ww + 1) * rl;
                    const bool in_lds = need <= zcap;
                    gen_cigar2_w(ix, o, w2, q_off, qb, lq, rb, re, &score, eh, in_lds ? z_lds : z_glob,
                                 in_lds ? (int)((size_t)wave * per_wave + eh_bytes) : -1,
                                 in_lds ? zcap : (int)(zslab_bytes < 0x7fffffff ? zslab_bytes : 0x7fffffff), cig,
                                 cp.cigar - 2, &ncig, ovf, cells, bases);
                }
                if (ovf) break;
                if (score == last_sc || w2 == o.w << 2) break;
                last_sc = score;
                w2 <<= 1;
            } while (++i < 3 && score < ar.truesc - o.a);
            if (ovf) break;
            int is_rev;
            (void)depos(ix, rb < ix.l_pac ? rb : re - 1, is_rev);
            if (ncig > 0) {
                if ((cig[0] & 0xf) == 2) {
                    --ncig;
                    for (int t = 0; t < ncig; ++t) cig[t] = cig[t + 1];
                } else if ((cig[ncig - 1] & 0xf) == 2) --ncig;
            }
            if (qb != 0 || qe != l_query) {
                const int clip5 = is_rev ? l_query - qe : qb, clip3 = is_rev ? qb : l_query - qe;
                if (clip5) {
                    for (int t = ncig; t > 0; --t) cig[t] = cig[t - 1];
                    cig[0] = (uint32_t)clip5 << 4 | 3;
                    ++ncig;
                }
                if (clip3) cig[ncig++] = (uint32_t)clip3 << 4 | 3;
            }
            Hit h;
            h.rb = rb; h.re = re; h.qb = qb; h.qe = qe; h.rid = ar.rid; h.score = ar.score; h.flag = flag;
            h.is_rev = is_rev; h.n_cigar = ncig; h.pad = 0;
            hits[(size_t)li * cp.regs + g] = h;
            tot += ncig;
        }
        if (ovf) {
            if (lane_id() == 0) status[li] |= ST_OVERFLOW;
            n_cig_read[li] = 0;
        } else n_cig_read[li] = tot;
    }
    }
    // every lane ran the same uniform control; count once per wave
    if (lane_id() != 0) { cells = 0; bases = 0; }
    wave_add(&ctr[STG_REG2ALN].dp_cells, cells);
    wave_add(&ctr[STG_REG2ALN].ref_bases, bases);
}

hipError_t launch_reg2aln_w(hipStream_t st, const DIndex &ix, const DOpts &o, const Caps &cp, const uint8_t *codes,
                            const int64_t *offs, int n, const Reg *regs, const int32_t *n_regs, Hit *hits,
                            uint32_t *cigars, int32_t *n_cig, uint32_t *status, Counters *ctr, int zcap,
                            uint8_t *zslab, int64_t zslab_bytes, int max_blocks, const int32_t *list,
                            const int32_t *list_n, int32_t *work)
{
    const int waves = 4;
    int grid = (n + waves - 1) / waves;
    if (grid > max_blocks) grid = max_blocks;
    if (grid == 0) return hipSuccess;
    const size_t eh_bytes = ((size_t)(cp.max_len + 2) * sizeof(int2) + 15) & ~(size_t)15;
    const size_t q_bytes = ((size_t)cp.max_len + 16) & ~(size_t)15;
    const size_t sh = (size_t)waves * (eh_bytes + (size_t)zcap + q_bytes);
    if (work) {
        const hipError_t e = hipMemsetAsync(work, 0, sizeof(int32_t), st);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_reg2aln_w, dim3(grid), dim3(64 * waves), sh, st, ix, o, cp, codes, offs, n, regs, n_regs, hits,
                       cigars, n_cig, status, ctr, zcap, zslab, zslab_bytes, list, list_n, work);
    return hipGetLastError();
}

// ================================================================================================
// Group mode: 64/G reads per wave, one per G-lane group (G = 16: one DPP row; G = 32: two rows),
// for reads whose every ksw_global2 band fits G columns -- the common case (the band is ~10k+3
// columns for a read with k mismatches).  Control is per group (uniform within it); the DP row
// update is the register-row recurrence of ksw_global2_reg with segment-local DPP.  A read that
// needs a wider band (or a bigger traceback matrix than its LDS slice) is appended to `defer`
// before it is aligned and goes to the next kernel (G = 32, then the whole-wave kernel), which
// recomputes it from scratch, so the output is independent of the path.
// ================================================================================================
template <int G> DEV int grp_excl_max(int v, int gl);
template <> DEV int grp_excl_max<16>(int v, int gl)
{
    DPP_STEP(v, 0x111, 0xf);
    DPP_STEP(v, 0x112, 0xf);
    DPP_STEP(v, 0x114, 0xf);
    DPP_STEP(v, 0x118, 0xf);
    return __builtin_amdgcn_update_dpp(NEG_SCAN, v, 0x111, 0xf, 0xf, false);   // row_shr:1
}
template <> DEV int grp_excl_max<32>(int v, int gl)
{
    DPP_STEP(v, 0x111, 0xf);
    DPP_STEP(v, 0x112, 0xf);
    DPP_STEP(v, 0x114, 0xf);
    DPP_STEP(v, 0x118, 0xf);
    DPP_STEP(v, 0x142, 0xa);   // row_bcast:15 into rows 1 and 3: 32-lane segment scan
    const int sv = __builtin_amdgcn_update_dpp(NEG_SCAN, v, 0x138, 0xf, 0xf, false);   // wave_shr:1
    return gl == 0 ? NEG_SCAN : sv;
}
// lane gl receives v of gl-1 (gl = 0: `first`)
template <int G> DEV int grp_shr1(int v, int first, int gl)
{
    if (G == 16) return __builtin_amdgcn_update_dpp(first, v, 0x111, 0xf, 0xf, false);
    const int sv = __builtin_amdgcn_update_dpp(first, v, 0x138, 0xf, 0xf, false);
    return gl == 0 ? first : sv;
}
// lane gl receives v of gl+1 (gl = G-1: `last`)
template <int G> DEV int grp_shl1(int v, int last, int gl)
{
    if (G == 16) return __builtin_amdgcn_update_dpp(last, v, 0x101, 0xf, 0xf, false);
    const int sv = __builtin_amdgcn_update_dpp(last, v, 0x130, 0xf, 0xf, false);
    return gl == G - 1 ? last : sv;
}

// ksw_global2 (global mode) for bands of at most G columns: rows as in ksw_global2_reg; target and
// query bases staged in the group's LDS slice, read one row ahead.
template <int G>
DEV int ksw_global2_g(const Score sc, int qlen, int q_off, int q_start, int q_dir, int t_off, int tlen, int o_del,
                      int e_del, int o_ins, int e_ins, int w, int n_col, int z_off, uint64_t &cells, int gl)
{
    const int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
    int qv = gl < qlen ? g_lds_dp[q_off + q_start + q_dir * gl] : 4;
    int Hd = gl == 0 ? 0 : (gl <= w ? -(o_ins + e_ins * gl) : MINUS_INF_W);
    int E = MINUS_INF_W;
    int beg = 0, last_end = 0, width = 0, h = 0;
    int tb = tlen > 0 ? g_lds_dp[t_off] : 0;
    for (int i = 0; i < tlen; ++i) {
        const int beg_next = i + 1 > w ? i + 1 - w : 0;
        const int tb_n = i + 1 < tlen ? g_lds_dp[t_off + i + 1] : 0;
        const int jn = beg_next + G - 1;
        const int qn = (beg_next != beg && jn < qlen) ? g_lds_dp[q_off + q_start + q_dir * jn] : 4;
        const int end = i + w + 1 < qlen ? i + w + 1 : qlen;
        width = end - beg;
        const bool act = gl < width;
        const int m = Hd + sc(tb, qv);
        const int tf = m - oe_ins;
        const int ex = grp_excl_max<G>(act ? tf + gl * e_ins : NEG_SCAN, gl);
        int f = MINUS_INF_W - gl * e_ins;
        if (gl > 0) { const int fs = ex - (gl - 1) * e_ins; f = f > fs ? f : fs; }
        int d = m >= E ? 0 : 1;
        h = m >= E ? m : E;
        d = h >= f ? d : 2;
        h = h >= f ? h : f;
        const int te = m - oe_del, e2 = E - e_del;
        d |= e2 > te ? 1 << 2 : 0;
        const int enew = e2 > te ? e2 : te;
        const int f2 = f - e_ins;
        d |= f2 > tf ? 2 << 4 : 0;
        if (act) g_lds_dp[z_off + i * n_col + gl] = (uint8_t)d;
        cells += (uint64_t)width;
        last_end = end;
        if (beg_next == beg) {
            Hd = grp_shr1<G>(h, -(o_del + e_del * (i + 1)), gl);
            E = gl < width ? enew : MINUS_INF_W;
        } else {
            Hd = h;
            const int es = grp_shl1<G>(enew, MINUS_INF_W, gl);
            E = gl + 1 < width ? es : MINUS_INF_W;
            qv = grp_shl1<G>(qv, qn, gl);
        }
        beg = beg_next;
        tb = tb_n;
    }
    const int hl = __shfl(h, width > 0 ? width - 1 : 0, G);
    if (tlen > 0 && last_end == qlen) return hl;
    return qlen == 0 ? 0 : (qlen <= w ? -(o_ins + e_ins * qlen) : MINUS_INF_W);
}

// bwa_gen_cigar2 for one group; sets dfr (and aligns nothing) when the band exceeds G columns or the
// traceback matrix / target exceed the group's LDS slice
template <int G>
DEV int gen_cigar2_g(const DIndex &ix, const DOpts &o, int w_, int q_off, int t_off, int tcap, int z_off, int zcap,
                     int qb, int l_query, int64_t rb, int64_t re, int *score, uint32_t *cig, int cap, int *ncig,
                     bool &ovf, bool &dfr, uint64_t &cells, uint64_t &bases, int gl)
{
    *ncig = 0;
    if (l_query <= 0 || rb >= re || (rb < ix.l_pac && re > ix.l_pac)) return 0;
    const int64_t rlen = re - rb;
    if (re > (ix.l_pac << 1) || rb < 0) return 0;
    const bool rev = rb >= ix.l_pac;
    const int q_start = rev ? qb + l_query - 1 : qb, q_dir = rev ? -1 : 1;
    const int64_t t_start = rev ? re - 1 : rb;
    const int t_dir = rev ? -1 : 1;
    const Score sc = score_of(o);
    if (l_query == rlen) {
        int sum = 0;
        for (int i = gl; i < l_query; i += G)
            sum += sc(ref_at(ix, t_start + (int64_t)t_dir * i), g_lds_dp[q_off + q_start + q_dir * i]);
        sum = grp_sum<G>(sum);
        if (w_ == 0 || diagonal_wins(o, l_query, sum) ||
            detour_free<G>(o, sc, l_query, sum, [&](int j, int &t, int &q) {
                t = ref_at(ix, t_start + (int64_t)t_dir * j);
                q = g_lds_dp[q_off + q_start + q_dir * j];
            }, gl)) {
            if (cap < 1) { ovf = true; return 0; }
            bases += (uint64_t)((rlen + 3) >> 2);
            cig[0] = (uint32_t)l_query << 4;
            *ncig = 1;
            *score = sum;
            return 1;
        }
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
    const int n_col = l_query < 2 * w + 1 ? l_query : 2 * w + 1;
    if (n_col > G || rlen >= (int64_t)l_query + w || rlen > tcap || (int64_t)n_col * rlen > zcap) {
        dfr = true;
        return 0;
    }
    bases += (uint64_t)((rlen + 3) >> 2);
    for (int i = gl; i < (int)rlen; i += G) g_lds_dp[t_off + i] = (uint8_t)ref_at(ix, t_start + (int64_t)t_dir * i);
    lds_fence();
    *score = ksw_global2_g<G>(sc, l_query, q_off, q_start, q_dir, t_off, (int)rlen, o.o_del, o.e_del, o.o_ins,
                              o.e_ins, w, n_col, z_off, cells, gl);
    traceback_w<true, G>(l_query, (int)rlen, w, n_col, z_off, nullptr, cig, cap, ncig, ovf, gl, lane_id() & ~(G - 1));
    return 1;
}

template <int G>
__global__ void __launch_bounds__(256) k_reg2aln_g(DIndex ix, DOpts o, Caps cp, const uint8_t *__restrict__ codes,
                                                   const int64_t *__restrict__ offs, int n,
                                                   const int32_t *__restrict__ list, const int32_t *__restrict__ list_n,
                                                   const Reg *__restrict__ regs, const int32_t *__restrict__ n_regs,
                                                   Hit *__restrict__ hits, uint32_t *__restrict__ cigars,
                                                   int32_t *__restrict__ n_cig_read, uint32_t *__restrict__ status,
                                                   int32_t *__restrict__ defer, int32_t *__restrict__ defer_n,
                                                   Counters *ctr, int per_wave)
{
    constexpr int NG = 64 / G;
    const int l = lane_id(), gl = l & (G - 1), grp = l / G;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int slice = (per_wave / NG) & ~15;
    const int q_off = wave * per_wave + grp * slice;
    const int qcap = (cp.max_len + 16) & ~15, tcap = (cp.max_len + 64 + 15) & ~15;
    const int t_off = q_off + qcap, z_off = t_off + tcap;
    const int zcap = slice - qcap - tcap;
    const int n_items = list ? *list_n : n;
    const int gw = blockIdx.x * (blockDim.x >> 6) + wave, nw = gridDim.x * (blockDim.x >> 6);
    uint64_t cells = 0, bases = 0;
    for (int b = gw; b * NG < n_items; b += nw) {
        const int k = b * NG + grp;
        const int li = k < n_items ? (list ? list[k] : k) : -1;
        if (li < 0) continue;
        if (status[li]) { n_cig_read[li] = 0; continue; }
        const uint8_t *q = codes + offs[li];
        const int l_query = (int)(offs[li + 1] - offs[li]);
        const int nr = n_regs[li];
        for (int j = gl; j < l_query; j += G) g_lds_dp[q_off + j] = q[j];
        lds_fence();
        bool ovf = false, dfr = false;
        int tot = 0;
        for (int g = 0; g < nr && !ovf && !dfr; ++g) {
            const Reg &ar = regs[(size_t)li * cp.regs + g];
            uint32_t *cig = cigars + ((size_t)li * cp.regs + g) * cp.cigar;
            const int qb = ar.qb, qe = ar.qe, truesc = ar.truesc;
            const int64_t rb = ar.rb, re = ar.re;
            const int flag = ar.secondary >= 0 ? 0x100 : 0;
            int tmp = infer_bw(qe - qb, (int)(re - rb), truesc, o.a, o.o_del, o.e_del);
            int w2 = infer_bw(qe - qb, (int)(re - rb), truesc, o.a, o.o_ins, o.e_ins);
            w2 = w2 > tmp ? w2 : tmp;
            if (w2 > o.w) w2 = w2 < ar.w ? w2 : ar.w;
            int i = 0, score = 0, last_sc = -(1 << 30), ncig = 0;
            do {
                w2 = w2 < o.w << 2 ? w2 : o.w << 2;
                gen_cigar2_g<G>(ix, o, w2, q_off, t_off, tcap, z_off, zcap, qb, qe - qb, rb, re, &score, cig,
                                cp.cigar - 2, &ncig, ovf, dfr, cells, bases, gl);
                if (ovf || dfr) break;
                if (score == last_sc || w2 == o.w << 2) break;
                last_sc = score;
                w2 <<= 1;
            } while (++i < 3 && score < truesc - o.a);
            if (ovf || dfr) break;
            int is_rev;
            (void)depos(ix, rb < ix.l_pac ? rb : re - 1, is_rev);
            if (ncig > 0) {
                if ((cig[0] & 0xf) == 2) {
                    --ncig;
                    for (int t = 0; t < ncig; ++t) cig[t] = cig[t + 1];
                } else if ((cig[ncig - 1] & 0xf) == 2) --ncig;
            }
            if (qb != 0 || qe != l_query) {
                const int clip5 = is_rev ? l_query - qe : qb, clip3 = is_rev ? qb : l_query - qe;
                if (clip5) {
                    for (int t = ncig; t > 0; --t) cig[t] = cig[t - 1];
                    cig[0] = (uint32_t)clip5 << 4 | 3;
                    ++ncig;
                }
                if (clip3) cig[ncig++] = (uint32_t)clip3 << 4 | 3;
            }
            Hit hh;
            hh.rb = rb; hh.re = re; hh.qb = qb; hh.qe = qe; hh.rid = ar.rid; hh.score = ar.score; hh.flag = flag;
            hh.is_rev = is_rev; hh.n_cigar = ncig; hh.pad = 0;
            hits[(size_t)li * cp.regs + g] = hh;
            tot += ncig;
        }
        if (dfr) {
            if (gl == 0) defer[atomicAdd(defer_n, 1)] = li;
        } else if (ovf) {
            if (gl == 0) status[li] |= ST_OVERFLOW;
            n_cig_read[li] = 0;
        } else n_cig_read[li] = tot;
    }
    if (gl != 0) { cells = 0; bases = 0; }   // group-uniform control: count once per group
    wave_add(&ctr[STG_REG2ALN].dp_cells, cells);
    wave_add(&ctr[STG_REG2ALN].ref_bases, bases);
}

template <int G>
static hipError_t launch_g(hipStream_t st, const DIndex &ix, const DOpts &o, const Caps &cp, const uint8_t *codes,
                           const int64_t *offs, int n, const int32_t *list, const int32_t *list_n, const Reg *regs,
                           const int32_t *n_regs, Hit *hits, uint32_t *cigars, int32_t *n_cig, uint32_t *status,
                           int32_t *defer, int32_t *defer_n, Counters *ctr, int zcap, int max_blocks)
{
    const int waves = 4;
    int grid = (n + waves * (64 / G) - 1) / (waves * (64 / G));
    if (grid > max_blocks) grid = max_blocks;
    if (grid == 0) return hipSuccess;
    const size_t eh_bytes = ((size_t)(cp.max_len + 2) * sizeof(int2) + 15) & ~(size_t)15;
    const size_t q_bytes = ((size_t)cp.max_len + 16) & ~(size_t)15;
    const size_t per_wave = eh_bytes + (size_t)zcap + q_bytes;
    hipLaunchKernelGGL(k_reg2aln_g<G>, dim3(grid), dim3(64 * waves), waves * per_wave, st, ix, o, cp, codes, offs, n,
                       list, list_n, regs, n_regs, hits, cigars, n_cig, status, defer, defer_n, ctr, (int)per_wave);
    return hipGetLastError();
}

// ================================================================================================
// Diagonal pass: one lane per read.  Most regions of 150-bp reads are gapless with a few mismatches, and
// bwa_gen_cigar2 returns "nM" for them without a DP (w == 0, diagonal_wins, or the exact detour test).  This
// kernel decides that per region sequentially in one lane (no LDS, every lane busy) and writes the read's
// records when every region of it is decided; a read with any region that needs the DP is appended (in
// input order, wave-aggregated) to `defer`, and the group kernel recomputes the whole read from scratch, so
// the output does not depend on which kernel produced it.  The per-region control is k_reg2aln_g's.
// ================================================================================================

// gen_cigar2_g's diagonal shortcut for one region, sequential: the diagonal score S of the n x n problem and
// whether w == 0, diagonal_wins(S) or detour_free(S) holds (detour_free's prefix sums / minima carried in a
// single pass: C1/Cm the sums of delta before j, m1/mm their running minima including C[0] = 0).
// Sequential reader of the query bases codes[a], codes[a + step], ... (step +-1) within [lo, hi]: 16-B aligned
// words of the batch's code buffer, the next one loaded while the current one is consumed (a byte load per base
// would wait on memory every step of the loop).
struct QStream {
    const uint8_t *codes;
    int64_t a, wlo, whi, cur_w;
    int step;
    uint4 cur, nxt;
    DEV uint4 load(int64_t w) const
    {
        return (w >= wlo && w <= whi) ? *reinterpret_cast<const uint4 *>(codes + 16 * w) : make_uint4(0u, 0u, 0u, 0u);
    }
    DEV void init(const uint8_t *c, int64_t start, int dir, int64_t lo, int64_t hi)
    {
        codes = c; a = start; step = dir; wlo = lo >> 4; whi = hi >> 4;
        cur_w = a >> 4;
        cur = load(cur_w);
        nxt = load(cur_w + step);
    }
    DEV int next()
    {
        const int64_t w = a >> 4;
        if (w != cur_w) { cur = w == cur_w + step ? nxt : load(w); cur_w = w; nxt = load(w + step); }
        const int k = (int)(a & 15);
        const uint32_t v = (k & 8) ? ((k & 4) ? cur.w : cur.z) : ((k & 4) ? cur.y : cur.x);
        a += step;
        return (int)((v >> ((k & 3) << 3)) & 0xffu);
    }
};

DEV bool diag_decides(const DIndex &ix, const DOpts &o, const Score sc, int w_, const uint8_t *codes, int64_t rd,
                      int l_read, int q_start, int q_dir, int64_t t_start, int t_dir, int n, int &S)
{
    TStream ts;
    ts.init(ix, t_start, t_dir);
    QStream qs;
    qs.init(codes, rd + q_start, q_dir, rd, rd + l_read - 1);
    int tj = ts.next(), qj = qs.next();
    int sum = 0, c1 = 0, cm = 0, m1 = 0, mm = 0, x = -0x3fffffff;
    for (int j = 0; j < n; ++j) {
        const bool nx = j + 1 < n;
        const int tn = nx ? ts.next() : 0, qn = nx ? qs.next() : 0;
        const int s0 = sc(tj, qj);
        sum += s0;
        m1 = m1 < c1 ? m1 : c1;
        mm = mm < cm ? mm : cm;
        const int a1 = c1 - m1 - s0, am = cm - mm - s0;
        x = x > a1 ? x : a1;
        x = x > am ? x : am;
        if (nx) { c1 += sc(tj, qn) - s0; cm += sc(tn, qj) - s0; }
        tj = tn; qj = qn;
    }
    S = sum;
    if (w_ == 0 || diagonal_wins(o, n, sum)) return true;
    const int64_t bound2 = (int64_t)(n - 2) * o.mat_max - (o.o_ins + o.o_del + 2 * (o.e_ins + o.e_del));
    return (int64_t)sum > bound2 && (int64_t)x < (int64_t)(o.o_ins + o.e_ins + o.o_del + o.e_del);
}

// mem_reg2aln's first band of a region: class 1 (<= 16 columns), 2 (<= 32) or 3 (wider)
DEV int band_class(const DOpts &o, int lq, int64_t rl, int w2)
{
    if (lq <= 0 || rl <= 0 || rl > (1 << 30)) return 1;   // gen_cigar2's early exits: no DP in any kernel
    int mg = idiv_plus(((lq + 1) >> 1) * o.mat_match - o.o_ins, o.e_ins, 1);
    int md = idiv_plus(((lq + 1) >> 1) * o.mat_match - o.o_del, o.e_del, 1);
    mg = mg > md ? mg : md; mg = mg > 1 ? mg : 1;
    int dl = (int)rl - lq; dl = dl < 0 ? -dl : dl;
    int ww = (mg + dl + 1) >> 1; ww = ww < w2 ? ww : w2; ww = ww > dl + 3 ? ww : dl + 3;
    const int nc = lq < 2 * ww + 1 ? lq : 2 * ww + 1;
    return nc <= 16 ? 1 : nc <= 32 ? 2 : 3;
}

// appends li (when `on`) to list/count in lane order: one atomic per wave
DEV void wave_append(bool on, int li, int32_t *list, int32_t *count)
{
    const uint64_t m = __ballot(on);
    int base = 0;
    if ((threadIdx.x & 63) == 0 && m) base = atomicAdd(count, __popcll(m));
    base = __shfl(base, 0, 64);
    if (on) list[base + __popcll(m & ((1ull << (threadIdx.x & 63)) - 1))] = li;
}

// Reads with a region the pass does not decide go straight to the kernel of their widest first band: <= 16 columns
// to `defer` (k_reg2aln_g<16>'s input), <= 32 to d0 (k_reg2aln_g<32>'s), wider to d1 (k_reg2aln_w's) -- each kernel
// recomputes a read from scratch and still defers what outgrows it.
__global__ void __launch_bounds__(256) k_reg2aln_diag(DIndex ix, DOpts o, Caps cp, const uint8_t *__restrict__ codes,
                                                      const int64_t *__restrict__ offs, int n,
                                                      const int32_t *__restrict__ list, const int32_t *__restrict__ list_n,
                                                      const Reg *__restrict__ regs, const int32_t *__restrict__ n_regs,
                                                      Hit *__restrict__ hits, uint32_t *__restrict__ cigars,
                                                      int32_t *__restrict__ n_cig_read, const uint32_t *__restrict__ status,
                                                      int32_t *__restrict__ defer, int32_t *__restrict__ defer_n,
                                                      int32_t *__restrict__ d0, int32_t *__restrict__ d1,
                                                      int32_t *__restrict__ dn, Counters *ctr)
{
    const int n_items = list ? *list_n : n;
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    const int li = k < n_items ? (list ? list[k] : k) : -1;
    int cls = 0;   // widest first-band class among the regions the pass leaves to the DP kernels
    uint64_t bases = 0;
    if (li >= 0) {
        if (status[li]) n_cig_read[li] = 0;
        else {
            const int64_t rd = offs[li];
            const int l_read = (int)(offs[li + 1] - rd);
            const int nr = n_regs[li];
            const Score sc = score_of(o);
            int tot = 0;
            bool dfr = cp.cigar < 3;   // "nM" plus two clips; smaller CIGAR slots take the group kernel's overflow path
            if (dfr) cls = 1;
            for (int g = 0; g < nr; ++g) {
                const Reg &ar = regs[(size_t)li * cp.regs + g];
                const int qb = ar.qb, qe = ar.qe, lq = qe - qb;
                const int64_t rb = ar.rb, re = ar.re, rlen = re - rb;
                int tmp = infer_bw(lq, (int)rlen, ar.truesc, o.a, o.o_del, o.e_del);
                int w2 = infer_bw(lq, (int)rlen, ar.truesc, o.a, o.o_ins, o.e_ins);
                w2 = w2 > tmp ? w2 : tmp;
                if (w2 > o.w) w2 = w2 < ar.w ? w2 : ar.w;
                w2 = w2 < o.w << 2 ? w2 : o.w << 2;
                if (dfr) {   // a region already left to the DP kernels: only the class of the rest matters
                    const int c = band_class(o, lq, rlen, w2);
                    cls = cls > c ? cls : c;
                    continue;
                }
                // gen_cigar2_g's early exits and the DP case belong to the group kernels
                const bool odd = lq <= 0 || rb >= re || (rb < ix.l_pac && re > ix.l_pac) || re > (ix.l_pac << 1) || rb < 0;
                const bool rev = rb >= ix.l_pac;
                int S = 0;
                if (odd || rlen != lq ||
                    !diag_decides(ix, o, sc, w2, codes, rd, l_read, rev ? qb + lq - 1 : qb, rev ? -1 : 1,
                                  rev ? re - 1 : rb, rev ? -1 : 1, lq, S)) {
                    dfr = true;
                    const int c = odd ? 1 : band_class(o, lq, rlen, w2);
                    cls = cls > c ? cls : c;
                    continue;
                }
                // the retry loop of k_reg2aln_g: a second call (doubled band) when the first band was not the
                // widest and S < truesc - a; it decides the same way (the shortcut does not depend on w > 0)
                bases += (uint64_t)((rlen + 3) >> 2);
                if (w2 != o.w << 2 && S < ar.truesc - o.a) bases += (uint64_t)((rlen + 3) >> 2);
                uint32_t *cig = cigars + ((size_t)li * cp.regs + g) * cp.cigar;
                int is_rev;
                (void)depos(ix, rb < ix.l_pac ? rb : re - 1, is_rev);
                int ncig = 0;
                const int clip5 = is_rev ? l_read - qe : qb, clip3 = is_rev ? qb : l_read - qe;
                if (clip5) cig[ncig++] = (uint32_t)clip5 << 4 | 3;
                cig[ncig++] = (uint32_t)lq << 4;
                if (clip3) cig[ncig++] = (uint32_t)clip3 << 4 | 3;
                Hit hh;
                hh.rb = rb; hh.re = re; hh.qb = qb; hh.qe = qe; hh.rid = ar.rid; hh.score = ar.score;
                hh.flag = ar.secondary >= 0 ? 0x100 : 0;
                hh.is_rev = is_rev; hh.n_cigar = ncig; hh.pad = 0;
                hits[(size_t)li * cp.regs + g] = hh;
                tot += ncig;
            }
            if (!dfr) n_cig_read[li] = tot;
        }
    }
    // the lists keep their input order within each (one atomic per wave and list)
    wave_append(cls == 1, li, defer, defer_n);
    wave_append(cls == 2, li, d0, dn);
    wave_append(cls >= 3, li, d1, dn + 1);
    wave_add(&ctr[STG_REG2ALN].ref_bases, bases);
}

// BSQ_R2A_STATIC=1: the whole-wave kernel takes its reads by a fixed stride (A/B measurements)
static bool r2a_static() { static const bool v = [] { const char *e = getenv("BSQ_R2A_STATIC"); return e && *e == '1'; }(); return v; }

// group kernels G = 16 then 32 over the reads (in `order` when given), the whole-wave kernel over what remains
// dn: 5 counters -- [0], [1] the group kernels' defer lists, [3] the diagonal pass's ([2] is order_n's home), [4] the
// whole-wave kernel's work counter;
// pre: n entries for the diagonal pass's list (nullptr: no diagonal pass)
hipError_t launch_reg2aln_chain(hipStream_t st, const DIndex &ix, const DOpts &o, const Caps &cp, const uint8_t *codes,
                                const int64_t *offs, int n, const Reg *regs, const int32_t *n_regs, Hit *hits,
                                uint32_t *cigars, int32_t *n_cig, uint32_t *status, Counters *ctr, int zcap,
                                uint8_t *zslab, int64_t zslab_bytes, int max_blocks, int32_t *d0, int32_t *d1,
                                int32_t *dn, const int32_t *order, const int32_t *order_n, int32_t *pre)
{
    hipError_t e = hipMemsetAsync(dn, 0, 2 * sizeof(int32_t), st);
    if (e != hipSuccess) return e;
    if (pre && n > 0) {
        e = hipMemsetAsync(dn + 3, 0, sizeof(int32_t), st);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_reg2aln_diag, dim3((n + 255) / 256), dim3(256), 0, st, ix, o, cp, codes, offs, n, order,
                           order_n, regs, n_regs, hits, cigars, n_cig, status, pre, dn + 3, d0, d1, dn, ctr);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
        order = pre;
        order_n = dn + 3;
    }
    e = launch_g<16>(st, ix, o, cp, codes, offs, n, order, order_n, regs, n_regs, hits, cigars, n_cig, status, d0,
                     dn, ctr, zcap, max_blocks);
    if (e != hipSuccess) return e;
    e = launch_g<32>(st, ix, o, cp, codes, offs, n, d0, dn, regs, n_regs, hits, cigars, n_cig, status, d1, dn + 1, ctr,
                     zcap, max_blocks);
    if (e != hipSuccess) return e;
    return launch_reg2aln_w(st, ix, o, cp, codes, offs, n, regs, n_regs, hits, cigars, n_cig, status, ctr, zcap, zslab,
                            zslab_bytes, max_blocks, d1, dn + 1, r2a_static() ? nullptr : dn + 4);
}

}  // namespace bsq
