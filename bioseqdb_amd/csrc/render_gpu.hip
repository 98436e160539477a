// render_gpu.hip -- bwa_result rows rendered on the GPU (host materialisation).
//
// The same bytes as bsq_render_tsv (render.cpp; reference: BwaIndex::align_sequence's BwaMatch fields,
// bioseqdb/bwa.cpp:159-175, extract_reference_subseq :55-68, cigar_compressed_to_string :70-77):
// one thread per row, in two passes -- the exact length of every row, an exclusive scan for the row
// offsets, then the text itself -- so the host receives one finished buffer.  ref_subseq comes from
// the pac in HBM with the reference's hole overlay (Q3: row-relative offsets on the concatenated axis,
// later holes win; Q7: reverse-strand rows as reverse-strand text), query_subseq from the read's codes
// with its own hole symbols.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/bsq.h"
#include "bsq_device.h"

namespace bsq {

#define DEV __device__ __forceinline__

struct RenderHole { int64_t beg, end; uint32_t order; uint32_t amb; };   // reference holes, by beg

struct RenderView {
    const bsq_hit *hits;
    const uint32_t *cigar;
    int64_t n_hits;
    const uint8_t *pac;
    int64_t l_pac;
    const RenderHole *holes;   // the reference's hole overlay: disjoint segments ordered by offset
    int64_t n_holes;
    const uint8_t *codes;      // read codes (nt4) of the batch, read r at offs[r]
    const int64_t *offs;
    const int64_t *rh_off;     // read r's holes: [rh_off[r], rh_off[r+1]) of rh (nullptr: none)
    const RenderHole *rh;      // read holes (beg/end relative to the read, order = hole index)
};

DEV int ndig(int64_t v)
{
    uint64_t u = v < 0 ? (uint64_t)(-(v + 1)) + 1 : (uint64_t)v;
    int n = 1;
    while (u >= 10) { u /= 10; ++n; }
    return n + (v < 0);
}

DEV char *put_int(char *o, int64_t v)
{
    const int n = ndig(v);
    uint64_t u = v < 0 ? (uint64_t)(-(v + 1)) + 1 : (uint64_t)v;
    char *e = o + n;
    char *p = e;
    do { *--p = (char)('0' + u % 10); u /= 10; } while (u);
    if (v < 0) *--p = '-';
    return e;
}

DEV int64_t row_len(const RenderView &v, const bsq_hit &x)
{
    int64_t n = ndig(x.ref_id) + 1 + (x.re - x.rb) + 1 + ndig(x.ref_match_start) + 1 + ndig(x.ref_match_end) + 1 +
                ndig(x.ref_match_len) + 1 + (x.qe - x.qb) + 1 + ndig(x.qb) + 1 + ndig(x.qe) + 1 + ndig(x.qe - x.qb) + 1 +
                6 + 1 + ndig(x.score) + 1;
    for (uint32_t c = 0; c < x.n_cigar; ++c) n += ndig(v.cigar[x.cigar_off + c] >> 4) + 1;
    return n;
}

__global__ void k_row_len(RenderView v, int64_t *len)
{
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < v.n_hits; k += (int64_t)gridDim.x * blockDim.x)
        len[k] = row_len(v, v.hits[k]);
}

DEV int pac_base(const uint8_t *pac, int64_t i) { return (pac[i >> 2] >> ((~i & 3) << 1)) & 3; }

// ref_subseq of one row at o; returns the end
DEV char *ref_subseq(const RenderView &v, const bsq_hit &x, char *o)
{
    char *s = o;
    const int64_t rb = x.rb, re = x.re;
    if (rb < v.l_pac) {
        for (int64_t i = rb; i < re; ++i) *o++ = "ACGT"[pac_base(v.pac, i)];
        // the hole overlay as disjoint segments (HoleIndex): the first one ending after rb, then in order
        int64_t lo = 0, hi = v.n_holes;
        while (lo < hi) { const int64_t mid = (lo + hi) >> 1; if (v.holes[mid].end <= rb) lo = mid + 1; else hi = mid; }
        for (int64_t h = lo; h < v.n_holes && v.holes[h].beg < re; ++h) {
            const RenderHole &H = v.holes[h];
            const int64_t a = H.beg > rb ? H.beg : rb, b = H.end < re ? H.end : re;
            for (int64_t i = a; i < b; ++i) s[i - rb] = (char)H.amb;
        }
    } else {   // Q7: the reverse-strand reference text
        for (int64_t i = rb; i < re; ++i) *o++ = "ACGT"[3 - pac_base(v.pac, (v.l_pac << 1) - 1 - i)];
    }
    return o;
}

// query_subseq of one row at o: the read's text (ns_to_text) over [qb, qe); returns the end
DEV char *query_subseq(const RenderView &v, const bsq_hit &x, char *o)
{
    const uint8_t *q = v.codes + v.offs[x.read_index];
    char *s = o;
    for (int j = x.qb; j < x.qe; ++j) { const int c = q[j]; *o++ = c < 4 ? "ACGT"[c] : 'N'; }
    if (v.rh_off) {
        const int64_t h0 = v.rh_off[x.read_index], h1 = v.rh_off[x.read_index + 1];
        for (int64_t h = h0; h < h1; ++h) {   // in the nuclseq's order: later holes win
            const RenderHole &H = v.rh[h];
            const int64_t a = H.beg > x.qb ? H.beg : x.qb, b = H.end < x.qe ? H.end : x.qe;
            for (int64_t i = a; i < b; ++i) s[i - x.qb] = (char)H.amb;
        }
    }
    return o;
}

__global__ void k_row_write(RenderView v, const int64_t *off, char *out)
{
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < v.n_hits; k += (int64_t)gridDim.x * blockDim.x) {
        const bsq_hit x = v.hits[k];
        char *o = out + off[k];
        o = put_int(o, x.ref_id); *o++ = '\t';
        o = ref_subseq(v, x, o);
        *o++ = '\t';
        o = put_int(o, x.ref_match_start); *o++ = '\t';
        o = put_int(o, x.ref_match_end); *o++ = '\t';
        o = put_int(o, x.ref_match_len); *o++ = '\t';
        o = query_subseq(v, x, o);
        *o++ = '\t';
        o = put_int(o, x.qb); *o++ = '\t';
        o = put_int(o, x.qe); *o++ = '\t';
        o = put_int(o, x.qe - x.qb); *o++ = '\t';
        *o++ = x.is_primary ? 't' : 'f'; *o++ = '\t';
        *o++ = x.is_secondary ? 't' : 'f'; *o++ = '\t';
        *o++ = x.is_reverse ? 't' : 'f'; *o++ = '\t';
        for (uint32_t c = 0; c < x.n_cigar; ++c) {
            const uint32_t op = v.cigar[x.cigar_off + c];
            o = put_int(o, op >> 4);
            *o++ = "MIDNSHP=XB"[op & 0xf];
        }
        *o++ = '\t';
        o = put_int(o, x.score);
        *o++ = '\n';
    }
}

// ---- build_tuple_bwa's nuclseq columns without the text round trip --------------------------------------------
// nuclseq_from_text of a text without holes (sequence.cpp:209-245) is {VARSIZE << 2, 0, len} then the pac bytes,
// whose bases past `len` (up to the byte boundary) are the first draws of std::minstd_rand(0 ^ len).  A row's
// ref_subseq has none when no reference hole overlaps [rb, re) (or the row is reverse-strand, Q7: pure text); its
// query_subseq has none when none of the read's holes overlaps [qb, qe).  Those texts are written straight from the
// reference pac / the read codes, 16 bases (one 4-byte word) at a time; the rest go through the generic path.

// text t = 2k (ref_subseq of row k) or 2k + 1 (query_subseq): 1 if it contains a hole
DEV bool col_holed(const RenderView &v, const bsq_hit &x, int which)
{
    if (which == 0) {
        if (x.rb >= v.l_pac) return false;   // Q7 reverse-strand text: no overlay
        int64_t lo = 0, hi = v.n_holes;
        while (lo < hi) { const int64_t mid = (lo + hi) >> 1; if (v.holes[mid].end <= x.rb) lo = mid + 1; else hi = mid; }
        return lo < v.n_holes && v.holes[lo].beg < x.re;
    }
    if (v.rh_off) {   // hole bases decode to code 4, so the read's hole list decides
        for (int64_t h = v.rh_off[x.read_index]; h < v.rh_off[x.read_index + 1]; ++h)
            if (v.rh[h].beg < x.qe && v.rh[h].end > x.qb) return true;
        return false;
    }
    const uint8_t *q = v.codes + v.offs[x.read_index];   // no hole list (codes given directly): code 4 prints N
    for (int j = x.qb; j < x.qe; ++j)
        if (q[j] > 3) return true;
    return false;
}

// size[t] = the 8-aligned varlena size of a hole-free text (0 for a holed one); holed[t] = 1 for a holed text;
// both with a 0 at [n] (exclusive scans of n + 1 entries)
__global__ void k_col_class(RenderView v, int64_t *size, int64_t *holed)
{
    const int64_t n = 2 * v.n_hits;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t <= n; t += (int64_t)gridDim.x * blockDim.x) {
        if (t == n) { size[t] = 0; holed[t] = 0; continue; }
        const bsq_hit x = v.hits[t >> 1];
        const int which = (int)(t & 1);
        const bool h = col_holed(v, x, which);
        const int64_t len = which ? (int64_t)x.qe - x.qb : x.re - x.rb;
        size[t] = h ? 0 : (12 + ((len + 3) >> 2) + 7) & ~(int64_t)7;
        holed[t] = h ? 1 : 0;
    }
}

// the holed texts as a list (hl[j] = text id, in order) with their text and pac lengths (+ a 0 at [nh])
__global__ void k_col_compact(RenderView v, const int64_t *hpos, int64_t *hl, int64_t *tl, int64_t *pl)
{
    const int64_t n = 2 * v.n_hits;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = hpos[t];
        if (hpos[t + 1] == j) continue;
        const bsq_hit x = v.hits[t >> 1];
        const int64_t len = (t & 1) ? (int64_t)x.qe - x.qb : x.re - x.rb;
        hl[j] = t; tl[j] = len; pl[j] = (len + 3) >> 2;
        if (j + 1 == hpos[n]) { tl[j + 1] = 0; pl[j + 1] = 0; }
    }
}

// the texts of the holed list at toff[j] (the generic encoder's input)
__global__ void k_sub_write_sel(RenderView v, const int64_t *hl, int64_t nh, const int64_t *toff, char *out)
{
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nh; j += (int64_t)gridDim.x * blockDim.x) {
        const int64_t t = hl[j];
        const bsq_hit x = v.hits[t >> 1];
        if (t & 1) query_subseq(v, x, out + toff[j]);
        else ref_subseq(v, x, out + toff[j]);
    }
}

// a holed text's varlena size is the generic encoder's (its output offsets are 8-aligned)
__global__ void k_col_holed_size(const int64_t *hl, int64_t nh, const int64_t *enc_off, int64_t *size)
{
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nh; j += (int64_t)gridDim.x * blockDim.x)
        size[hl[j]] = enc_off[j + 1] - enc_off[j];
}

__global__ void k_col_copy_holed(const int64_t *hl, int64_t nh, const int64_t *enc_off, const uint8_t *enc,
                                 const int64_t *off, uint8_t *out)
{
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < nh; j += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t *src = reinterpret_cast<const uint64_t *>(enc + enc_off[j]);
        uint64_t *dst = reinterpret_cast<uint64_t *>(out + off[hl[j]]);
        for (int64_t w = 0; w < (enc_off[j + 1] - enc_off[j]) >> 3; ++w) dst[w] = src[w];
    }
}

DEV uint64_t be64_at(const uint8_t *pac, int64_t q) { return __builtin_bswap64(reinterpret_cast<const uint64_t *>(pac)[q]); }

// forward bases f .. f+15 of the pac as one big-endian 32-bit word (base f in the top two bits); f may be negative
// (those fields are 0).  The device pac carries 16 bytes of padding, so the second 8-byte word is always mapped.
DEV uint32_t fwd16(const uint8_t *pac, int64_t f)
{
    int sh = 0;
    if (f < 0) { sh = (int)(-f); f = 0; }
    if (sh >= 16) return 0;
    const int64_t b = 2 * f;
    const int r = (int)(b & 63);
    uint64_t x = be64_at(pac, b >> 6) << r;
    if (r > 32) x |= be64_at(pac, (b >> 6) + 1) >> (64 - r);
    return (uint32_t)(x >> 32) >> (2 * sh);
}

// 16 2-bit fields in reverse order
DEV uint32_t rev2(uint32_t x)
{
    x = ((x >> 2) & 0x33333333u) | ((x & 0x33333333u) << 2);
    x = ((x >> 4) & 0x0F0F0F0Fu) | ((x & 0x0F0F0F0Fu) << 4);
    return __builtin_bswap32(x);
}

// query codes j .. j+15 of a read (all < 4) as one big-endian 32-bit word; the code buffer is padded past its end
DEV uint32_t codes16(const uint8_t *q, int64_t j)
{
    uint32_t w = 0;
    for (int k = 0; k < 4; ++k) {
        const uint8_t *p = q + j + 4 * k;
        const uintptr_t a = reinterpret_cast<uintptr_t>(p);
        const uint32_t *al = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
        const uint64_t two = (uint64_t)al[0] | ((uint64_t)al[1] << 32);
        const uint32_t c = (uint32_t)(two >> ((a & 3) * 8));   // codes j+4k .. j+4k+3, first in the low byte
        const uint32_t byte = ((c & 3) << 6) | (((c >> 8) & 3) << 4) | (((c >> 16) & 3) << 2) | ((c >> 24) & 3);
        w |= byte << (24 - 8 * k);
    }
    return w;
}

// the varlenas of the hole-free texts at off[t] (hpos: the exclusive scan of the holed flags)
__global__ void k_col_direct(RenderView v, const int64_t *off, const int64_t *hpos, uint8_t *out)
{
    const int64_t n = 2 * v.n_hits;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
        if (hpos[t + 1] != hpos[t]) continue;   // a holed text: copied from the generic encoder's output
        const bsq_hit x = v.hits[t >> 1];
        const bool qry = t & 1;
        const int64_t len = qry ? (int64_t)x.qe - x.qb : x.re - x.rb;
        const int64_t pb = (len + 3) >> 2, size = 12 + pb;
        uint32_t *o = reinterpret_cast<uint32_t *>(out + off[t]);
        o[0] = (uint32_t)(size << 2);
        o[1] = 0;
        o[2] = (uint32_t)len;
        // padding bases len .. 4 pb - 1: the first draws of minstd_rand(len) (2 bits each)
        uint32_t pad = 0;
        {
            uint64_t st = (uint64_t)len % 2147483647ull;
            if (!st) st = 1;
            for (int64_t i = len; i < 4 * pb; ++i) {
                st = st * 48271ull % 2147483647ull;
                pad |= (uint32_t)(st & 3) << (2 * (15 - (i & 15)));
            }
        }
        const int64_t words = (pb + 3) >> 2;
        const uint8_t *q = v.codes + v.offs[x.read_index] + x.qb;
        const bool fwd = x.rb < v.l_pac;
        const int64_t p0 = 2 * v.l_pac - 1 - x.rb;   // reverse strand: text base i is the complement of fwd p0 - i
        for (int64_t c = 0; c < words; ++c) {
            uint32_t w;
            if (qry) w = codes16(q, 16 * c);
            else if (fwd) w = fwd16(v.pac, x.rb + 16 * c);
            else w = ~rev2(fwd16(v.pac, p0 - 16 * c - 15));
            const int64_t rem = len - 16 * c;   // text bases in this word
            if (rem < 16) w = (rem > 0 ? (w & ~(0xFFFFFFFFu >> (2 * rem))) : 0u) | pad;
            o[3 + c] = __builtin_bswap32(w);   // pac bytes in order (first base in the top bits of byte 0)
        }
        for (int64_t k = 12 + 4 * words; k < ((size + 7) & ~(int64_t)7); k += 4) o[k >> 2] = 0;   // alignment tail
    }
}

inline dim3 rgrid(int64_t n) { const int64_t b = (n + 255) / 256; return dim3((unsigned)(b < 65536 ? (b ? b : 1) : 65536)); }

hipError_t launch_row_len(hipStream_t st, const RenderView &v, int64_t *len)
{
    hipLaunchKernelGGL(k_row_len, rgrid(v.n_hits), dim3(256), 0, st, v, len);
    return hipGetLastError();
}

hipError_t launch_row_write(hipStream_t st, const RenderView &v, const int64_t *off, char *out)
{
    hipLaunchKernelGGL(k_row_write, rgrid(v.n_hits), dim3(256), 0, st, v, off, out);
    return hipGetLastError();
}

hipError_t launch_col_class(hipStream_t st, const RenderView &v, int64_t *size, int64_t *holed)
{
    hipLaunchKernelGGL(k_col_class, rgrid(2 * v.n_hits + 1), dim3(256), 0, st, v, size, holed);
    return hipGetLastError();
}

hipError_t launch_col_holed(hipStream_t st, const RenderView &v, const int64_t *hpos, int64_t nh, int64_t *hl,
                            int64_t *tl, int64_t *pl)
{
    hipLaunchKernelGGL(k_col_compact, rgrid(2 * v.n_hits), dim3(256), 0, st, v, hpos, hl, tl, pl);
    return hipGetLastError();
}

hipError_t launch_sub_write_sel(hipStream_t st, const RenderView &v, const int64_t *hl, int64_t nh, const int64_t *toff,
                                char *out)
{
    hipLaunchKernelGGL(k_sub_write_sel, rgrid(nh), dim3(256), 0, st, v, hl, nh, toff, out);
    return hipGetLastError();
}

hipError_t launch_col_holed_size(hipStream_t st, const int64_t *hl, int64_t nh, const int64_t *enc_off, int64_t *size)
{
    hipLaunchKernelGGL(k_col_holed_size, rgrid(nh), dim3(256), 0, st, hl, nh, enc_off, size);
    return hipGetLastError();
}

hipError_t launch_col_write(hipStream_t st, const RenderView &v, const int64_t *off, const int64_t *hpos,
                            const int64_t *hl, int64_t nh, const int64_t *enc_off, const uint8_t *enc, uint8_t *out)
{
    hipLaunchKernelGGL(k_col_direct, rgrid(2 * v.n_hits), dim3(256), 0, st, v, off, hpos, out);
    if (nh) hipLaunchKernelGGL(k_col_copy_holed, rgrid(nh), dim3(256), 0, st, hl, nh, enc_off, enc, off, out);
    return hipGetLastError();
}

}  // namespace bsq
