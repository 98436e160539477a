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

// the two subsequence texts of every row (build_tuple_bwa's nuclseq_from_text inputs, extension.cpp:285,290):
// text 2k = ref_subseq of row k, text 2k+1 = its query_subseq, at toff[]
__global__ void k_sub_write(RenderView v, const int64_t *toff, char *out)
{
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < v.n_hits; k += (int64_t)gridDim.x * blockDim.x) {
        const bsq_hit x = v.hits[k];
        ref_subseq(v, x, out + toff[2 * k]);
        query_subseq(v, x, out + toff[2 * k + 1]);
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

// lengths of the two subsequence texts of every row (text 2k: re - rb, text 2k+1: qe - qb) and their pac bytes,
// with a 0 at [2 n_hits] so an exclusive scan of n + 1 entries gives the offsets and the totals
__global__ void k_col_lens(const bsq_hit *hits, int64_t n_hits, int64_t *tl, int64_t *pl)
{
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n_hits; k += (int64_t)gridDim.x * blockDim.x) {
        const bsq_hit x = hits[k];
        const int64_t l0 = x.re - x.rb, l1 = (int64_t)x.qe - x.qb;
        tl[2 * k] = l0; tl[2 * k + 1] = l1;
        pl[2 * k] = (l0 + 3) >> 2; pl[2 * k + 1] = (l1 + 3) >> 2;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) { tl[2 * n_hits] = 0; pl[2 * n_hits] = 0; }
}

hipError_t launch_col_lens(hipStream_t st, const RenderView &v, int64_t *tl, int64_t *pl)
{
    hipLaunchKernelGGL(k_col_lens, rgrid(v.n_hits), dim3(256), 0, st, v.hits, v.n_hits, tl, pl);
    return hipGetLastError();
}

hipError_t launch_sub_write(hipStream_t st, const RenderView &v, const int64_t *toff, char *out)
{
    hipLaunchKernelGGL(k_sub_write, rgrid(v.n_hits), dim3(256), 0, st, v, toff, out);
    return hipGetLastError();
}

}  // namespace bsq
