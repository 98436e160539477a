// codec_gpu.hip -- the nuclseq codec over whole batches on the GPU (nuclseq_in /
// nuclseq_out and the conversion step of the bioseqdb-import loader for 3 Gbp references).
//
// Encode = nuclseq_in (extension.cpp:46-61) + nuclseq_from_text (sequence.cpp:209-245) for n texts at
// once.  The reference walks each text serially: holes are runs of one non-ACGT symbol
// (calculate_num_of_holes :46-57) and every hole base, then every padding base up to the byte boundary,
// takes the next draw of std::minstd_rand(holes_num ^ len).  Here one lane owns one output pac byte
// (4 bases) of one text, 256 lanes a tile:
//   pass 1  per-tile counts of hole bases and hole starts, each text's exclusive count inside the tile
//           of its first byte, the alphabet check (first offending character by atomicMin);
//   scans   tile prefixes -> per-text hole bases, hole count, varlena size -> output offsets;
//   pass 2  pac bytes and hole records: a lane's first draw is seed * 48271^d mod (2^31 - 1), d the
//           1-based index of that draw in its text (jump-ahead by square-and-multiply), later draws step
//           the LCG; hole starts write offset/amb, hole ends write end+1 into the length field;
//   pass 3  headers (+ zeroed alignment tail), and every hole's length = end - offset.
// Decode = to_text_palloc / inplace_to_text (sequence.cpp:71-81,162-166): four characters per lane from
// one pac byte, then the hole overlay in hole order (later holes win), one block per text with holes.
#include <string.h>
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

namespace bsq {

#define DEV __device__ __forceinline__

static constexpr int CT = 256;                     // lanes (= pac bytes) per tile
static constexpr uint64_t MSTD = 2147483647ull;   // minstd_rand modulus 2^31 - 1

struct EncView {
    const uint8_t *text;   // concatenated texts
    const int64_t *toff;   // n+1 text offsets
    const int64_t *poff;   // n+1 pac-byte offsets (ceil(len/4) prefix): the lane space
    int64_t n, slots;
    int validate;
};

DEV int nt4_dev(uint32_t c)   // nst_nt4_table (sequence.h:51-53)
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

DEV bool allowed_dev(uint32_t c)   // "ACGTNWSMKRYBDHV" (sequence.h:16)
{
    switch (c) {
    case 'A': case 'C': case 'G': case 'T': case 'N': case 'W': case 'S': case 'M':
    case 'K': case 'R': case 'Y': case 'B': case 'D': case 'H': case 'V': return true;
    default: return false;
    }
}

DEV uint64_t mulmod31(uint64_t a, uint64_t b)
{
    uint64_t p = a * b;   // < 2^62
    p = (p & MSTD) + (p >> 31);
    p = (p & MSTD) + (p >> 31);
    return p >= MSTD ? p - MSTD : p;
}

DEV uint64_t minstd_jump(uint64_t x0, uint64_t d)   // x0 * 48271^d mod M: the d-th draw after seeding
{
    uint64_t r = x0, b = 48271;
    d %= (MSTD - 1);   // M is prime: 48271^(M-1) = 1
    while (d) {
        if (d & 1) r = mulmod31(r, b);
        b = mulmod31(b, b);
        d >>= 1;
    }
    return r;
}

// largest s in [lo, hi] with poff[s] <= g (skips texts without bytes)
DEV int64_t text_of(const int64_t *poff, int64_t g, int64_t lo, int64_t hi)
{
    while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (poff[mid] <= g) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// tile_first[t] = the text holding pac byte t * CT (every tile start lies in exactly one text with bytes), so a tile
// finds its texts with two loads instead of two binary searches by its first lane while the other 255 wait (a batch
// of row columns holds ~2M texts of ~40 bytes: 21 dependent loads per tile before any lane could start)
__global__ void k_enc_tiles(const int64_t *poff, int64_t n, int64_t ntiles, int64_t *tile_first)
{
    // one thread per tile (each search independent, all in flight at once: a few huge texts or millions of
    // short ones alike)
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t <= ntiles; t += (int64_t)gridDim.x * blockDim.x)
        tile_first[t] = t < ntiles ? text_of(poff, t * CT, 0, n - 1) : (n > 0 ? n - 1 : 0);
}

// the tile's first text and an upper bound of its last (the text holding the next tile's first byte)
DEV void tile_texts(const int64_t *tile_first, int64_t tile, int64_t &s_lo, int64_t &s_hi)
{
    s_lo = tile_first[tile];
    s_hi = tile_first[tile + 1];
}

// hole bases (low 16 bits) and hole starts (high 16 bits) among the lane's 4 bases
DEV uint32_t lane_counts(const EncView &v, int64_t s, int64_t i0, unsigned long long *bad)
{
    const int64_t b = v.toff[s], len = v.toff[s + 1] - b;
    const int64_t e = i0 + 4 < len ? i0 + 4 : len;
    uint32_t prev = i0 > 0 ? v.text[b + i0 - 1] : 0, hb = 0, hs = 0;
    for (int64_t i = i0; i < e; ++i) {
        const uint32_t c = v.text[b + i];
        if (nt4_dev(c) >= 4) { ++hb; hs += c != prev; }
        if (bad && !allowed_dev(c)) atomicMin(bad, (unsigned long long)(b + i));
        prev = c;
    }
    return hb | hs << 16;
}

using TileScan = hipcub::BlockScan<uint32_t, CT>;

__global__ __launch_bounds__(CT) void k_enc_count(EncView v, int64_t ntiles, const int64_t *tile_first, int64_t *tile_hb,
                                                  int64_t *tile_hs, uint32_t *loc, unsigned long long *bad)
{
    __shared__ typename TileScan::TempStorage ts;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        int64_t s_lo, s_hi;
        tile_texts(tile_first, tile, s_lo, s_hi);
        const int64_t g = tile * CT + threadIdx.x;
        uint32_t cnt = 0;
        int64_t s = -1, i0 = 0;
        if (g < v.slots) {
            s = text_of(v.poff, g, s_lo, s_hi);
            i0 = (g - v.poff[s]) * 4;
            cnt = lane_counts(v, s, i0, v.validate ? bad : nullptr);
        }
        uint32_t excl, total;
        TileScan(ts).ExclusiveSum(cnt, excl, total);
        if (threadIdx.x == 0) { tile_hb[tile] = total & 0xffff; tile_hs[tile] = total >> 16; }
        if (s >= 0 && i0 == 0) {   // the text's first byte, and the texts without bytes just before it
            loc[s] = excl;
            for (int64_t t = s - 1; t >= 0 && v.poff[t] == g; --t) loc[t] = excl;
        }
        __syncthreads();
    }
}

// per text: global ranks of its first hole base / hole start; [n] = the totals
__global__ void k_enc_meta(EncView v, const int64_t *tile_hb, const int64_t *tile_hs, int64_t ntiles,
                           const uint32_t *loc, int64_t *hb_base, int64_t *hs_base)
{
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s <= v.n; s += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p = v.poff[s];
        if (s < v.n && p < v.slots) {
            hb_base[s] = tile_hb[p / CT] + (loc[s] & 0xffff);
            hs_base[s] = tile_hs[p / CT] + (loc[s] >> 16);
        } else {
            hb_base[s] = tile_hb[ntiles];
            hs_base[s] = tile_hs[ntiles];
        }
    }
}

// varlena sizes rounded to 8 bytes (the scan input of the output offsets)
__global__ void k_enc_size(EncView v, const int64_t *hs_base, int64_t *size)
{
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s <= v.n; s += (int64_t)gridDim.x * blockDim.x) {
        if (s == v.n) { size[s] = 0; continue; }
        const int64_t sz = 12 + 16 * (hs_base[s + 1] - hs_base[s]) + (v.poff[s + 1] - v.poff[s]);
        size[s] = (sz + 7) & ~(int64_t)7;
    }
}

DEV void st32(uint8_t *p, uint32_t x) { *reinterpret_cast<uint32_t *>(p) = x; }   // 4-byte aligned
DEV uint32_t ld32(const uint8_t *p) { return *reinterpret_cast<const uint32_t *>(p); }

__global__ __launch_bounds__(CT) void k_enc_write(EncView v, int64_t ntiles, const int64_t *tile_first,
                                                  const int64_t *tile_hb, const int64_t *tile_hs, const int64_t *hb_base,
                                                  const int64_t *hs_base, const int64_t *out_off, uint8_t *out)
{
    __shared__ typename TileScan::TempStorage ts;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        int64_t s_lo, s_hi;
        tile_texts(tile_first, tile, s_lo, s_hi);
        const int64_t g = tile * CT + threadIdx.x;
        uint32_t cnt = 0;
        int64_t s = -1, i0 = 0;
        if (g < v.slots) {
            s = text_of(v.poff, g, s_lo, s_hi);
            i0 = (g - v.poff[s]) * 4;
            cnt = lane_counts(v, s, i0, nullptr);
        }
        uint32_t excl, total;
        TileScan(ts).ExclusiveSum(cnt, excl, total);
        if (s >= 0) {
            const int64_t b = v.toff[s], len = v.toff[s + 1] - b;
            const int64_t nh = hs_base[s + 1] - hs_base[s];
            uint64_t d = (uint64_t)(tile_hb[tile] + (excl & 0xffff) - hb_base[s]) + 1;   // next draw, 1-based
            int64_t h = tile_hs[tile] + (excl >> 16) - hs_base[s];                        // next hole start
            uint8_t *holes = out + out_off[s] + 12;
            uint64_t seed = ((uint64_t)(uint32_t)nh ^ (uint64_t)len) % MSTD;
            if (!seed) seed = 1;
            uint64_t x = 0;   // state after draw d-1 (0: not computed yet)
            uint32_t prev = i0 > 0 ? v.text[b + i0 - 1] : 0, byte = 0;
            for (int j = 0; j < 4; ++j) {
                const int64_t i = i0 + j;
                uint32_t code;
                if (i < len) {
                    const uint32_t c = v.text[b + i];
                    code = (uint32_t)nt4_dev(c);
                    if (code >= 4) {
                        x = x ? mulmod31(x, 48271) : minstd_jump(seed, d);
                        ++d;
                        code = (uint32_t)x & 3;
                        if (c != prev) {   // a new hole: offset (int64 as two aligned words), amb + zero padding
                            uint8_t *r = holes + 16 * h;
                            st32(r, (uint32_t)i); st32(r + 4, (uint32_t)((uint64_t)i >> 32));
                            st32(r + 12, c);
                            ++h;
                        }
                        if (i + 1 == len || v.text[b + i + 1] != c) st32(holes + 16 * (h - 1) + 8, (uint32_t)(i + 1));
                    }
                    prev = c;
                } else {   // padding bases after the last hole base
                    x = x ? mulmod31(x, 48271) : minstd_jump(seed, d);
                    ++d;
                    code = (uint32_t)x & 3;
                }
                byte |= code << ((3 - j) << 1);
            }
            out[out_off[s] + 12 + 16 * nh + (g - v.poff[s])] = (uint8_t)byte;
        }
        __syncthreads();
    }
}

// headers {VARSIZE << 2, holes_num, len} and the zeroed alignment tail of every varlena
__global__ void k_enc_header(EncView v, const int64_t *hs_base, const int64_t *out_off, uint8_t *out)
{
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < v.n; s += (int64_t)gridDim.x * blockDim.x) {
        const int64_t nh = hs_base[s + 1] - hs_base[s], len = v.toff[s + 1] - v.toff[s];
        const int64_t size = 12 + 16 * nh + (v.poff[s + 1] - v.poff[s]);
        uint8_t *p = out + out_off[s];
        st32(p, (uint32_t)(size << 2));
        st32(p + 4, (uint32_t)nh);
        st32(p + 8, (uint32_t)len);
        for (int64_t k = size; k < out_off[s + 1] - out_off[s]; ++k) p[k] = 0;
    }
}

// hole lengths: the length field holds end+1 after k_enc_write
__global__ void k_enc_holes(EncView v, const int64_t *hs_base, int64_t n_holes, const int64_t *out_off, uint8_t *out)
{
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n_holes; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = text_of(hs_base, k, 0, v.n - 1);
        uint8_t *r = out + out_off[s] + 12 + 16 * (k - hs_base[s]);
        const uint32_t off = ld32(r), end = ld32(r + 8);   // offsets < 2^29 (nuclseq_in's length limit)
        st32(r + 8, end - off);
    }
}

inline dim3 cgrid(int64_t n, int per = 256)
{
    const int64_t b = (n + per - 1) / per;
    return dim3((unsigned)(b < (1 << 20) ? (b ? b : 1) : (1 << 20)));
}

// tile_first: ntiles + 1 entries of scratch, filled here and read again by launch_enc_write
hipError_t launch_enc_count(hipStream_t st, const EncView &v, int64_t ntiles, int64_t *tile_first, int64_t *tile_hb,
                            int64_t *tile_hs, uint32_t *loc, unsigned long long *bad)
{
    if (ntiles) {
        hipLaunchKernelGGL(k_enc_tiles, cgrid(ntiles + 1), dim3(256), 0, st, v.poff, v.n, ntiles, tile_first);
        hipLaunchKernelGGL(k_enc_count, cgrid(ntiles, 1), dim3(CT), 0, st, v, ntiles, tile_first, tile_hb, tile_hs,
                           loc, bad);
    }
    return hipGetLastError();
}

hipError_t launch_enc_meta(hipStream_t st, const EncView &v, const int64_t *tile_hb, const int64_t *tile_hs,
                           int64_t ntiles, const uint32_t *loc, int64_t *hb_base, int64_t *hs_base, int64_t *size)
{
    hipLaunchKernelGGL(k_enc_meta, cgrid(v.n + 1), dim3(256), 0, st, v, tile_hb, tile_hs, ntiles, loc, hb_base, hs_base);
    hipLaunchKernelGGL(k_enc_size, cgrid(v.n + 1), dim3(256), 0, st, v, hs_base, size);
    return hipGetLastError();
}

hipError_t launch_enc_write(hipStream_t st, const EncView &v, int64_t ntiles, const int64_t *tile_first,
                            const int64_t *tile_hb, const int64_t *tile_hs, const int64_t *hb_base,
                            const int64_t *hs_base, const int64_t *out_off, int64_t n_holes, uint8_t *out)
{
    if (ntiles)
        hipLaunchKernelGGL(k_enc_write, cgrid(ntiles, 1), dim3(CT), 0, st, v, ntiles, tile_first, tile_hb, tile_hs,
                           hb_base, hs_base, out_off, out);
    if (v.n) hipLaunchKernelGGL(k_enc_header, cgrid(v.n), dim3(256), 0, st, v, hs_base, out_off, out);
    if (n_holes) hipLaunchKernelGGL(k_enc_holes, cgrid(n_holes), dim3(256), 0, st, v, hs_base, n_holes, out_off, out);
    return hipGetLastError();
}

// ---- decode ----------------------------------------------------------------------------------------
struct DecView {
    const uint8_t *in;      // concatenated varlenas (each 8-byte aligned)
    const int64_t *in_off;  // n+1
    const int64_t *poff;    // n+1 pac-byte offsets (the lane space)
    const int64_t *toff;    // n+1 text offsets of the output
    int64_t n, slots;
};

// CODES: nt4 codes (0..3, holes 4) for the alignment path instead of text
template <bool CODES>
__global__ void k_dec_bases(DecView v, char *out)
{
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < v.slots; g += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = text_of(v.poff, g, 0, v.n - 1);
        const uint8_t *ns = v.in + v.in_off[s];
        const uint32_t nh = ld32(ns + 4);
        const int64_t len = v.toff[s + 1] - v.toff[s], j = g - v.poff[s];
        const uint32_t byte = ns[12 + 16 * (int64_t)nh + j];
        char *o = out + v.toff[s] + 4 * j;
        for (int k = 0; k < 4 && 4 * j + k < len; ++k) {
            const uint32_t c = (byte >> ((3 - k) << 1)) & 3;
            o[k] = CODES ? (char)c : "ACGT"[c];
        }
    }
}

// Short texts (reads: ~38 pac bytes): one lane per text walks its pac words -- k_dec_bases' per-byte lanes each
// binary-search the text over all n (18 dependent loads per byte for a 262k-read fetch).  The pac bytes start 4-byte
// aligned (8-aligned varlena + 12 + 16 per hole).
template <bool CODES>
__global__ void k_dec_bases_lane(DecView v, char *out)
{
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < v.n; s += (int64_t)gridDim.x * blockDim.x) {
        const uint8_t *ns = v.in + v.in_off[s];
        const uint32_t nh = ld32(ns + 4);
        const int64_t len = v.toff[s + 1] - v.toff[s];
        const uint8_t *pac = ns + 12 + 16 * (int64_t)nh;
        char *o = out + v.toff[s];
        for (int64_t i = 0; i < len; i += 16) {
            const uint32_t w = ld32(pac + (i >> 2));   // bytes i/4 .. i/4+3: bases i .. i+15, first byte lowest
            const int m = len - i < 16 ? (int)(len - i) : 16;
            for (int k = 0; k < m; ++k) {
                const uint32_t c = (w >> (((k >> 2) << 3) + ((3 - (k & 3)) << 1))) & 3;
                o[i + k] = CODES ? (char)c : "ACGT"[c];
            }
        }
    }
}

// one block per text with holes: holes in order, later ones overwrite (inplace_to_text :77-78); as nt4
// codes every hole base is 4 (ns_to_nt4: hole symbols are never ACGT)
template <bool CODES>
__global__ void k_dec_holes(DecView v, const int64_t *texts, char *out)
{
    const int64_t s = texts[blockIdx.x];
    const uint8_t *ns = v.in + v.in_off[s];
    const uint32_t nh = ld32(ns + 4);
    const int64_t len = v.toff[s + 1] - v.toff[s];
    char *o = out + v.toff[s];
    for (uint32_t h = 0; h < nh; ++h) {
        const uint8_t *r = ns + 12 + 16 * (int64_t)h;
        const int64_t off = (int64_t)((uint64_t)ld32(r) | (uint64_t)ld32(r + 4) << 32);
        const int32_t hl = (int32_t)ld32(r + 8);
        const char amb = CODES ? (char)4 : (char)r[12];
        const int64_t a = off < 0 ? 0 : off, e = off + hl < len ? off + hl : len;
        for (int64_t i = a + threadIdx.x; i < e; i += blockDim.x) o[i] = amb;
        __syncthreads();
    }
}

template <bool CODES>
static hipError_t dec(hipStream_t st, const DecView &v, const int64_t *hole_texts, int64_t n_hole_texts, char *out)
{
    if (v.slots && v.slots <= 64 * v.n) hipLaunchKernelGGL(k_dec_bases_lane<CODES>, cgrid(v.n), dim3(256), 0, st, v, out);
    else if (v.slots) hipLaunchKernelGGL(k_dec_bases<CODES>, cgrid(v.slots), dim3(256), 0, st, v, out);
    for (int64_t k = 0; k < n_hole_texts; k += 65535)   // one block per text with holes
        hipLaunchKernelGGL(k_dec_holes<CODES>, dim3((unsigned)(n_hole_texts - k < 65535 ? n_hole_texts - k : 65535)),
                           dim3(256), 0, st, v, hole_texts + k, out);
    return hipGetLastError();
}

hipError_t launch_dec(hipStream_t st, const DecView &v, const int64_t *hole_texts, int64_t n_hole_texts, char *out)
{
    return dec<false>(st, v, hole_texts, n_hole_texts, out);
}

hipError_t launch_dec_codes(hipStream_t st, const DecView &v, const int64_t *hole_texts, int64_t n_hole_texts,
                            uint8_t *codes)
{
    return dec<true>(st, v, hole_texts, n_hole_texts, reinterpret_cast<char *>(codes));
}

}  // namespace bsq
