// index_gpu.hip -- the alignment index built on the GPU.
//
// Replaces the host construction of BwaIndex::build (bioseqdb/bwa.cpp:107-128 -> libbwa is_bwt,
// bwt_bwtupdate_core, bwt_cal_sa; index_build.cpp here) for references whose host suffix sort is the
// slow step (minutes at 3 Gbp).  Output: the same device tables bsq_index_upload produces from a host
// build, bit for bit (the suffix array of T$ is unique, so any correct suffix sort gives the same SA,
// BWT, occurrence blocks, primary row and L2):
//   * T = pac || revcomp(pac) (the text pac2bwt sorts, bwa.cpp:20-53), T$ with $ smallest;
//   * suffix array by prefix doubling on rocPRIM radix sorts: every suffix is keyed by its first 21
//     characters over {$, A, C, G, T} (3 bits each, so a suffix reaching $ gets a unique key), sorted
//     once; then only the suffixes still tied are re-sorted each round by (tie group, rank of the
//     suffix h characters on), h = 21, 42, 84, ... until every group is a singleton;
//   * BWT ($ removed, primary = row of suffix 0) straight into 128-base OccBlocks: one 64-lane wave per
//     half block, the two bit-planes by ballot, block counts by an exclusive scan.
// Integer/byte work only (sorts, scans, gathers): HBM-bound, no MFMA.
#include <hip/hip_runtime.h>
#include <string.h>

#include <rocprim/rocprim.hpp>
#include <stdint.h>

#include <stdio.h>
#include <stdlib.h>

#include <string>

#include "bsq_device.h"

namespace bsq {

#define DEV __device__ __forceinline__

namespace {

// code of T$[i] over {$ = 0, A = 1, C = 2, G = 3, T = 4}; n = 2 l_pac, T$[n] = $ (and beyond: 0)
DEV uint32_t tchar(const uint8_t *pac, int64_t l_pac, uint64_t i)
{
    const uint64_t n = (uint64_t)l_pac << 1;
    if (i >= n) return 0;
    const uint64_t f = i < (uint64_t)l_pac ? i : n - 1 - i;
    const uint32_t b = (pac[f >> 2] >> ((~f & 3) << 1)) & 3;
    return i < (uint64_t)l_pac ? b + 1 : 4 - b;
}

constexpr int KCH = 21;   // characters in the first-round key (3 bits each, 63 bits)

// A dispatch holds < 2^32 work-items, and texts here reach 6e9 suffixes: every index-space kernel is a
// grid-stride loop over a capped grid (grid_of).
#define GRID_LOOP(i, m) for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (m); i += (uint64_t)gridDim.x * blockDim.x)

template <typename P>
__global__ void k_init_keys(const uint8_t *pac, int64_t l_pac, uint64_t N, uint64_t *key, P *val)
{
    GRID_LOOP(i, N) {
        uint64_t k = 0;
    #pragma unroll
        for (int c = 0; c < KCH; ++c) k = k << 3 | tchar(pac, l_pac, i + c);
        key[i] = k;
        val[i] = (P)i;
    }
}

// hv[j] = j if slot j starts a run of equal keys, else 0 (its inclusive max-scan is the run's first slot)
template <typename P>
__global__ void k_run_heads(const uint64_t *key, uint64_t m, const P *slot, P *hv)
{
    GRID_LOOP(j, m) {
        const bool head = j == 0 || key[j] != key[j - 1];
        const P s = slot ? slot[j] : (P)j;
        hv[j] = head ? s : (P)0;
    }
}

// rank[SA[j]] = group head of slot j
template <typename P>
__global__ void k_set_ranks(uint64_t N, const P *sa, const P *gid, P *rank)
{
    GRID_LOOP(j, N) {
        rank[sa[j]] = gid[j];
    }
}

// flag[u] = slot list[u] (list == nullptr: slot u) is in a group of more than one suffix
template <typename P>
__global__ void k_tied(uint64_t m, const P *g, uint8_t *flag)
{
    GRID_LOOP(u, m) {
        const P h = g[u];
        flag[u] = (u > 0 && g[u - 1] == h) || (u + 1 < m && g[u + 1] == h);
    }
}

// chunked scans: apply the previous chunk's last output to this chunk (max or sum)
template <typename P>
__global__ void k_carry(P *x, uint64_t m, const P *prev, int is_max)
{
    GRID_LOOP(u, m) {
        const P c = *prev;
        x[u] = is_max ? (x[u] > c ? x[u] : c) : x[u] + c;
    }
}

// keys out of order after a sort (a self-check of the sort at sizes beyond 2^32, BSQ_IDX_CHECK=1)
__global__ void k_count_unsorted(uint64_t m, const uint64_t *key, unsigned long long *cnt)
{
    for (uint64_t b0 = (uint64_t)blockIdx.x * blockDim.x; b0 < m; b0 += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t u = b0 + threadIdx.x;
        const int c = __syncthreads_count(u > 0 && u < m && key[u] < key[u - 1]);
        if (threadIdx.x == 0 && c) atomicAdd(cnt, (unsigned long long)c);
    }
}

// MSD split for texts of >= 2^32 suffixes: bucket = the first two characters (key bits 57..62); each
// block reserves its items' places per bucket with one atomic, so the scatter is one pass
constexpr int SB_ITEMS = 16;
__global__ void __launch_bounds__(256) k_bucket_hist(uint64_t N, const uint64_t *key, unsigned long long *cnt)
{
    __shared__ unsigned int h[64];
    if (threadIdx.x < 64) h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * 256 * SB_ITEMS;
    for (int k = 0; k < SB_ITEMS; ++k) {
        const uint64_t i = base + threadIdx.x + (uint64_t)k * 256;
        if (i < N) atomicAdd(&h[key[i] >> 57], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 64 && h[threadIdx.x]) atomicAdd(&cnt[threadIdx.x], (unsigned long long)h[threadIdx.x]);
}

template <typename P>
__global__ void __launch_bounds__(256) k_bucket_scatter(uint64_t N, const uint64_t *key, const P *val,
                                                        unsigned long long *cursor, uint64_t *okey, P *oval)
{
    __shared__ unsigned int h[64];
    __shared__ unsigned long long b0[64];
    if (threadIdx.x < 64) h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * 256 * SB_ITEMS;
    unsigned int loc[SB_ITEMS];
    for (int k = 0; k < SB_ITEMS; ++k) {
        const uint64_t i = base + threadIdx.x + (uint64_t)k * 256;
        loc[k] = i < N ? atomicAdd(&h[key[i] >> 57], 1u) : 0u;
    }
    __syncthreads();
    if (threadIdx.x < 64) b0[threadIdx.x] = h[threadIdx.x] ? atomicAdd(&cursor[threadIdx.x], (unsigned long long)h[threadIdx.x]) : 0ull;
    __syncthreads();
    for (int k = 0; k < SB_ITEMS; ++k) {
        const uint64_t i = base + threadIdx.x + (uint64_t)k * 256;
        if (i >= N) continue;
        const uint64_t kk = key[i];
        const uint64_t d = b0[kk >> 57] + loc[k];
        okey[d] = kk;
        oval[d] = val[i];
    }
}

// SA certificate (BSQ_IDX_CHECK=1): adjacent suffixes strictly increasing, every position present once
template <typename P>
__global__ void k_verify_sa(const uint8_t *pac, int64_t l_pac, uint64_t N, const P *sa, uint32_t *seen,
                            unsigned long long *bad)
{
    GRID_LOOP(j, N) {
        const uint64_t a = sa[j];
        if (a >= N) { atomicAdd(bad, 1ull); continue; }
        const uint32_t old = atomicOr(&seen[a >> 5], 1u << (a & 31));
        if (old & (1u << (a & 31))) atomicAdd(bad, 1ull);
        if (j + 1 == N) continue;
        const uint64_t b = sa[j + 1];
        if (b >= N) continue;
        for (uint64_t k = 0;; ++k) {   // T$ ends in the unique $, so the loop ends by the shorter suffix
            const uint32_t ca = tchar(pac, l_pac, a + k), cb = tchar(pac, l_pac, b + k);
            if (ca != cb) { if (ca > cb) atomicAdd(bad, 1ull); break; }
            if (ca == 0) { atomicAdd(bad, 1ull); break; }   // equal up to $: the same suffix twice
        }
    }
}

// number of set flags (one atomic per block)
__global__ void k_count_flags(uint64_t m, const uint8_t *flag, unsigned long long *cnt)
{
    for (uint64_t b0 = (uint64_t)blockIdx.x * blockDim.x; b0 < m; b0 += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t u = b0 + threadIdx.x;
        const int c = __syncthreads_count(u < m && flag[u]);
        if (threadIdx.x == 0 && c) atomicAdd(cnt, (unsigned long long)c);
    }
}

// gather gid of the tied slots and mark the first slot of each tie group
template <typename P>
__global__ void k_group_heads(uint64_t m, const P *U, const P *gid, P *hd)
{
    GRID_LOOP(u, m) {
        hd[u] = (u == 0 || gid[U[u]] != gid[U[u - 1]]) ? (P)1 : (P)0;
    }
}

// doubling key of tied slot U[u]: (tie group index, rank of the suffix h characters on)
template <typename P>
__global__ void k_double_keys(uint64_t m, const P *U, const P *gc, const P *sa, const P *rank, uint64_t h, int rb,
                              uint64_t *key, P *val)
{
    GRID_LOOP(u, m) {
        const P p = sa[U[u]];
        key[u] = (uint64_t)(gc[u] - 1) << rb | (uint64_t)rank[(uint64_t)p + h];
        val[u] = p;
    }
}

template <typename P>
__global__ void k_double_write(uint64_t m, const P *U, const P *val, const P *g, P *sa, P *gid, P *rank)
{
    GRID_LOOP(u, m) {
        const P j = U[u], h = g[u], p = val[u];
        sa[j] = p;
        gid[j] = h;
        rank[p] = h;
    }
}

template <typename P>
__global__ void k_find_primary(uint64_t N, const P *sa, unsigned long long *primary)
{
    GRID_LOOP(j, N) if (sa[j] == 0) *primary = j;
}

// BWT ($ removed) into the bit-planes of 128-base OccBlocks, one wave per half block; per-half counts
template <typename P>
__global__ void __launch_bounds__(256) k_bwt_planes(const uint8_t *pac, int64_t l_pac, const P *sa, uint64_t primary,
                                                    OccBlock *occ, uint64_t *hcnt)
{
    const uint64_t n = (uint64_t)l_pac << 1;
    for (uint64_t p0 = (uint64_t)blockIdx.x * blockDim.x; p0 < n; p0 += (uint64_t)gridDim.x * blockDim.x) {   // block-uniform
        const uint64_t p = p0 + threadIdx.x;
        const bool act = p < n;
        uint32_t ch = 0;
        if (act) {
            const uint64_t row = p + (p >= primary);
            ch = tchar(pac, l_pac, (uint64_t)sa[row] - 1) - 1;   // row != primary: SA[row] >= 1
        }
        const uint64_t hi = __ballot(act && (ch & 2)), lo = __ballot(act && (ch & 1));
        const uint64_t any = __ballot(act);
        if ((threadIdx.x & 63) == 0 && any) {
            const uint64_t half = p >> 6;
            OccBlock &b = occ[half >> 1];
            b.hi[half & 1] = hi;
            b.lo[half & 1] = lo;
            const uint64_t n3 = __popcll(hi & lo), n2 = __popcll(hi & ~lo), n1 = __popcll(~hi & lo);
            const uint64_t n0 = __popcll(any) - n1 - n2 - n3;
            const uint64_t nh = (n + 63) >> 6;
            hcnt[0 * nh + half] = n0; hcnt[1 * nh + half] = n1; hcnt[2 * nh + half] = n2; hcnt[3 * nh + half] = n3;
        }
    }
}

// block counts (sum of the two halves) of base c, one entry per OccBlock (the extra last blocks get 0)
__global__ void k_block_counts(uint64_t nblk, uint64_t nh, const uint64_t *hcnt, uint64_t *bc)
{
    GRID_LOOP(b, nblk) {
        for (int c = 0; c < 4; ++c) {
            const uint64_t h0 = 2 * b, h1 = 2 * b + 1;
            bc[c * nblk + b] = (h0 < nh ? hcnt[c * nh + h0] : 0) + (h1 < nh ? hcnt[c * nh + h1] : 0);
        }
    }
}

__global__ void k_occ_counts(uint64_t nblk, const uint64_t *ex, OccBlock *occ)
{
    GRID_LOOP(b, nblk) {
        for (int c = 0; c < 4; ++c) occ[b].cnt[c] = ex[c * nblk + b];
    }
}

inline dim3 grid_of(uint64_t m)
{
    const uint64_t b = (m + 255) / 256;
    return dim3((unsigned)(b < (1u << 20) ? (b ? b : 1) : (1u << 20)));   // <= 2^28 work-items per dispatch
}

struct Bufs {   // frees whatever is still allocated on every exit path
    void *p[48] = {};
    int n = 0;
    template <typename T> hipError_t alloc(T *&out, uint64_t count)
    {
        void *q = nullptr;
        int slot = 0;
        while (slot < n && p[slot]) ++slot;   // reuse a released slot
        if (slot == 48) return hipErrorOutOfMemory;
        hipError_t e = hipMalloc(&q, (size_t)(count ? count : 1) * sizeof(T));
        if (e != hipSuccess) return e;
        p[slot] = q;
        if (slot == n) ++n;
        out = (T *)q;
        return hipSuccess;
    }
    void release(void *q)
    {
        for (int i = 0; i < n; ++i) if (p[i] == q) { hipFree(q); p[i] = nullptr; }
    }
    void keep(void *q) { for (int i = 0; i < n; ++i) if (p[i] == q) p[i] = nullptr; }
    ~Bufs() { for (int i = 0; i < n; ++i) if (p[i]) hipFree(p[i]); }
};

#define GCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { err = std::string(#x) + ": " + hipGetErrorString(e_); return e_; } } while (0)

// The SA certificate over a suffix array in HBM: range, every position once (a bitmap of N bits) and
// adjacent suffixes strictly increasing; *bad = the number of violations (0 = it is the SA of T$).
template <typename P>
hipError_t certify_impl(const uint8_t *d_pac, int64_t l_pac, const P *sa, hipStream_t st, uint64_t *bad)
{
    const uint64_t N = ((uint64_t)l_pac << 1) + 1;
    uint32_t *seen = nullptr;
    unsigned long long *d_bad = nullptr;
    hipError_t e = hipMalloc(&seen, (N + 31) / 32 * 4);
    if (e == hipSuccess) e = hipMalloc(&d_bad, 8);
    if (e == hipSuccess) e = hipMemsetAsync(seen, 0, (N + 31) / 32 * 4, st);
    if (e == hipSuccess) e = hipMemsetAsync(d_bad, 0, 8, st);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_verify_sa<P>, grid_of(N), dim3(256), 0, st, d_pac, l_pac, N, sa, seen, d_bad);
        e = hipGetLastError();
    }
    unsigned long long h = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&h, d_bad, 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    hipFree(seen);
    hipFree(d_bad);
    *bad = h;
    return e;
}

template <typename P>
hipError_t build_impl(const uint8_t *d_pac, int64_t l_pac, hipStream_t st, void **sa_out, OccBlock **occ_out,
                      uint64_t *primary_out, uint64_t L2[5], uint64_t *nblk_out, int *rounds_out, uint64_t *tied_out,
                      std::string &err)
{
    const uint64_t n = (uint64_t)l_pac << 1, N = n + 1;   // suffixes of T$, row 0 = $
    Bufs B;
    uint64_t *ka, *kb;
    P *va, *vb;
    GCHK(B.alloc(ka, N)); GCHK(B.alloc(kb, N)); GCHK(B.alloc(va, N)); GCHK(B.alloc(vb, N));
    hipLaunchKernelGGL(k_init_keys<P>, grid_of(N), dim3(256), 0, st, d_pac, l_pac, N, ka, va);
    GCHK(hipGetLastError());
    void *tmp = nullptr;
    size_t tmp_bytes = 0;
    auto ensure_tmp = [&](size_t need) -> hipError_t {
        if (need <= tmp_bytes) return hipSuccess;
        if (tmp) B.release(tmp);
        uint8_t *t = nullptr;
        hipError_t e = B.alloc(t, need);
        if (e != hipSuccess) return e;
        tmp = t; tmp_bytes = need;
        return hipSuccess;
    };
    // rocPRIM scans and selects run in chunks of 2^30 items (sizes here reach 6e9 at 3 Gbp)
    const uint64_t CH = 1ull << 30;
    auto scan = [&](const P *in, P *out, uint64_t m, bool is_max) -> hipError_t {
        for (uint64_t s0 = 0; s0 < m; s0 += CH) {
            const uint64_t len = m - s0 < CH ? m - s0 : CH;
            size_t need = 0;
            hipError_t e = is_max ? rocprim::inclusive_scan(nullptr, need, in + s0, out + s0, len, rocprim::maximum<P>(), st)
                                  : rocprim::inclusive_scan(nullptr, need, in + s0, out + s0, len, rocprim::plus<P>(), st);
            if (e != hipSuccess || (e = ensure_tmp(need)) != hipSuccess) return e;
            need = tmp_bytes;
            e = is_max ? rocprim::inclusive_scan(tmp, need, in + s0, out + s0, len, rocprim::maximum<P>(), st)
                       : rocprim::inclusive_scan(tmp, need, in + s0, out + s0, len, rocprim::plus<P>(), st);
            if (e != hipSuccess) return e;
            if (s0) {
                hipLaunchKernelGGL(k_carry<P>, grid_of(len), dim3(256), 0, st, out + s0, len, (const P *)(out + s0 - 1),
                                   is_max ? 1 : 0);
                if ((e = hipGetLastError()) != hipSuccess) return e;
            }
        }
        return hipSuccess;
    };
    size_t *d_sel = nullptr;
    GCHK(B.alloc(d_sel, 1));
    // out <- src[u] (src == nullptr: u) for the flagged u < m, in order; returns the count in *cnt
    auto select = [&](const P *src, const uint8_t *flg, uint64_t m, P *out, uint64_t *cnt) -> hipError_t {
        uint64_t w = 0;
        for (uint64_t s0 = 0; s0 < m; s0 += CH) {
            const uint64_t len = m - s0 < CH ? m - s0 : CH;
            size_t need = 0;
            hipError_t e = src ? rocprim::select(nullptr, need, src + s0, flg + s0, out + w, d_sel, len, st)
                               : rocprim::select(nullptr, need, rocprim::counting_iterator<P>((P)s0), flg + s0, out + w, d_sel, len, st);
            if (e != hipSuccess || (e = ensure_tmp(need)) != hipSuccess) return e;
            need = tmp_bytes;
            e = src ? rocprim::select(tmp, need, src + s0, flg + s0, out + w, d_sel, len, st)
                    : rocprim::select(tmp, need, rocprim::counting_iterator<P>((P)s0), flg + s0, out + w, d_sel, len, st);
            if (e != hipSuccess) return e;
            size_t c = 0;
            if ((e = hipMemcpyAsync(&c, d_sel, sizeof c, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
            if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
            w += c;
        }
        *cnt = w;
        return hipSuccess;
    };
    const bool check = getenv("BSQ_IDX_CHECK") && getenv("BSQ_IDX_CHECK")[0] == '1';
    auto sorted_ok = [&](const uint64_t *key, uint64_t m) -> hipError_t {
        if (!check) return hipSuccess;
        unsigned long long *c = reinterpret_cast<unsigned long long *>(d_sel);
        hipError_t e = hipMemsetAsync(c, 0, 8, st);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_count_unsorted, grid_of(m), dim3(256), 0, st, m, key, c);
        unsigned long long h = 0;
        if ((e = hipMemcpyAsync(&h, c, 8, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
        fprintf(stderr, "[bsq index] sorted %llu keys, %llu out of order\n", (unsigned long long)m, h);
        if (h) { err = "radix sort self-check failed"; return hipErrorUnknown; }
        return hipSuccess;
    };
    // ---- round 0: sort every suffix by its first 21 characters ----
    uint64_t *skey;
    P *sa, *rank, *gid;
    const bool force_split = getenv("BSQ_IDX_SPLIT") && getenv("BSQ_IDX_SPLIT")[0] == '1';   // tests of the >= 2^32 path
    if (N < (1ull << 32) && !force_split) {
        rocprim::double_buffer<uint64_t> dk(ka, kb);
        rocprim::double_buffer<P> dv(va, vb);
        size_t need = 0;
        GCHK(rocprim::radix_sort_pairs(nullptr, need, dk, dv, N, 0, 3 * KCH, st));
        GCHK(ensure_tmp(need));
        need = tmp_bytes;
        GCHK(rocprim::radix_sort_pairs(tmp, need, dk, dv, N, 0, 3 * KCH, st));
        skey = dk.current(); sa = dv.current(); rank = dv.alternate();
        gid = reinterpret_cast<P *>(dk.alternate());   // 8N bytes: room for N slots of P
    } else {
        // >= 2^32 suffixes: split on the first two characters, then one sort per bucket (each < 2^32 items)
        unsigned long long *cnt;
        GCHK(B.alloc(cnt, 64));
        GCHK(hipMemsetAsync(cnt, 0, 64 * 8, st));
        const dim3 gb((unsigned)((N + 256 * SB_ITEMS - 1) / (256 * SB_ITEMS)));
        hipLaunchKernelGGL(k_bucket_hist, gb, dim3(256), 0, st, N, (const uint64_t *)ka, cnt);
        GCHK(hipGetLastError());
        unsigned long long hc[64], start[65];
        GCHK(hipMemcpyAsync(hc, cnt, sizeof hc, hipMemcpyDeviceToHost, st));
        GCHK(hipStreamSynchronize(st));
        start[0] = 0;
        for (int b = 0; b < 64; ++b) start[b + 1] = start[b] + hc[b];
        for (int b = 0; b < 64; ++b)
            if (hc[b] >= (1ull << 32)) { err = "a two-character bucket holds >= 2^32 suffixes"; return hipErrorUnknown; }
        GCHK(hipMemcpyAsync(cnt, start, sizeof hc, hipMemcpyHostToDevice, st));
        hipLaunchKernelGGL(k_bucket_scatter<P>, gb, dim3(256), 0, st, N, (const uint64_t *)ka, (const P *)va, cnt, kb, vb);
        GCHK(hipGetLastError());
        for (int b = 0; b < 64; ++b) {
            const uint64_t c = hc[b], s0 = start[b];
            if (!c) continue;
            size_t need = 0;
            GCHK(rocprim::radix_sort_pairs(nullptr, need, kb + s0, ka + s0, vb + s0, va + s0, c, 0, 57, st));
            GCHK(ensure_tmp(need));
            need = tmp_bytes;
            GCHK(rocprim::radix_sort_pairs(tmp, need, kb + s0, ka + s0, vb + s0, va + s0, c, 0, 57, st));
        }
        B.release(cnt);
        skey = ka; sa = va; rank = vb;
        gid = reinterpret_cast<P *>(kb);
    }
    GCHK(sorted_ok(skey, N));
    // group heads of the sorted keys (run starts, max-scanned) go through the rank buffer, then into gid;
    // the rank scatter comes last, so no N-sized scratch array is needed beside the sort buffers
    hipLaunchKernelGGL(k_run_heads<P>, grid_of(N), dim3(256), 0, st, skey, N, (const P *)nullptr, rank);
    GCHK(hipGetLastError());
    GCHK(scan(rank, gid, N, true));
    hipLaunchKernelGGL(k_set_ranks<P>, grid_of(N), dim3(256), 0, st, N, (const P *)sa, (const P *)gid, rank);
    GCHK(hipGetLastError());
    GCHK(hipStreamSynchronize(st));
    B.release(skey);   // the round-0 keys are no longer needed
    B.release(tmp); tmp = nullptr; tmp_bytes = 0;   // the big sort's scratch: later scans need far less
    // tied slots of round 0: counted first, so the list and every round buffer are sized to them
    uint8_t *flag;
    size_t *d_cnt;
    GCHK(B.alloc(flag, N)); GCHK(B.alloc(d_cnt, 1));
    hipLaunchKernelGGL(k_tied<P>, grid_of(N), dim3(256), 0, st, N, (const P *)gid, flag);
    GCHK(hipGetLastError());
    GCHK(hipMemsetAsync(d_cnt, 0, sizeof(size_t), st));
    hipLaunchKernelGGL(k_count_flags, grid_of(N), dim3(256), 0, st, N, (const uint8_t *)flag, (unsigned long long *)d_cnt);
    GCHK(hipGetLastError());
    uint64_t m = 0;
    GCHK(hipMemcpyAsync(&m, d_cnt, 8, hipMemcpyDeviceToHost, st));
    GCHK(hipStreamSynchronize(st));
    P *U = nullptr, *aux = nullptr;
    GCHK(B.alloc(U, m)); GCHK(B.alloc(aux, m));
    auto compact = [&](uint64_t mm, const P *src, uint64_t &out_m) -> hipError_t {
        // U <- the flagged slots (src == nullptr: slot numbers 0..mm-1, else src[u]), in order
        if (!src) return select(nullptr, flag, mm, U, &out_m);
        hipError_t e = select(src, flag, mm, aux, &out_m);
        if (e == hipSuccess && out_m) e = hipMemcpyAsync(U, aux, out_m * sizeof(P), hipMemcpyDeviceToDevice, st);
        return e;
    };
    {
        uint64_t m2 = 0;
        GCHK(compact(N, nullptr, m2));
        if (m2 != m) { err = "tied-suffix count mismatch"; return hipErrorUnknown; }
    }
    *tied_out = m;
    // rank bits: ranks are slot numbers < N
    int rb = 1;
    while (rb < 64 && (N >> rb)) ++rb;
    uint64_t *rk = nullptr, *rk2 = nullptr;
    P *rv = nullptr, *rv2 = nullptr, *gc = nullptr;
    if (m) {   // round buffers sized for the first tied set (later sets are subsets)
        GCHK(B.alloc(rk, m)); GCHK(B.alloc(rk2, m)); GCHK(B.alloc(rv, m)); GCHK(B.alloc(rv2, m)); GCHK(B.alloc(gc, m));
    }
    int rounds = 0;
    for (uint64_t h = KCH; m > 0; h <<= 1) {
        if (++rounds > 64 || h > N) { err = "suffix sort did not converge"; return hipErrorUnknown; }
        // tie groups among the tied slots -> group index (1-based inclusive sum of group heads)
        hipLaunchKernelGGL(k_group_heads<P>, grid_of(m), dim3(256), 0, st, m, (const P *)U, (const P *)gid, gc);
        GCHK(hipGetLastError());
        GCHK(scan(gc, gc, m, false));
        P ngroups = 0;
        GCHK(hipMemcpyAsync(&ngroups, gc + (m - 1), sizeof(P), hipMemcpyDeviceToHost, st));
        GCHK(hipStreamSynchronize(st));
        int gb = 1;
        while (gb < 64 && ((uint64_t)ngroups >> gb)) ++gb;
        if (rb + gb > 64) { err = "too many tied suffixes for a 64-bit doubling key"; return hipErrorUnknown; }
        hipLaunchKernelGGL(k_double_keys<P>, grid_of(m), dim3(256), 0, st, m, (const P *)U, (const P *)gc,
                           (const P *)sa, (const P *)rank, h, rb, rk, rv);
        GCHK(hipGetLastError());
        rocprim::double_buffer<uint64_t> rdk(rk, rk2);
        rocprim::double_buffer<P> rdv(rv, rv2);
        {
            size_t need = 0;
            GCHK(rocprim::radix_sort_pairs(nullptr, need, rdk, rdv, m, 0, rb + gb, st));
            GCHK(ensure_tmp(need));
            need = tmp_bytes;
            GCHK(rocprim::radix_sort_pairs(tmp, need, rdk, rdv, m, 0, rb + gb, st));
        }
        GCHK(sorted_ok(rdk.current(), m));
        if (check) fprintf(stderr, "[bsq index] round %d: h %llu, %llu tied suffixes in %llu groups\n", rounds,
                           (unsigned long long)h, (unsigned long long)m, (unsigned long long)ngroups);
        // new groups: runs of equal (group, rank) keys, headed by their first slot
        hipLaunchKernelGGL(k_run_heads<P>, grid_of(m), dim3(256), 0, st, (const uint64_t *)rdk.current(), m, (const P *)U, gc);
        GCHK(hipGetLastError());
        GCHK(scan(gc, gc, m, true));
        hipLaunchKernelGGL(k_double_write<P>, grid_of(m), dim3(256), 0, st, m, (const P *)U, (const P *)rdv.current(),
                           (const P *)gc, sa, gid, rank);
        GCHK(hipGetLastError());
        hipLaunchKernelGGL(k_tied<P>, grid_of(m), dim3(256), 0, st, m, (const P *)gc, flag);
        GCHK(hipGetLastError());
        uint64_t m2 = 0;
        GCHK(compact(m, U, m2));
        m = m2;
    }
    *rounds_out = rounds;
    B.release(rk); B.release(rk2); B.release(rv); B.release(rv2); B.release(gc);
    B.release(gid); B.release(rank); B.release(U); B.release(aux); B.release(flag);
    // ---- primary row, BWT -> OccBlocks ----
    unsigned long long *d_prim;
    GCHK(B.alloc(d_prim, 1));
    GCHK(hipMemsetAsync(d_prim, 0xff, 8, st));
    hipLaunchKernelGGL(k_find_primary<P>, grid_of(N), dim3(256), 0, st, N, (const P *)sa, d_prim);
    GCHK(hipGetLastError());
    unsigned long long primary = 0;
    GCHK(hipMemcpyAsync(&primary, d_prim, 8, hipMemcpyDeviceToHost, st));
    GCHK(hipStreamSynchronize(st));
    if (primary == ~0ull) { err = "suffix array has no row for position 0"; return hipErrorUnknown; }
    const uint64_t nblk = (n + 127) / 128 + 1, nh = (n + 63) >> 6;
    OccBlock *occ;
    uint64_t *hcnt, *bc;
    GCHK(B.alloc(occ, nblk)); GCHK(B.alloc(hcnt, 4 * nh)); GCHK(B.alloc(bc, 4 * nblk));
    GCHK(hipMemsetAsync(occ, 0, nblk * sizeof(OccBlock), st));
    hipLaunchKernelGGL(k_bwt_planes<P>, grid_of(n), dim3(256), 0, st, d_pac, l_pac, (const P *)sa, (uint64_t)primary, occ, hcnt);
    GCHK(hipGetLastError());
    hipLaunchKernelGGL(k_block_counts, grid_of(nblk), dim3(256), 0, st, nblk, nh, (const uint64_t *)hcnt, bc);
    GCHK(hipGetLastError());
    uint64_t tot[4];
    for (int c = 0; c < 4; ++c) {   // exclusive scan of base c over the blocks (in place), total from the last block
        uint64_t last = 0;
        GCHK(hipMemcpyAsync(&last, bc + c * nblk + nblk - 1, 8, hipMemcpyDeviceToHost, st));
        size_t need = 0;
        GCHK(rocprim::exclusive_scan(nullptr, need, bc + c * nblk, bc + c * nblk, (uint64_t)0, nblk, rocprim::plus<uint64_t>(), st));
        GCHK(ensure_tmp(need));
        need = tmp_bytes;
        GCHK(rocprim::exclusive_scan(tmp, need, bc + c * nblk, bc + c * nblk, (uint64_t)0, nblk, rocprim::plus<uint64_t>(), st));
        uint64_t ex = 0;
        GCHK(hipMemcpyAsync(&ex, bc + c * nblk + nblk - 1, 8, hipMemcpyDeviceToHost, st));
        GCHK(hipStreamSynchronize(st));
        tot[c] = ex + last;
    }
    hipLaunchKernelGGL(k_occ_counts, grid_of(nblk), dim3(256), 0, st, nblk, (const uint64_t *)bc, occ);
    GCHK(hipGetLastError());
    GCHK(hipStreamSynchronize(st));
    L2[0] = 0;
    for (int c = 0; c < 4; ++c) L2[c + 1] = L2[c] + tot[c];
    if (check) {
        uint64_t bad = 0;
        GCHK(certify_impl<P>(d_pac, l_pac, (const P *)sa, st, &bad));
        fprintf(stderr, "[bsq index] SA certificate over %llu suffixes: %llu violations\n", (unsigned long long)N,
                (unsigned long long)bad);
        if (bad) { err = "suffix array certificate failed"; return hipErrorUnknown; }
    }
    B.keep(sa); B.keep(occ);
    *sa_out = sa;
    *occ_out = occ;
    *primary_out = primary;
    *nblk_out = nblk;
    return hipSuccess;
}

}  // namespace

// Suffix array + OccBlocks of T$ for the forward pac already in device memory (d_pac, l_pac bases).
// wide: 64-bit SA entries.  On success the caller owns *sa (N = 2 l_pac + 1 entries) and *occ
// (*nblk blocks) and receives primary, L2, the number of prefix-doubling rounds and the number of
// suffixes still tied after the first (21-character) sort.
hipError_t gpu_build_index(const uint8_t *d_pac, int64_t l_pac, bool wide, hipStream_t st, void **sa, OccBlock **occ,
                           uint64_t *primary, uint64_t L2[5], uint64_t *nblk, int *rounds, uint64_t *tied, std::string &err)
{
    if (wide) return build_impl<uint64_t>(d_pac, l_pac, st, sa, occ, primary, L2, nblk, rounds, tied, err);
    return build_impl<uint32_t>(d_pac, l_pac, st, sa, occ, primary, L2, nblk, rounds, tied, err);
}

// The certificate of a suffix array already in HBM (bsq_index_certify_sa): *violations = 0 iff sa is the SA of T$.
hipError_t gpu_certify_sa(const uint8_t *d_pac, int64_t l_pac, bool wide, const void *sa, hipStream_t st,
                          uint64_t *violations)
{
    if (wide) return certify_impl<uint64_t>(d_pac, l_pac, (const uint64_t *)sa, st, violations);
    return certify_impl<uint32_t>(d_pac, l_pac, (const uint32_t *)sa, st, violations);
}

}  // namespace bsq

namespace bsq {
namespace {
// 64-base rank blocks from the 128-base ones (the device twin of the host loop in bsq_api.cpp upload_impl)
__global__ void k_occ32(uint64_t nblk, const OccBlock *occ, OccBlock32 *o32)
{
    GRID_LOOP(b, nblk) {
        const OccBlock B = occ[b];
        const uint64_t hi = B.hi[0], lo = B.lo[0];
        const uint32_t n3 = (uint32_t)__popcll(hi & lo), n2 = (uint32_t)__popcll(hi & ~lo), n1 = (uint32_t)__popcll(~hi & lo);
        const uint32_t n0 = 64u - n1 - n2 - n3;
        OccBlock32 a, c;
        for (int t = 0; t < 4; ++t) a.cnt[t] = (uint32_t)B.cnt[t];
        a.hi = B.hi[0]; a.lo = B.lo[0];
        c.cnt[0] = (uint32_t)B.cnt[0] + n0; c.cnt[1] = (uint32_t)B.cnt[1] + n1;
        c.cnt[2] = (uint32_t)B.cnt[2] + n2; c.cnt[3] = (uint32_t)B.cnt[3] + n3;
        c.hi = B.hi[1]; c.lo = B.lo[1];
        o32[2 * b] = a;
        o32[2 * b + 1] = c;
    }
}

// 64-bit rows: the same blocks with counts relative to the superblock (2^16 64-base blocks = 2^15 OccBlocks),
// and the superblocks' absolute counts after the 2 * nblk blocks (written by the thread of its first block)
__global__ void k_occ32_wide(uint64_t nblk, const OccBlock *occ, OccBlock32 *o32, SupBlock *sup)
{
    GRID_LOOP(b, nblk) {
        const OccBlock B = occ[b];
        const uint64_t sb = (2 * b) >> SUP_SHIFT;
        const OccBlock &S = occ[sb << (SUP_SHIFT - 1)];
        const uint64_t hi = B.hi[0], lo = B.lo[0];
        const uint32_t n3 = (uint32_t)__popcll(hi & lo), n2 = (uint32_t)__popcll(hi & ~lo), n1 = (uint32_t)__popcll(~hi & lo);
        const uint32_t n0 = 64u - n1 - n2 - n3;
        OccBlock32 a, c;
        for (int t = 0; t < 4; ++t) a.cnt[t] = (uint32_t)(B.cnt[t] - S.cnt[t]);
        a.hi = B.hi[0]; a.lo = B.lo[0];
        c.cnt[0] = a.cnt[0] + n0; c.cnt[1] = a.cnt[1] + n1; c.cnt[2] = a.cnt[2] + n2; c.cnt[3] = a.cnt[3] + n3;
        c.hi = B.hi[1]; c.lo = B.lo[1];
        o32[2 * b] = a;
        o32[2 * b + 1] = c;
        if (((2 * b) & ((1ull << SUP_SHIFT) - 1)) == 0) {
            SupBlock u;
            for (int t = 0; t < 4; ++t) u.cnt[t] = S.cnt[t];
            u.gt[3] = 0; u.gt[2] = S.cnt[3]; u.gt[1] = S.cnt[3] + S.cnt[2]; u.gt[0] = S.cnt[3] + S.cnt[2] + S.cnt[1];
            sup[sb] = u;
        }
    }
}
}  // namespace

hipError_t launch_occ32(hipStream_t st, const OccBlock *occ, uint64_t nblk, OccBlock32 *o32, int wide)
{
    if (!nblk) return hipSuccess;
    if (wide)
        hipLaunchKernelGGL(k_occ32_wide, grid_of(nblk), dim3(256), 0, st, nblk, occ, o32,
                           reinterpret_cast<SupBlock *>(o32 + 2 * nblk));
    else
        hipLaunchKernelGGL(k_occ32, grid_of(nblk), dim3(256), 0, st, nblk, occ, o32);
    return hipGetLastError();
}

}  // namespace bsq
