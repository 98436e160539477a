// bsq_api.cpp -- C-ABI implementation (include/bsq.h): index lifecycle, HBM upload, batch workspace
// management, kernel orchestration on a per-batch HIP stream, overflow retry, result packing.
//
// Host-side orchestration of the path that bioseqdb runs as BwaIndex::align_sequence per cursor row
// (bioseqdb/bwa.cpp:141-181, bioseqdb/extension.cpp:362-370).  There is no CPU fallback: every
// alignment result comes from the HIP kernels in align_kernels.hip; without a device the calls fail
// with BSQ_E_NODEV.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <queue>
#include <string>
#include <thread>
#include <vector>

#include "../../include/bsq.h"
#include "bsq_device.h"
#include "bsq_index.h"
#include "bsq_internal.h"

namespace bsq {
hipError_t launch_smem(int, hipStream_t, const DIndex &, const DOpts &, const Caps &, const uint8_t *, const int64_t *,
                       const int32_t *, int, Intv *, int32_t *, uint32_t *, uint8_t *, Counters *);
hipError_t launch_chain(int, hipStream_t, const DIndex &, const DOpts &, const Caps &, const int64_t *, const int32_t *,
                        int, const Intv *, const int32_t *, ChainDesc *, Seed *, int32_t *, uint32_t *, uint8_t *,
                        Counters *);
hipError_t launch_extend(int, hipStream_t, const DIndex &, const DOpts &, const Caps &, const uint8_t *, const int64_t *,
                         const int32_t *, const int64_t *, int, const ChainDesc *, const Seed *, const int32_t *, Reg *,
                         int32_t *, uint32_t *, uint8_t *, Counters *, const int32_t *, const int32_t *, int32_t *);
hipError_t launch_flt_seeds(int, hipStream_t, const DIndex &, const DOpts &, const Caps &, const uint8_t *, const int64_t *,
                            const int32_t *, int, ChainDesc *, Seed *, const int32_t *, const uint32_t *, int32_t *,
                            uint8_t *, Counters *);
hipError_t launch_ext_key(hipStream_t, const Caps &, const int64_t *, const int32_t *, int, const ChainDesc *,
                          const Seed *, const int32_t *, const uint32_t *, const int32_t *, uint32_t *, int32_t *);
hipError_t launch_reg2aln(int, hipStream_t, const DIndex &, const DOpts &, const Caps &, const uint8_t *, const int64_t *,
                          const int32_t *, int, const Reg *, const int32_t *, Hit *, uint32_t *, int32_t *, uint32_t *,
                          uint8_t *, Counters *);
struct SlotView { const Hit *hits; const uint32_t *cigars; const int32_t *n_regs; const int32_t *n_cig; Caps cp; };
hipError_t launch_counts(hipStream_t, int, const SlotView &, const SlotView &, const int32_t *, const uint32_t *, int64_t *,
                         int64_t *, unsigned long long *);
hipError_t launch_pack(hipStream_t, int, const SlotView &, const SlotView &, const int32_t *, const int64_t *,
                       const int64_t *, const int64_t *, const int64_t *, bsq_hit *, uint32_t *, int, int64_t);
hipError_t launch_add_base(hipStream_t, int64_t *, int, int64_t);
hipError_t launch_collect_overflow(hipStream_t, int, const uint32_t *, int32_t *, int32_t *);
hipError_t launch_reg2aln_chain(hipStream_t, const DIndex &, const DOpts &, const Caps &, const uint8_t *,
                                const int64_t *, int, const Reg *, const int32_t *, Hit *, uint32_t *, int32_t *,
                                uint32_t *, Counters *, int, uint8_t *, int64_t, int, int32_t *, int32_t *, int32_t *,
                                const int32_t *, const int32_t *, int32_t *);
bool wide_z32(const DIndex &);
hipError_t launch_smem_lds(hipStream_t, const DIndex &, const DOpts &, const Caps &, const uint8_t *, const int64_t *, int,
                           Intv *, int32_t *, uint32_t *, Counters *, int, uint8_t *, int, uint8_t *);
hipError_t launch_kmer_build(hipStream_t, const DIndex &, uint32_t *, int);
struct RenderHole { int64_t beg, end; uint32_t order; uint32_t amb; };
struct RenderView {
    const bsq_hit *hits; const uint32_t *cigar; int64_t n_hits; const uint8_t *pac; int64_t l_pac;
    const RenderHole *holes; int64_t n_holes; const uint8_t *codes; const int64_t *offs;
    const int64_t *rh_off; const RenderHole *rh;
};
hipError_t launch_row_len(hipStream_t, const RenderView &, int64_t *);
hipError_t launch_row_write(hipStream_t, const RenderView &, const int64_t *, char *);
hipError_t launch_col_class(hipStream_t, const RenderView &, int64_t *, int64_t *);
hipError_t launch_col_holed(hipStream_t, const RenderView &, const int64_t *, int64_t, int64_t *, int64_t *, int64_t *);
hipError_t launch_sub_write_sel(hipStream_t, const RenderView &, const int64_t *, int64_t, const int64_t *, char *);
hipError_t launch_col_holed_size(hipStream_t, const int64_t *, int64_t, const int64_t *, int64_t *);
hipError_t launch_col_write(hipStream_t, const RenderView &, const int64_t *, const int64_t *, const int64_t *, int64_t,
                            const int64_t *, const uint8_t *, uint8_t *);
hipError_t gpu_build_index(const uint8_t *, int64_t, bool, hipStream_t, void **, OccBlock **, uint64_t *, uint64_t[5],
                           uint64_t *, int *, uint64_t *, std::string &);
hipError_t gpu_certify_sa(const uint8_t *, int64_t, bool, const void *, hipStream_t, uint64_t *);
hipError_t launch_occ32(hipStream_t, const OccBlock *, uint64_t, OccBlock32 *, int);
hipError_t launch_intv_counts(hipStream_t, int, const int32_t *, const uint32_t *, int64_t *);
hipError_t launch_intv_pack(hipStream_t, int, int, const Intv *, const int32_t *, const uint32_t *, const int64_t *,
                            uint64_t *);
// codec_gpu.hip
struct EncView { const uint8_t *text; const int64_t *toff; const int64_t *poff; int64_t n, slots; int validate; };
struct DecView { const uint8_t *in; const int64_t *in_off; const int64_t *poff; const int64_t *toff; int64_t n, slots; };
hipError_t launch_enc_count(hipStream_t, const EncView &, int64_t, int64_t *, int64_t *, int64_t *, uint32_t *,
                            unsigned long long *);
hipError_t launch_enc_meta(hipStream_t, const EncView &, const int64_t *, const int64_t *, int64_t, const uint32_t *,
                           int64_t *, int64_t *, int64_t *);
hipError_t launch_enc_write(hipStream_t, const EncView &, int64_t, const int64_t *, const int64_t *, const int64_t *, const int64_t *,
                            const int64_t *, const int64_t *, int64_t, uint8_t *);
hipError_t launch_dec(hipStream_t, const DecView &, const int64_t *, int64_t, char *);
hipError_t launch_dec_codes(hipStream_t, const DecView &, const int64_t *, int64_t, uint8_t *);
}  // namespace bsq

using namespace bsq;

// roctx range over a host-side phase (index build / upload, the stage launches of a batch, the record copy):
// rocprofv3 --marker-trace shows them beside the kernels; without a profiler they cost a call.
struct Range {
    explicit Range(const char *name) { roctxRangePushA(name); }
    ~Range() { roctxRangePop(); }
    void next(const char *name) { roctxRangePop(); roctxRangePushA(name); }   // the following phase
    Range(const Range &) = delete;
    Range &operator=(const Range &) = delete;
};

static thread_local std::string g_err;
static std::atomic<int64_t> g_sort_guard{0};   // bsq_sort_guard_total: every batch run in the process
static void set_err(const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
}

#define HIPCHK(x)                                                                                  \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            set_err("%s failed: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, __LINE__);       \
            return BSQ_E_HIP;                                                                      \
        }                                                                                          \
    } while (0)

// Grow-only device scratch of a batch's renderers: chunks allocated once and carved again on every call, so a
// steady cursor loop never calls hipMalloc/hipFree (hipFree synchronises the whole device, stalling every other
// batch's stream).  reset() at the start of a call; the chunks are freed with the batch.
struct DevArena {
    std::vector<std::pair<void *, size_t>> chunks;
    size_t ci = 0, used = 0;
    void reset() { ci = 0; used = 0; }
    template <typename T>
    hipError_t get(T *&out, size_t count)
    {
        const size_t bytes = (std::max<size_t>(count, 1) * sizeof(T) + 255) & ~(size_t)255;
        while (ci < chunks.size() && used + bytes > chunks[ci].second) { ++ci; used = 0; }
        if (ci == chunks.size()) {
            void *q = nullptr;
            const size_t cap = std::max<size_t>(bytes, (size_t)64 << 20);
            const hipError_t e = hipMalloc(&q, cap);
            if (e != hipSuccess) return e;
            chunks.emplace_back(q, cap);
            used = 0;
        }
        out = reinterpret_cast<T *>(static_cast<uint8_t *>(chunks[ci].first) + used);
        used += bytes;
        return hipSuccess;
    }
    ~DevArena() { for (auto &c : chunks) hipFree(c.first); }
};

extern "C" const char *bsq_last_error(void) { return g_err.c_str(); }
// for the other translation units of the library (group.cpp); not part of include/bsq.h
extern "C" void bsq_internal_set_error(const char *msg) { g_err = msg ? msg : ""; }
extern "C" const char *bsq_version(void) { return "bsq 0.1 (gfx950)"; }

// The concurrent batch and pipeline streams of one process need more than HIP's default 4 hardware queues: the 4-batch
// C3 step measured 45 M reads/s on 4 queues against 57 M on 8 (profiles/r06/streams_queues/ab.txt; 16 level with 8).
// A process that has not chosen gets 8 -- set when the library is loaded, before its first HIP call (the runtime reads
// the variable when it initialises, on the first HIP call).  An explicit GPU_MAX_HW_QUEUES, or a HIP runtime that
// another library of the process has already initialised, is left as it is.
__attribute__((constructor)) static void bsq_default_hw_queues() { setenv("GPU_MAX_HW_QUEUES", "8", 0); }
extern "C" void bsq_free(void *p) { free(p); }

extern "C" int bsq_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

// BSQ_R2A_DIAG=0: no lane-per-read diagonal pass before the reg2aln group kernels (A/B measurements)
static bool no_r2a_diag() { const char *e = getenv("BSQ_R2A_DIAG"); return e && *e == '0'; }
// BSQ_EXT_STATIC=1: k_extend takes its reads by a fixed stride instead of a work counter (A/B measurements)
static bool ext_static() { static const bool v = [] { const char *e = getenv("BSQ_EXT_STATIC"); return e && *e == '1'; }(); return v; }
static bool tiny_caps() { const char *e = getenv("BSQ_TEST_TINY_CAPS"); return e && *e && *e != '0'; }

static int default_threads()
{
    const char *e = getenv("BSQ_THREADS");
    if (!e) e = getenv("OMP_NUM_THREADS");
    int t = e ? atoi(e) : 0;
    if (t <= 0) {
        t = (int)std::thread::hardware_concurrency();
        if (t > 16) t = 16;
    }
    return t < 1 ? 1 : t;
}

// ================================================================================================
// index
// ================================================================================================
namespace bsq {
struct DeviceIndex {
    int device = -1;
    OccBlock *occ = nullptr;
    void *sa = nullptr;
    uint8_t *pac = nullptr;
    int64_t *ann_off = nullptr, *ann_id = nullptr;
    int32_t *ann_len = nullptr;
    uint32_t *kmer = nullptr;
    OccBlock32 *occ32 = nullptr;
    bool owned = true;   // false: the tables live in caller-owned buffers (bsq_index_upload_into / _import)
    DIndex view{};
    ~DeviceIndex()
    {
        if (!owned) return;
        if (device >= 0) hipSetDevice(device);
        hipFree(occ); hipFree(sa); hipFree(pac); hipFree(ann_off); hipFree(ann_id); hipFree(ann_len); hipFree(kmer); hipFree(occ32);
    }
};
}  // namespace bsq


extern "C" int bsq_index_create(bsq_index **out)
{
    if (!out) { set_err("null out"); return BSQ_E_INVALID; }
    *out = new (std::nothrow) bsq_index();
    if (!*out) { set_err("out of memory"); return BSQ_E_NOMEM; }
    return BSQ_OK;
}

extern "C" void bsq_index_free(bsq_index *idx)
{
    if (!idx) return;
    bsq_pipeline_free(idx->pipe);
    if (idx->d_rh) {
        if (idx->h.dev) hipSetDevice(idx->h.dev->device);
        hipFree(idx->d_rh);
    }
    delete idx->h.dev;
    delete idx;
}

extern "C" int bsq_index_add_ref(bsq_index *idx, int64_t id, const void *nuclseq)
{
    if (!idx || !nuclseq) { set_err("null argument"); return BSQ_E_INVALID; }
    if (idx->h.dev) { set_err("index already uploaded; references are immutable"); return BSQ_E_INVALID; }
    idx->h.add_ref(id, static_cast<const uint8_t *>(nuclseq));
    return BSQ_OK;
}

extern "C" int bsq_index_build(bsq_index *idx, int threads)
{
    Range rg("bsq_index_build");
    if (!idx) { set_err("null index"); return BSQ_E_INVALID; }
    std::string err;
    try {
        if (idx->h.build(threads > 0 ? threads : default_threads(), err) != 0) {
            set_err("index build failed: %s", err.c_str());
            return BSQ_E_INVALID;
        }
    } catch (const std::bad_alloc &) {
        set_err("out of host memory building the index");
        return BSQ_E_NOMEM;
    }
    return BSQ_OK;
}

// bns->l_pac = 4 * pac_forward.size() (bwa.cpp:118), known as soon as the rows are added
extern "C" int64_t bsq_index_l_pac(const bsq_index *idx)
{
    return idx ? std::max<int64_t>(idx->h.l_pac, 4 * (int64_t)idx->h.pac.size()) : -1;
}
extern "C" int64_t bsq_index_seq_len(const bsq_index *idx) { return idx ? (int64_t)idx->h.seq_len : -1; }
extern "C" int64_t bsq_index_primary(const bsq_index *idx) { return idx ? (int64_t)idx->h.primary : -1; }
extern "C" int32_t bsq_index_n_refs(const bsq_index *idx) { return idx ? (int32_t)idx->h.anns.size() : -1; }

extern "C" int bsq_index_same_refs(const bsq_index *a, const bsq_index *b)
{
    if (!a || !b) return -1;
    const HostIndex &x = a->h, &y = b->h;
    // (rows as added: l_pac is only set by a build, and a fresh index is compared against a built one)
    if (x.anns.size() != y.anns.size() || x.holes.size() != y.holes.size() || x.pac.size() != y.pac.size())
        return 0;
    for (size_t i = 0; i < x.anns.size(); ++i) {
        const Ann &p = x.anns[i], &q = y.anns[i];
        if (p.offset != q.offset || p.len != q.len || p.n_ambs != q.n_ambs || p.id != q.id) return 0;
    }
    for (size_t i = 0; i < x.holes.size(); ++i) {
        const Hole &p = x.holes[i], &q = y.holes[i];
        if (p.offset != q.offset || p.len != q.len || p.amb != q.amb) return 0;
    }
    return x.pac.empty() || memcmp(x.pac.data(), y.pac.data(), x.pac.size()) == 0 ? 1 : 0;
}

static bool host_tables(const HostIndex &h) { return !h.occ.empty(); }   // false: device-built, not downloaded

extern "C" int64_t bsq_index_sa(const bsq_index *idx, int64_t row)
{
    if (!idx || !idx->h.built || row < 0 || (uint64_t)row > idx->h.seq_len || idx->h.seq_len == 0) return -1;
    if (!host_tables(idx->h)) return -1;
    return (int64_t)idx->h.sa((uint64_t)row);
}

extern "C" int bsq_index_occ4(const bsq_index *idx, int64_t k, uint64_t cnt[4])
{
    if (!idx || !idx->h.built || idx->h.seq_len == 0) { set_err("index not built"); return BSQ_E_INVALID; }
    if (k < -1 || (k >= 0 && (uint64_t)k > idx->h.seq_len)) { set_err("row out of range"); return BSQ_E_INVALID; }
    if (!host_tables(idx->h)) { set_err("device-built index: call bsq_index_download first"); return BSQ_E_INVALID; }
    idx->h.occ4((uint64_t)k, cnt);
    return BSQ_OK;
}

extern "C" const void *bsq_index_sa_data(const bsq_index *idx, int *elem_bytes)
{
    if (!idx || !idx->h.built || idx->h.seq_len == 0 || !host_tables(idx->h)) return nullptr;
    if (!idx->h.sa32.empty()) { if (elem_bytes) *elem_bytes = 4; return idx->h.sa32.data(); }
    if (elem_bytes) *elem_bytes = 8;
    return idx->h.sa64.data();
}

// ---- device tables of an index (bsq_index_layout order) and the metadata that travels with them ----
enum { T_OCC = 0, T_OCC32, T_SA, T_PAC, T_ANN_OFF, T_ANN_ID, T_ANN_LEN, T_KMER, T_N };
static_assert(T_N == BSQ_N_TABLES, "table list");

struct IndexMeta {   // fixed header of the metadata blob; followed by Ann[n_anns] and Hole[n_holes]
    char magic[8];
    uint64_t l_pac, seq_len, primary, L2[5];
    int32_t wide, kmer_k;
    uint64_t n_anns, n_holes, pac_bytes;
    uint64_t table_bytes[T_N];
};

static int kmer_depth(uint64_t seq_len, bool wide)
{
    if (seq_len == 0) return 0;
    // ~log4(rows), at most 10 while the rank blocks (32 B per 64 rows) fit the 256 MB Infinity Cache: the table
    // competes with them for it (C3, 100 MB of rank blocks: seeding 10.45 ms at K = 10 with a 22 MB table, 10.7 at
    // 11 with 89 MB, 11.3-12.1 at 12-14, 10.9 at 9); else at most 13: the rank blocks' lines miss anyway and each
    // level answers more backward extensions with one line (C4, 3 Gbp: 28.0 M reads/s at 11, 30.0 M at 13 with a
    // 2.9 GB table, round 5; 32.5 M at 15 with a 46 GB table against 31.7 M at 13, round 6).
    // Depth 15 only for 64-bit rows, the kernels that preload 15 levels (and the only ones measured there; the table
    // is at most 46 GB beside a >= 8 GB suffix array): u32 rows of a 256 Mbp - 2 Gbp text stay at 10, where u32
    // kernels preload 11 levels and read deeper ones one per step (slower at C3: 11.3-12.1 ms against 10.45).
    const int kmax = wide && seq_len / 2 > (256ull << 20) ? 15 : 10;
    int K = 0;
    while (K < kmax && (1ull << (2 * (K + 1))) <= seq_len) ++K;
    // BSQ_KMER_K: 0 disables; up to 15 (the kernels preload levels <= 11 and read deeper levels one per step;
    // 32-bit table indices and codes)
    if (const char *e = getenv("BSQ_KMER_K")) K = std::max(0, std::min(15, atoi(e)));
    return K;
}

static void table_sizes(const HostIndex &h, uint64_t bytes[T_N], int &K, int &wide)
{
    for (int t = 0; t < T_N; ++t) bytes[t] = 0;
    const bool dev_only = h.dev_built && h.occ.empty();
    wide = dev_only ? h.dev_wide : (h.sa32.empty() ? 1 : 0);
    const uint64_t nann = h.anns.size() ? h.anns.size() : 1;
    bytes[T_ANN_OFF] = nann * 8; bytes[T_ANN_ID] = nann * 8; bytes[T_ANN_LEN] = nann * 4;
    K = 0;
    if (h.seq_len == 0) return;
    const uint64_t nblk = dev_only ? h.dev_nblk : h.occ.size();
    bytes[T_OCC] = nblk * sizeof(OccBlock);
    bytes[T_OCC32] = nblk * 2 * sizeof(OccBlock32) + (wide ? occ32_sup_count(2 * nblk) * sizeof(SupBlock) : 0);
    bytes[T_SA] = (h.seq_len + 1) * (wide ? 8 : 4);
    bytes[T_PAC] = h.pac.size() + 16;
    K = kmer_depth(h.seq_len, wide != 0);
    bytes[T_KMER] = K ? (((uint64_t)1 << (2 * (K + 1))) - 4) / 3 * (wide ? 32 : 16) : 0;
}

static void set_view(DeviceIndex *d, const IndexMeta &m)
{
    DIndex &v = d->view;
    v = DIndex{};
    v.occ = d->occ;
    v.sa32 = m.wide ? nullptr : (const uint32_t *)d->sa;
    v.sa64 = m.wide ? (const uint64_t *)d->sa : nullptr;
    v.pac = d->pac;
    v.ann_off = d->ann_off;
    v.ann_len = d->ann_len;
    v.n_anns = (int32_t)m.n_anns;
    for (int c = 0; c < 5; ++c) v.L2[c] = m.L2[c];
    v.primary = m.primary;
    v.seq_len = m.seq_len;
    v.l_pac = (int64_t)m.l_pac;
    v.wide = m.wide;
    v.occ32 = d->occ32;
    v.sup = m.wide && d->occ32 ? reinterpret_cast<const SupBlock *>(d->occ32 + 2 * (m.table_bytes[T_OCC] / sizeof(OccBlock)))
                               : nullptr;
    v.kmer = m.kmer_k ? d->kmer : nullptr;
    v.kmer_k = m.kmer_k;
}

static IndexMeta meta_of(const HostIndex &h)
{
    IndexMeta m{};
    memcpy(m.magic, "BSQIDX1", 8);
    m.l_pac = (uint64_t)h.l_pac; m.seq_len = h.seq_len; m.primary = h.primary;
    for (int c = 0; c < 5; ++c) m.L2[c] = h.L2[c];
    int K = 0, wide = 0;
    table_sizes(h, m.table_bytes, K, wide);
    m.wide = wide; m.kmer_k = K;
    m.n_anns = h.anns.size(); m.n_holes = h.holes.size(); m.pac_bytes = h.pac.size();
    return m;
}

// A device-built index is already uploaded: bsq_index_upload on its device is a no-op, and
// bsq_index_upload_into copies its tables into the caller's buffers (device to device) and adopts them.
static int move_device_tables(bsq_index *idx, int device, const bsq_table *ext)
{
    HostIndex &h = idx->h;
    DeviceIndex *d = h.dev;
    if (device != d->device) { set_err("index was built on device %d", d->device); return BSQ_E_INVALID; }
    if (!ext) return BSQ_OK;
    HIPCHK(hipSetDevice(device));
    const IndexMeta m = meta_of(h);
    void *cur[T_N] = {d->occ, d->occ32, d->sa, d->pac, d->ann_off, d->ann_id, d->ann_len, d->kmer};
    for (int t = 0; t < T_N; ++t) {
        if (!m.table_bytes[t]) continue;
        if (!ext[t].ptr || ext[t].bytes < m.table_bytes[t]) { set_err("table %d: buffer of %llu bytes, %llu needed", t,
            (unsigned long long)ext[t].bytes, (unsigned long long)m.table_bytes[t]); return BSQ_E_INVALID; }
        HIPCHK(hipMemcpy(ext[t].ptr, cur[t], m.table_bytes[t], hipMemcpyDeviceToDevice));
    }
    DeviceIndex *nd = new DeviceIndex();
    nd->device = device;
    nd->owned = false;
    nd->occ = (OccBlock *)ext[T_OCC].ptr; nd->occ32 = (OccBlock32 *)ext[T_OCC32].ptr; nd->sa = ext[T_SA].ptr;
    nd->pac = (uint8_t *)ext[T_PAC].ptr; nd->ann_off = (int64_t *)ext[T_ANN_OFF].ptr; nd->ann_id = (int64_t *)ext[T_ANN_ID].ptr;
    nd->ann_len = (int32_t *)ext[T_ANN_LEN].ptr; nd->kmer = (uint32_t *)ext[T_KMER].ptr;
    set_view(nd, m);
    delete d;
    h.dev = nd;
    return BSQ_OK;
}

// Uploads the host index into its own allocations (ext == nullptr) or into caller-owned buffers.
static int upload_impl(bsq_index *idx, int device, const bsq_table *ext)
{
    Range rg("bsq_index_upload");
    if (!idx || !idx->h.built) { set_err("index not built"); return BSQ_E_INVALID; }
    const HostIndex &h = idx->h;
    if (h.dev_built && h.dev) return move_device_tables(idx, device, ext);
    if (h.seq_len > 0 && h.occ.empty()) { set_err("device-only index (imported): nothing to upload from the host"); return BSQ_E_INVALID; }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0) {
        set_err("no HIP device %d (found %d); the alignment path has no CPU fallback", device, ndev);
        return BSQ_E_NODEV;
    }
    HIPCHK(hipSetDevice(device));
    const IndexMeta m = meta_of(h);
    void *ptr[T_N] = {};
    for (int t = 0; t < T_N; ++t) {
        if (!m.table_bytes[t]) continue;
        if (ext) {
            if (!ext[t].ptr || ext[t].bytes < m.table_bytes[t]) { set_err("table %d: buffer of %llu bytes, %llu needed", t,
                (unsigned long long)ext[t].bytes, (unsigned long long)m.table_bytes[t]); return BSQ_E_INVALID; }
            ptr[t] = ext[t].ptr;
        } else HIPCHK(hipMalloc(&ptr[t], m.table_bytes[t]));
    }
    delete idx->h.dev;
    DeviceIndex *d = idx->h.dev = new DeviceIndex();
    d->device = device;
    d->owned = ext == nullptr;
    d->occ = (OccBlock *)ptr[T_OCC]; d->occ32 = (OccBlock32 *)ptr[T_OCC32]; d->sa = ptr[T_SA];
    d->pac = (uint8_t *)ptr[T_PAC]; d->ann_off = (int64_t *)ptr[T_ANN_OFF]; d->ann_id = (int64_t *)ptr[T_ANN_ID];
    d->ann_len = (int32_t *)ptr[T_ANN_LEN]; d->kmer = (uint32_t *)ptr[T_KMER];
    const size_t nann = h.anns.size() ? h.anns.size() : 1;
    std::vector<int64_t> off(nann, 0), id(nann, 0);
    std::vector<int32_t> len(nann, 0);
    for (size_t i = 0; i < h.anns.size(); ++i) { off[i] = h.anns[i].offset; id[i] = h.anns[i].id; len[i] = h.anns[i].len; }
    HIPCHK(hipMemcpy(d->ann_off, off.data(), nann * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d->ann_id, id.data(), nann * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d->ann_len, len.data(), nann * 4, hipMemcpyHostToDevice));
    if (h.seq_len > 0) {
        HIPCHK(hipMemcpy(d->occ, h.occ.data(), h.occ.size() * sizeof(OccBlock), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(d->sa, m.wide ? (const void *)h.sa64.data() : (const void *)h.sa32.data(), m.table_bytes[T_SA],
                         hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(d->pac, h.pac.data(), h.pac.size(), hipMemcpyHostToDevice));
    }
    if (h.seq_len > 0) {   // 64-base blocks (+ superblocks for 64-bit rows) from the uploaded 128-base ones
        HIPCHK(launch_occ32(nullptr, d->occ, (uint64_t)h.occ.size(), d->occ32, m.wide));
        HIPCHK(hipDeviceSynchronize());
    }
    IndexMeta mv = m;
    mv.kmer_k = 0;
    set_view(d, mv);
    // k-mer interval table (u32 rows: 89 MB at K = 11, stays in the Infinity Cache beside the occ array at
    // 100 Mbp; 64-bit rows: 32-B entries, 179 MB); BSQ_KMER_K overrides, 0 disables
    if (m.kmer_k > 0) {
        d->view.kmer = d->kmer;
        HIPCHK(launch_kmer_build(nullptr, d->view, d->kmer, m.kmer_k));
        HIPCHK(hipDeviceSynchronize());
        d->view.kmer_k = m.kmer_k;
    }
    return BSQ_OK;
}

extern "C" int bsq_index_upload(bsq_index *idx, int device) { return upload_impl(idx, device, nullptr); }

extern "C" int bsq_index_build_device(bsq_index *idx, int device)
{
    Range rg("bsq_index_build_device");
    if (!idx) { set_err("null index"); return BSQ_E_INVALID; }
    HostIndex &h = idx->h;
    if (h.dev) { set_err("index already uploaded"); return BSQ_E_INVALID; }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0) {
        set_err("no HIP device %d (found %d); the index build has no CPU fallback here (bsq_index_build is the host path)",
                device, ndev);
        return BSQ_E_NODEV;
    }
    HIPCHK(hipSetDevice(device));
    h.occ.clear(); h.sa32.clear(); h.sa64.clear();
    h.l_pac = (int64_t)h.pac.size() * 4;
    h.seq_len = (uint64_t)h.l_pac * 2;
    h.primary = 0;
    for (int c = 0; c < 5; ++c) h.L2[c] = 0;
    const char *fw = getenv("BSQ_FORCE_WIDE");   // same row-width rule as the host build
    h.dev_wide = (h.seq_len >= 0xFFFFFFFFull || (fw && *fw && *fw != '0')) ? 1 : 0;
    h.dev_nblk = h.seq_len ? (h.seq_len + 127) / 128 + 1 : 0;
    h.dev_built = true;
    h.built = true;
    const IndexMeta m = meta_of(h);
    DeviceIndex *d = h.dev = new DeviceIndex();
    d->device = device;
    auto fail = [&](int rc) { delete h.dev; h.dev = nullptr; h.built = false; h.dev_built = false; return rc; };
    void *ptr[T_N] = {};
    for (int t : {(int)T_PAC, (int)T_ANN_OFF, (int)T_ANN_ID, (int)T_ANN_LEN, (int)T_OCC32, (int)T_KMER}) {
        if (!m.table_bytes[t]) continue;
        if (hipMalloc(&ptr[t], m.table_bytes[t]) != hipSuccess) { set_err("out of device memory (table %d)", t); return fail(BSQ_E_NOMEM); }
    }
    d->pac = (uint8_t *)ptr[T_PAC]; d->ann_off = (int64_t *)ptr[T_ANN_OFF]; d->ann_id = (int64_t *)ptr[T_ANN_ID];
    d->ann_len = (int32_t *)ptr[T_ANN_LEN]; d->occ32 = (OccBlock32 *)ptr[T_OCC32]; d->kmer = (uint32_t *)ptr[T_KMER];
    const size_t nann = h.anns.size() ? h.anns.size() : 1;
    std::vector<int64_t> off(nann, 0), id(nann, 0);
    std::vector<int32_t> len(nann, 0);
    for (size_t i = 0; i < h.anns.size(); ++i) { off[i] = h.anns[i].offset; id[i] = h.anns[i].id; len[i] = h.anns[i].len; }
    if (hipMemcpy(d->ann_off, off.data(), nann * 8, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d->ann_id, id.data(), nann * 8, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d->ann_len, len.data(), nann * 4, hipMemcpyHostToDevice) != hipSuccess) {
        set_err("uploading the annotations"); return fail(BSQ_E_HIP);
    }
    if (h.seq_len == 0) { set_view(d, m); return BSQ_OK; }
    if (hipMemset(d->pac, 0, m.table_bytes[T_PAC]) != hipSuccess ||
        hipMemcpy(d->pac, h.pac.data(), h.pac.size(), hipMemcpyHostToDevice) != hipSuccess) {
        set_err("uploading the pac"); return fail(BSQ_E_HIP);
    }
    std::string err;
    int rounds = 0;
    uint64_t tied = 0, nblk = 0, primary = 0, L2[5];
    void *sa = nullptr;
    OccBlock *occ = nullptr;
    hipError_t e = gpu_build_index(d->pac, h.l_pac, h.dev_wide != 0, nullptr, &sa, &occ, &primary, L2, &nblk, &rounds,
                                   &tied, err);
    if (e != hipSuccess) {
        set_err("GPU index build: %s", err.c_str());
        return fail(e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation ? BSQ_E_NOMEM : BSQ_E_HIP);
    }
    d->sa = sa;
    d->occ = occ;
    h.primary = primary;
    for (int c = 0; c < 5; ++c) h.L2[c] = L2[c];
    h.dev_nblk = nblk;
    h.dev_rounds = rounds;
    h.dev_tied = tied;
    const IndexMeta m2 = meta_of(h);
    if (launch_occ32(nullptr, d->occ, nblk, d->occ32, m2.wide) != hipSuccess) { set_err("occ32 build"); return fail(BSQ_E_HIP); }
    IndexMeta mv = m2;
    mv.kmer_k = 0;
    set_view(d, mv);
    if (m2.kmer_k > 0) {
        d->view.kmer = d->kmer;
        if (launch_kmer_build(nullptr, d->view, d->kmer, m2.kmer_k) != hipSuccess) { set_err("k-mer table build"); return fail(BSQ_E_HIP); }
        d->view.kmer_k = m2.kmer_k;
    }
    if (hipDeviceSynchronize() != hipSuccess) { set_err("GPU index build: %s", hipGetErrorString(hipGetLastError())); return fail(BSQ_E_HIP); }
    return BSQ_OK;
}

extern "C" int bsq_index_certify_sa(const bsq_index *idx, uint64_t *suffixes, uint64_t *violations)
{
    Range rg("bsq_index_certify_sa");
    if (!idx || !idx->h.built || !idx->h.dev) { set_err("index not on a device"); return BSQ_E_INVALID; }
    const HostIndex &h = idx->h;
    if (suffixes) *suffixes = h.seq_len ? h.seq_len + 1 : 0;
    if (violations) *violations = 0;
    if (h.seq_len == 0) return BSQ_OK;
    HIPCHK(hipSetDevice(h.dev->device));
    uint64_t bad = 0;
    const hipError_t e = gpu_certify_sa(h.dev->pac, h.l_pac, meta_of(h).wide != 0, h.dev->sa, nullptr, &bad);
    if (e != hipSuccess) {
        set_err("SA certificate: %s", hipGetErrorString(e));
        return e == hipErrorOutOfMemory ? BSQ_E_NOMEM : BSQ_E_HIP;
    }
    if (violations) *violations = bad;
    return BSQ_OK;
}

extern "C" int bsq_index_build_stats(const bsq_index *idx, int *rounds, uint64_t *tied)
{
    if (!idx || !idx->h.dev_built) { set_err("not a device-built index"); return BSQ_E_INVALID; }
    if (rounds) *rounds = idx->h.dev_rounds;
    if (tied) *tied = idx->h.dev_tied;
    return BSQ_OK;
}

extern "C" int bsq_index_download(bsq_index *idx)
{
    if (!idx || !idx->h.built || !idx->h.dev) { set_err("index not on a device"); return BSQ_E_INVALID; }
    HostIndex &h = idx->h;
    if (!h.occ.empty() || h.seq_len == 0) return BSQ_OK;
    HIPCHK(hipSetDevice(h.dev->device));
    const IndexMeta m = meta_of(h);
    try {
        h.occ.resize(m.table_bytes[T_OCC] / sizeof(OccBlock));
        if (m.wide) h.sa64.resize(h.seq_len + 1); else h.sa32.resize(h.seq_len + 1);
    } catch (const std::bad_alloc &) {
        h.occ.clear(); h.sa32.clear(); h.sa64.clear();
        set_err("out of host memory"); return BSQ_E_NOMEM;
    }
    HIPCHK(hipMemcpy(h.occ.data(), h.dev->occ, m.table_bytes[T_OCC], hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(m.wide ? (void *)h.sa64.data() : (void *)h.sa32.data(), h.dev->sa, m.table_bytes[T_SA],
                     hipMemcpyDeviceToHost));
    return BSQ_OK;
}

extern "C" int bsq_index_layout(const bsq_index *idx, uint64_t *bytes, void *meta, uint64_t *meta_bytes)
{
    if (!idx || !idx->h.built || !meta_bytes) { set_err("index not built / invalid argument"); return BSQ_E_INVALID; }
    const HostIndex &h = idx->h;
    if (h.seq_len > 0 && h.occ.empty() && !h.dev_built) { set_err("device-only index (imported) has no host layout"); return BSQ_E_INVALID; }
    const IndexMeta m = meta_of(h);
    if (bytes) for (int t = 0; t < T_N; ++t) bytes[t] = m.table_bytes[t];
    const uint64_t need = sizeof(IndexMeta) + h.anns.size() * sizeof(Ann) + h.holes.size() * sizeof(Hole);
    if (meta) {
        if (*meta_bytes < need) { set_err("metadata buffer of %llu bytes, %llu needed", (unsigned long long)*meta_bytes,
                                          (unsigned long long)need); return BSQ_E_INVALID; }
        uint8_t *p = (uint8_t *)meta;
        memcpy(p, &m, sizeof m); p += sizeof m;
        if (!h.anns.empty()) { memcpy(p, h.anns.data(), h.anns.size() * sizeof(Ann)); p += h.anns.size() * sizeof(Ann); }
        if (!h.holes.empty()) memcpy(p, h.holes.data(), h.holes.size() * sizeof(Hole));
    }
    *meta_bytes = need;
    return BSQ_OK;
}

extern "C" int bsq_index_device_tables(const bsq_index *idx, int *device, bsq_table *tables, int n_tables)
{
    if (!idx || !idx->h.built || !idx->h.dev || !tables || n_tables != BSQ_N_TABLES) {
        set_err("index not on a device / invalid argument"); return BSQ_E_INVALID;
    }
    const DeviceIndex *d = idx->h.dev;
    const IndexMeta m = meta_of(idx->h);
    void *cur[T_N] = {d->occ, d->occ32, d->sa, d->pac, d->ann_off, d->ann_id, d->ann_len, d->kmer};
    for (int t = 0; t < T_N; ++t) tables[t] = bsq_table{m.table_bytes[t] ? cur[t] : nullptr, m.table_bytes[t]};
    if (device) *device = d->device;
    return BSQ_OK;
}

extern "C" int bsq_index_upload_into(bsq_index *idx, int device, const bsq_table *tables, int n_tables)
{
    if (!tables || n_tables != BSQ_N_TABLES) { set_err("expected %d tables", BSQ_N_TABLES); return BSQ_E_INVALID; }
    return upload_impl(idx, device, tables);
}

extern "C" int bsq_index_import(const void *meta, uint64_t meta_bytes, int device, const bsq_table *tables, int n_tables,
                                bsq_index **out)
{
    if (!meta || !out || !tables || n_tables != BSQ_N_TABLES || meta_bytes < sizeof(IndexMeta)) {
        set_err("invalid argument"); return BSQ_E_INVALID;
    }
    IndexMeta m;
    memcpy(&m, meta, sizeof m);
    if (memcmp(m.magic, "BSQIDX1", 8) != 0) { set_err("not an index metadata blob"); return BSQ_E_INVALID; }
    if (meta_bytes != sizeof m + m.n_anns * sizeof(Ann) + m.n_holes * sizeof(Hole)) { set_err("metadata size mismatch"); return BSQ_E_INVALID; }
    for (int t = 0; t < T_N; ++t)
        if (m.table_bytes[t] && (!tables[t].ptr || tables[t].bytes < m.table_bytes[t])) { set_err("table %d missing or short", t); return BSQ_E_INVALID; }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0) {
        set_err("no HIP device %d (found %d); the alignment path has no CPU fallback", device, ndev);
        return BSQ_E_NODEV;
    }
    HIPCHK(hipSetDevice(device));
    bsq_index *idx = new (std::nothrow) bsq_index();
    if (!idx) { set_err("out of memory"); return BSQ_E_NOMEM; }
    HostIndex &h = idx->h;
    const uint8_t *p = (const uint8_t *)meta + sizeof m;
    h.anns.resize(m.n_anns);
    if (m.n_anns) { memcpy(h.anns.data(), p, m.n_anns * sizeof(Ann)); p += m.n_anns * sizeof(Ann); }
    h.holes.resize(m.n_holes);
    if (m.n_holes) memcpy(h.holes.data(), p, m.n_holes * sizeof(Hole));
    h.l_pac = (int64_t)m.l_pac; h.seq_len = m.seq_len; h.primary = m.primary;
    for (int c = 0; c < 5; ++c) h.L2[c] = m.L2[c];
    h.pac.resize(m.pac_bytes);   // host copy for rendering (extract_reference_subseq)
    if (m.pac_bytes && hipMemcpy(h.pac.data(), tables[T_PAC].ptr, m.pac_bytes, hipMemcpyDeviceToHost) != hipSuccess) {
        delete idx; set_err("reading the broadcast pac"); return BSQ_E_HIP;
    }
    h.built = true;
    DeviceIndex *d = h.dev = new DeviceIndex();
    d->device = device;
    d->owned = false;
    d->occ = (OccBlock *)tables[T_OCC].ptr; d->occ32 = (OccBlock32 *)tables[T_OCC32].ptr; d->sa = tables[T_SA].ptr;
    d->pac = (uint8_t *)tables[T_PAC].ptr; d->ann_off = (int64_t *)tables[T_ANN_OFF].ptr;
    d->ann_id = (int64_t *)tables[T_ANN_ID].ptr; d->ann_len = (int32_t *)tables[T_ANN_LEN].ptr;
    d->kmer = (uint32_t *)tables[T_KMER].ptr;
    set_view(d, m);
    *out = idx;
    return BSQ_OK;
}

// ================================================================================================
// lrand48 (Q10): X_{k+1} = (0x5DEECE66D X_k + 0xB) mod 2^48 from X_0 = 0, value X >> 17
// ================================================================================================
static uint64_t lrand48_state_at(uint64_t calls)
{
    const uint64_t M = (1ULL << 48) - 1;
    uint64_t C = 0, a = 0x5DEECE66DULL, c = 0xB, e = calls;
    while (e) {
        if (e & 1) C = (a * C + c) & M;
        c = (a * c + c) & M;
        a = (a * a) & M;
        e >>= 1;
    }
    return C;
}
extern "C" int64_t bsq_lrand48_at(uint64_t pos) { return (int64_t)(lrand48_state_at(pos + 1) >> 17); }

// ids[i] = the lrand48 value of call first + i (read i of the batch), by jump-ahead per read
__global__ void k_lrand_ids(uint64_t first, int n, int64_t *ids)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t M = (1ULL << 48) - 1;
    uint64_t C = 0, a = 0x5DEECE66DULL, c = 0xB, e = first + (uint64_t)i + 1;
    while (e) {
        if (e & 1) C = (a * C + c) & M;
        c = (a * c + c) & M;
        a = (a * a) & M;
        e >>= 1;
    }
    ids[i] = (int64_t)(C >> 17);
}

// ================================================================================================
// batch workspace
// ================================================================================================
namespace {

constexpr int N_RETRY_LEVELS = 3;   // retry workspaces per batch (retry_caps)

struct Workspace {
    Caps cp{};
    int32_t max_reads = 0;
    int grid = 0;
    int64_t scratch_total = 0;
    uint32_t *status = nullptr;
    Intv *intv = nullptr;
    int32_t *n_intv = nullptr, *n_chains = nullptr, *n_regs = nullptr, *n_cig = nullptr;
    ChainDesc *chains = nullptr;
    Seed *seeds = nullptr;
    Reg *regs = nullptr;
    Hit *hits = nullptr;
    uint32_t *cigars = nullptr;
    uint8_t *scratch = nullptr;
    int32_t *sel = nullptr;   // local slot -> read (retry workspace only)
    int32_t *sscore = nullptr; // seed scores of mem_flt_chained_seeds (long-read workspaces only)
    uint8_t *zslab = nullptr; // per-wave traceback spill slabs of the wave reg2aln kernel
    int64_t zslab_bytes = 0;
    int zslab_blocks = 0;
    int32_t *dlist0 = nullptr, *dlist1 = nullptr, *dcount = nullptr;   // reads deferred by the group kernels
    uint8_t *lspill = nullptr;   // SMEM list entries beyond the LDS share (main pass), LSPILL per read
    uint8_t *codes_t = nullptr;  // wave-transposed read codes for the main-pass seeding kernel (reads <= 1024 bases)
    uint32_t *ekey0 = nullptr, *ekey1 = nullptr;   // extension work keys (main pass) and their sort
    int32_t *eidx0 = nullptr, *eidx1 = nullptr;
    void *esort_tmp = nullptr;
    size_t esort_bytes = 0;

    void release()
    {
        hipFree(status); hipFree(intv); hipFree(n_intv); hipFree(n_chains); hipFree(n_regs); hipFree(n_cig);
        hipFree(chains); hipFree(seeds); hipFree(regs); hipFree(hits); hipFree(cigars); hipFree(scratch); hipFree(sel);
        hipFree(sscore);
        hipFree(zslab); hipFree(dlist0); hipFree(dlist1); hipFree(dcount);
        hipFree(ekey0); hipFree(ekey1); hipFree(eidx0); hipFree(eidx1); hipFree(esort_tmp); hipFree(lspill); hipFree(codes_t);
        *this = Workspace{};
    }
};

// mem_flt_chained_seeds is active for a read of length l when !(5.5f*ln(l) > 0.05f*l) (bwamem.c), i.e.
// l >= ~700; a workspace for such lengths carries seed scores and runs k_flt_seeds
bool long_reads(int max_len)
{
    if (max_len < 2) return false;
    return !(5.5f * std::log((double)max_len) > (double)(0.05f * (float)max_len));
}

// k_extend's scratch per thread (align_kernels.hip k_extend: tmp regions, their index, seed sort keys, the
// global eh row of the non-LDS kernel, the introsort stack)
static int64_t ext_scratch_bytes(const Caps &c)
{
    const int64_t ext = (int64_t)c.regs * (int64_t)sizeof(Reg) + ((c.regs * 4 + 15) & ~15) + (int64_t)c.seeds * 8 +
                        (int64_t)(c.max_len + 2) * 8 + 192 * 4;
    return (ext + 255) & ~255LL;
}

int64_t scratch_bytes(const Caps &c, int64_t z_cap)
{
    int64_t smem = 3LL * (c.max_len + 2) * (int64_t)sizeof(Intv);
    // + the sort / tree-walk stacks kept in this scratch instead of private memory (align_kernels.hip)
    int64_t chain = (int64_t)c.seeds * 24 + (int64_t)c.chains * 40 + (int64_t)(c.chains / 2 + 8) * 84 + 2LL * c.chains * 4 +
                    (192 + 72) * 4;
    int64_t ext = ext_scratch_bytes(c);
    int64_t r2a = (((int64_t)(c.max_len + 2) * 8 + 63) & ~63LL) + z_cap;
    int64_t m = std::max(std::max(smem, chain), std::max(ext, r2a));
    return (m + 255) & ~255LL;
}

static const int LSPILL = 48;   // SMEM list entries per read beyond the LDS share

int ws_alloc(Workspace &w, const Caps &cp, int32_t max_reads, int workers, int64_t z_cap, bool with_sel)
{
    w.cp = cp;
    w.cp.scratch = scratch_bytes(cp, z_cap);
    w.cp.scr_ext = ext_scratch_bytes(cp);
    w.max_reads = max_reads;
    int threads = std::min<int64_t>(std::max(max_reads, 1), workers);
    w.grid = (threads + 255) / 256;
    const size_t R = (size_t)std::max(max_reads, 1);
    HIPCHK(hipMalloc(&w.status, R * 4));
    HIPCHK(hipMalloc(&w.intv, (size_t)intv_slot_reads((int64_t)R) * cp.intv * sizeof(Intv)));   // whole waves
    HIPCHK(hipMalloc(&w.n_intv, R * 4));
    HIPCHK(hipMalloc(&w.n_chains, R * 4));
    HIPCHK(hipMalloc(&w.n_regs, R * 4));
    HIPCHK(hipMalloc(&w.n_cig, R * 4));
    HIPCHK(hipMalloc(&w.chains, R * cp.chains * sizeof(ChainDesc)));
    HIPCHK(hipMalloc(&w.seeds, R * cp.seeds * sizeof(Seed)));
    HIPCHK(hipMalloc(&w.regs, R * cp.regs * sizeof(Reg)));
    HIPCHK(hipMalloc(&w.hits, R * cp.regs * sizeof(Hit)));
    HIPCHK(hipMalloc(&w.cigars, R * cp.regs * cp.cigar * 4));
    // Every stage kernel derives its scratch pointer from the thread id but dereferences it only inside
    // `for (li = tid; li < n; ...)`; a retry workspace runs n <= max_reads reads per launch, so only
    // max_reads threads ever touch scratch (the main pass may run more reads than threads: full grid).
    // The main pass's k_chain lays its state out per wave of 64 threads (the grid is whole blocks); the retry
    // kernels keep each thread's scratch contiguous (k_chain<1>), so a level-2 workspace of one read holds one
    // read's scratch, not a wave's.
    w.scratch_total = (with_sel ? (int64_t)std::max(max_reads, 1) : (int64_t)w.grid * 256) * w.cp.scratch;
    HIPCHK(hipMalloc(&w.scratch, (size_t)w.scratch_total));
    if (with_sel) HIPCHK(hipMalloc(&w.sel, R * 4));
    if (long_reads(cp.max_len)) HIPCHK(hipMalloc(&w.sscore, R * cp.seeds * 4));
    if (!with_sel) {
        // (bands of long reads that need more go to the retry pass, whose per-thread scratch holds 4 MB)
        w.zslab_bytes = std::min<int64_t>((int64_t)(2 * cp.max_len + 8) * (int64_t)(2 * cp.max_len + 64), 4 << 20);
        w.zslab_blocks = (int)std::min<int64_t>(((int64_t)R + 3) / 4, 3 * 256);
        HIPCHK(hipMalloc(&w.zslab, (size_t)w.zslab_blocks * 4 * (size_t)w.zslab_bytes));
        HIPCHK(hipMalloc(&w.dlist0, R * 4));
        HIPCHK(hipMalloc(&w.dlist1, R * 4));
        HIPCHK(hipMalloc(&w.dcount, 32));   // launch_reg2aln_chain's 5 counters, then k_extend's work counter
        HIPCHK(hipMalloc(&w.lspill, (size_t)intv_slot_reads((int64_t)R) * LSPILL * (2 * 8 + 4)));   // whole waves
        if (cp.max_len <= 1024) HIPCHK(hipMalloc(&w.codes_t, (size_t)intv_slot_reads((int64_t)R) * (size_t)cp.max_len));
        HIPCHK(hipMalloc(&w.ekey0, R * 4));
        HIPCHK(hipMalloc(&w.ekey1, R * 4));
        HIPCHK(hipMalloc(&w.eidx0, R * 4));
        HIPCHK(hipMalloc(&w.eidx1, R * 4));
        HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, w.esort_bytes, w.ekey0, w.ekey1, w.eidx0, w.eidx1, (int)R,
                                                  0, 30));   // the widest key sorted (the extension's, 30 bits)
        HIPCHK(hipMalloc(&w.esort_tmp, std::max<size_t>(w.esort_bytes, 16)));
    }
    return BSQ_OK;
}

DOpts make_dopts(const bsq_opts &o)
{
    DOpts d{};
    d.a = o.a; d.b = o.b; d.o_del = o.o_del; d.e_del = o.e_del; d.o_ins = o.o_ins; d.e_ins = o.e_ins;
    d.pen_clip5 = o.pen_clip5; d.pen_clip3 = o.pen_clip3; d.w = o.w; d.zdrop = o.zdrop;
    d.min_seed_len = o.min_seed_len; d.max_occ = o.max_occ;
    d.split_width = 10; d.max_chain_gap = 10000; d.min_chain_weight = 0; d.max_chain_extend = 1 << 30;
    d.max_mem_intv = 20; d.split_factor = 1.5f; d.mask_level = 0.50f; d.drop_ratio = 0.50f; d.mask_level_redun = 0.95f;
    // mem_opt_init fills mat with a=1, b=4 and bioseqdb never refills it (Q2)
    d.mat_match = 1; d.mat_mismatch = -4; d.mat_amb = -1; d.mat_max = 1;
    return d;
}

}  // namespace

struct bsq_batch {
    bsq_index *idx = nullptr;
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t cstream = nullptr;  // the nuclseq columns (high priority: created on first use)
    int32_t max_reads = 0;
    int64_t max_bases = 0;
    int32_t n_reads = 0;
    int32_t max_len = 0;
    uint8_t *codes = nullptr;
    int64_t *offs = nullptr;
    int64_t *ids = nullptr;
    std::vector<int64_t> h_offs;
    std::vector<uint8_t> h_codes;   // staging copy of set_reads' codes
    // bsq_batch_set_nuclseqs: packed varlenas and their offsets on the device (grown on demand)
    NsStage stage;                  // host staging of bsq_batch_set_nuclseqs
    uint8_t *ns_dev = nullptr;
    int64_t ns_dev_cap = 0;
    int64_t *ns_meta = nullptr;   // in_off | poff | holed texts
    int64_t ns_meta_cap = 0;
    Workspace main, retry[N_RETRY_LEVELS];
    Counters *ctr = nullptr;
    // packing
    int64_t *cnt_hits = nullptr, *cnt_cig = nullptr, *off_hits = nullptr, *off_cig = nullptr;
    unsigned long long *unresolved = nullptr;
    int32_t *ovf_list = nullptr, *ovf_count = nullptr;
    void *cub_tmp = nullptr;
    size_t cub_bytes = 0;
    bsq_hit *d_out = nullptr;
    uint32_t *d_out_cig = nullptr;
    int64_t out_cap = 0, out_cig_cap = 0;
    bsq_hit *h_pinned = nullptr;
    uint32_t *h_pinned_cig = nullptr;
    int64_t *h_pinned_off = nullptr;
    int64_t h_cap = 0, h_cig_cap = 0, h_off_cap = 0;
    // seeding-only runs (bsq_batch_seed): main-pass intervals stay in the workspace slots, reads that
    // needed the retry kernel keep theirs here; bsq_batch_intervals packs both on demand
    int32_t chunk = 0;   // reads per workspace pass; larger batches run in chunks [lo, lo + chunk)
    int32_t chunk0 = 0;  // the pass size for short reads (BSQ_CHUNK or 1M)
    int32_t lo = 0;      // first read of the chunk being run (stage kernels see offs + lo, ids + lo)
    bool seeded = false, seed_packed = false;
    std::vector<std::pair<int32_t, std::vector<uint64_t>>> seed_retry;
    std::vector<int64_t> seed_off;
    std::vector<uint64_t> seed_intv;
    uint64_t *d_intv = nullptr;
    int64_t d_intv_cap = 0;
    // results
    std::vector<bsq_hit> main_hits;  // main-pass results of a chunk that needed the retry pass
    std::vector<uint32_t> main_cig;
    std::vector<int64_t> main_off;
    std::vector<bsq_hit> res_hits;
    std::vector<uint32_t> res_cig;
    std::vector<int64_t> res_off;
    bsq_hits view{};
    // GPU rendering (bsq_batch_render): device copies of the records, row lengths/offsets, text
    bsq_hit *r_hits = nullptr; uint32_t *r_cig = nullptr; int64_t *r_len = nullptr; char *r_text = nullptr;
    int64_t r_hits_cap = 0, r_cig_cap = 0, r_len_cap = 0, r_text_cap = 0;
    char *r_host = nullptr; int64_t r_host_cap = 0;
    void *r_tmp = nullptr; size_t r_tmp_bytes = 0;
    RenderHole *r_qh = nullptr; int64_t r_qh_cap = 0;   // the reads' own hole symbols
    int64_t *r_qoff = nullptr; int64_t r_qoff_cap = 0;
    DevArena arena;                                     // encode scratch of the nuclseq columns
    uint8_t *c_host = nullptr; int64_t c_host_cap = 0;  // the columns' varlenas and offsets (pinned; borrowed out)
    int64_t *c_off = nullptr; int64_t c_off_cap = 0;
    hipEvent_t ev[STG_N + 1]{};
    float stage_ms[STG_N]{};
    double stage_bytes[STG_N]{};
    double stage_work[STG_N]{};
    int64_t sort_guard = 0;   // ks_introsort scans stopped by the bound over every run of this batch (must stay 0)
    int64_t retried = 0;
    bool dev_whole = false;   // d_out / d_out_cig hold the whole last run's view (one chunk, no retried read)
    // record route (bsq_batch_set_record_route): the packed records cross to relay_dev's HBM by peer DMA (xGMI between
    // devices) and reach the pinned view over that device's PCIe link instead of this device's own
    int relay_dev = -1;
    uint8_t *relay = nullptr;
    int64_t relay_cap = 0;
    hipStream_t relay_stream = nullptr;   // on relay_dev
    hipEvent_t relay_in = nullptr;        // on this device: the records are packed
    hipEvent_t relay_out = nullptr;       // on relay_dev: they are in host memory
};

static const char *kStageNames[STG_N] = {"smem", "chain", "extend", "reg2aln", "pack", "d2h"};
extern "C" const char *bsq_stage_name(int s) { return (s >= 0 && s < STG_N) ? kStageNames[s] : ""; }

static Caps main_caps(int max_len)
{
    Caps c{};
    if (tiny_caps()) {   // test knob: force most reads through the overflow -> retry path
        c.max_len = max_len; c.intv = 6; c.seeds = 8; c.chains = 2; c.regs = 1; c.cigar = 6;
        return c;
    }
    c.max_len = max_len;
    c.intv = 64 + max_len / 4;
    c.seeds = 256 + max_len;
    c.chains = 64;
    c.regs = 16;
    c.cigar = 40;
    return c;
}

// Retry levels: a read that overflows the main pass is re-run at level 0 (256 reads per launch); one that
// overflows that too (e.g. min_seed_len = 0 with a large max_occ expands thousands of SA hits per read) at
// level 1 and then level 2, each with ~8x the per-read capacities and 1/16 the reads per launch.  libbwa's
// own vectors are unbounded; only a read beyond level 2 fails (BSQ_E_UNSUPPORTED).
static int retry_chunk(int level) { return 256 >> (4 * level); }            // 256, 16, 1 reads
static int64_t retry_zcap(int level) { return (int64_t)(4 << 20) << (2 * level); }   // 4, 16, 64 MB traceback
static Caps retry_caps(int max_len, int level)
{
    Caps c{};
    const int f = 1 << (3 * level);
    c.max_len = max_len;
    c.intv = (4 * max_len + 64) * f;
    c.seeds = 32768 * f;
    c.chains = 32768 * f;
    c.regs = 2048 << (2 * level);
    c.cigar = (2 * max_len + 8) * (1 + level);
    return c;
}

static int device_workers(int device)
{
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, device) != hipSuccess) return 65536;
    return p.multiProcessorCount * 1024;
}

extern "C" int bsq_batch_create(bsq_index *idx, int32_t max_reads, int64_t max_bases, bsq_batch **out)
{
    if (!idx || !out || max_reads < 0 || max_bases < 0) { set_err("invalid argument"); return BSQ_E_INVALID; }
    if (!idx->h.dev) { set_err("index not uploaded to a device"); return BSQ_E_INVALID; }
    bsq_batch *b = new (std::nothrow) bsq_batch();
    if (!b) { set_err("out of memory"); return BSQ_E_NOMEM; }
    b->idx = idx;
    b->device = idx->h.dev->device;
    b->max_reads = max_reads;
    b->max_bases = max_bases;
    {   // workspace pass size (BSQ_CHUNK overrides; tests use it to exercise multi-chunk batches)
        const char *e = getenv("BSQ_CHUNK");
        const int c = e && atoi(e) > 0 ? atoi(e) : (1 << 20);
        b->chunk = b->chunk0 = std::max(1, std::min(std::max(max_reads, 1), c));
    }
    *out = b;
    HIPCHK(hipSetDevice(b->device));
    HIPCHK(hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking));
    for (auto &e : b->ev) HIPCHK(hipEventCreate(&e));
    const size_t R = (size_t)std::max(max_reads, 1);
    // whole 16-B words plus one: the reg2aln query stream loads the aligned word holding a read's last base
    // 32 bytes of padding past the last 16-base word: render_gpu.hip's codes16 loads 8 bytes from an aligned
    // address up to 12 bytes beyond a word's start, i.e. up to 19 bytes past the last base
    HIPCHK(hipMalloc(&b->codes, (size_t)((std::max<int64_t>(max_bases, 1) + 15) / 16 * 16 + 32)));
    HIPCHK(hipMalloc(&b->offs, (R + 1) * 8));
    HIPCHK(hipMalloc(&b->ids, R * 8));
    HIPCHK(hipMalloc(&b->ctr, sizeof(Counters) * STG_N));
    HIPCHK(hipMalloc(&b->cnt_hits, (R + 1) * 8));
    HIPCHK(hipMalloc(&b->cnt_cig, (R + 1) * 8));
    HIPCHK(hipMalloc(&b->off_hits, (R + 1) * 8));
    HIPCHK(hipMalloc(&b->off_cig, (R + 1) * 8));
    HIPCHK(hipMalloc(&b->unresolved, 8));
    HIPCHK(hipMalloc(&b->ovf_list, R * 4));
    HIPCHK(hipMalloc(&b->ovf_count, 4));
    size_t t1 = 0;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, t1, b->cnt_hits, b->off_hits, (int)(R + 1), b->stream));
    b->cub_bytes = t1;
    HIPCHK(hipMalloc(&b->cub_tmp, b->cub_bytes));
    return BSQ_OK;
}

extern "C" void bsq_batch_free(bsq_batch *b)
{
    if (!b) return;
    hipSetDevice(b->device);
    if (b->stream) hipStreamSynchronize(b->stream);
    b->main.release();
    for (auto &r : b->retry) r.release();
    hipFree(b->codes); hipFree(b->offs); hipFree(b->ids); hipFree(b->ctr);
    hipFree(b->cnt_hits); hipFree(b->cnt_cig); hipFree(b->off_hits); hipFree(b->off_cig); hipFree(b->unresolved);
    hipFree(b->ovf_list); hipFree(b->ovf_count); hipFree(b->cub_tmp); hipFree(b->d_out); hipFree(b->d_out_cig);
    hipHostFree(b->h_pinned); hipHostFree(b->h_pinned_cig); hipHostFree(b->h_pinned_off); hipFree(b->d_intv);
    hipFree(b->r_hits); hipFree(b->r_cig); hipFree(b->r_len); hipFree(b->r_text); hipFree(b->r_tmp); hipHostFree(b->r_host);
    hipFree(b->r_qh); hipFree(b->r_qoff); hipHostFree(b->c_host); hipHostFree(b->c_off);
    hipFree(b->ns_dev); hipFree(b->ns_meta);
    for (auto &e : b->ev) if (e) hipEventDestroy(e);
    if (b->relay_in) hipEventDestroy(b->relay_in);
    if (b->relay_dev >= 0) {
        hipSetDevice(b->relay_dev);
        if (b->relay_stream) { hipStreamSynchronize(b->relay_stream); hipStreamDestroy(b->relay_stream); }
        if (b->relay_out) hipEventDestroy(b->relay_out);
        hipFree(b->relay);
        hipSetDevice(b->device);
    }
    if (b->stream) hipStreamDestroy(b->stream);
    if (b->cstream && b->cstream != b->stream) { hipStreamSynchronize(b->cstream); hipStreamDestroy(b->cstream); }
    delete b;
}

static int prepare_workspace(bsq_batch *b, int max_len);

extern "C" int bsq_batch_set_reads(bsq_batch *b, const uint8_t *codes, const int64_t *offsets, int32_t n_reads)
{
    if (!b || (n_reads > 0 && (!codes || !offsets)) || n_reads < 0) { set_err("invalid argument"); return BSQ_E_INVALID; }
    if (n_reads > b->max_reads) { set_err("batch holds at most %d reads", b->max_reads); return BSQ_E_INVALID; }
    int64_t total = n_reads ? offsets[n_reads] - offsets[0] : 0;
    if (total > b->max_bases) { set_err("batch holds at most %lld bases", (long long)b->max_bases); return BSQ_E_INVALID; }
    HIPCHK(hipSetDevice(b->device));
    b->h_offs.assign(offsets, offsets + n_reads + 1);
    int max_len = 0;
    for (int i = 0; i < n_reads; ++i) {
        int64_t l = offsets[i + 1] - offsets[i];
        if (l < 0) { set_err("negative read length at %d", i); return BSQ_E_INVALID; }
        max_len = std::max<int64_t>(max_len, l);
    }
    const int64_t base0 = n_reads ? offsets[0] : 0;
    for (auto &o : b->h_offs) o -= base0;
    b->h_codes.assign(codes + base0, codes + base0 + total);
    b->n_reads = n_reads;
    b->max_len = max_len;
    if (n_reads) {
        HIPCHK(hipMemcpyAsync(b->codes, b->h_codes.data(), (size_t)total, hipMemcpyHostToDevice, b->stream));
        HIPCHK(hipMemcpyAsync(b->offs, b->h_offs.data(), (size_t)(n_reads + 1) * 8, hipMemcpyHostToDevice, b->stream));
    }
    { const int rc = prepare_workspace(b, max_len); if (rc) return rc; }
    HIPCHK(hipStreamSynchronize(b->stream));
    return BSQ_OK;
}

// (re)allocate the main workspace for this read length; the per-read slots grow with the length, so
// long reads run in proportionally smaller workspace passes (~ the bytes of 1M x 150 bp)
static int prepare_workspace(bsq_batch *b, int max_len)
{
    const int32_t want = max_len > 150 ? std::max<int32_t>(1, std::min<int64_t>(b->chunk0, (int64_t)b->chunk0 * 150 / max_len))
                                       : b->chunk0;
    // (a workspace lent by a pipeline's pool may hold more reads than this batch's pass: it is used as it is)
    if (!b->main.status || b->main.cp.max_len < max_len || tiny_caps() != (b->main.cp.regs == 1) || b->main.max_reads < want) {
        b->main.release();
        // per-thread scratch: the main pass's reg2aln keeps its traceback in LDS and the zslab unless reads are
        // longer than 1024 bases (then the serial kernel's 32 KB traceback area is needed)
        int rc = ws_alloc(b->main, main_caps(std::max(max_len, 1)), want, device_workers(b->device),
                          max_len > 1024 ? 32 * 1024 : 0, false);
        if (rc) return rc;
    }
    b->chunk = want;
    return BSQ_OK;
}

template <typename T>
static int grow_dev(T *&p, int64_t &cap, int64_t need);

// Reads given as nuclseq varlenas (the cursor's detoasted values): the varlenas are
// packed and uploaded as they are and turned into nt4 codes on the device (codec_gpu.hip, the same
// pass as nuclseq_out with hole bases as code 4), instead of a per-read host conversion.  The host half
// (stage_nuclseqs) and the device half (batch_upload_staged) are separate so a pipeline can release a fetch's
// tuples as soon as it is staged and upload it later from a worker thread (pipeline.cpp).
namespace bsq {

NsStage::~NsStage() { if (host) hipHostFree(host); }

void set_error(const std::string &msg) { g_err = msg; }
int32_t batch_max_reads(const bsq_batch *b) { return b->max_reads; }
int64_t batch_max_bases(const bsq_batch *b) { return b->max_bases; }

int stage_nuclseqs(NsStage &s, const void *const *reads, int32_t n_reads)
{
    if (n_reads < 0 || (n_reads && !reads)) { set_err("invalid argument"); return BSQ_E_INVALID; }
    // invalid until this staging succeeds: a RERUN of a failed staging must not find the old read count
    s.n = -1;
    s.host_bytes = 0;
    const size_t n = (size_t)n_reads;
    // Two passes over contiguous ranges of the reads, on up to 8 host threads for a large fetch (a cursor
    // fetch of 256k reads is ~13 MB of varlenas): sizes and offsets, then the copy into pinned memory.  A pipeline
    // stages its deferred fetches one at a time in submission order (pipeline.cpp prep_job).
    const int T = n >= 65536 ? (int)std::max<unsigned>(1, std::min<unsigned>(8, std::thread::hardware_concurrency())) : 1;
    std::vector<size_t> lo((size_t)T + 1);
    for (int t = 0; t <= T; ++t) lo[(size_t)t] = n * (size_t)t / (size_t)T;
    s.meta.assign(2 * (n + 1), 0);   // in_off | poff, then the holed reads
    s.offs.assign(n + 1, 0);
    int64_t *in_off = s.meta.data(), *poff = s.meta.data() + n + 1, *boff = s.offs.data();
    struct Part { int64_t in = 0, pac = 0, bases = 0; int max_len = 0; std::vector<int64_t> holed;
                  size_t bad = SIZE_MAX; int kind = 0; uint64_t vl = 0, need = 0; };
    std::vector<Part> part((size_t)T);
    auto pass1 = [&](int t) {   // per-read sizes at [i] (a range's thread alone touches [lo, hi))
        Part &q = part[(size_t)t];
        for (size_t i = lo[(size_t)t]; i < lo[(size_t)t + 1]; ++i) {
            const uint8_t *ns = static_cast<const uint8_t *>(reads[i]);
            if (!ns) { q.bad = i; q.kind = 1; return; }
            uint32_t vl; memcpy(&vl, ns, 4);
            const uint64_t nh = ns_holes_num(ns), len = ns_len(ns), need = 12 + 16 * nh + pac_byte_size(len);
            if ((vl >> 2) < need) { q.bad = i; q.kind = 2; q.vl = vl >> 2; q.need = need; return; }
            if (nh) q.holed.push_back((int64_t)i);
            in_off[i] = (int64_t)((need + 7) & ~7ull);
            poff[i] = (int64_t)pac_byte_size(len);
            boff[i] = (int64_t)len;
            q.in += in_off[i];
            q.pac += poff[i];
            q.bases += (int64_t)len;
            q.max_len = std::max<int>(q.max_len, (int)len);
        }
    };
    auto run = [&](auto f) {
        std::vector<std::thread> th;
        for (int t = 1; t < T; ++t) th.emplace_back(f, t);
        f(0);
        for (auto &x : th) x.join();
    };
    run(pass1);
    for (const Part &q : part)
        if (q.bad != SIZE_MAX) {
            if (q.kind == 1) set_err("read %zu is NULL", q.bad);
            else set_err("read %zu: varlena of %llu bytes, %llu needed", q.bad, (unsigned long long)q.vl,
                         (unsigned long long)q.need);
            return BSQ_E_INVALID;
        }
    std::vector<int64_t> base_in((size_t)T + 1, 0), base_pac((size_t)T + 1, 0), base_b((size_t)T + 1, 0);
    int max_len = 0;
    for (int t = 0; t < T; ++t) {
        base_in[(size_t)t + 1] = base_in[(size_t)t] + part[(size_t)t].in;
        base_pac[(size_t)t + 1] = base_pac[(size_t)t] + part[(size_t)t].pac;
        base_b[(size_t)t + 1] = base_b[(size_t)t] + part[(size_t)t].bases;
        max_len = std::max(max_len, part[(size_t)t].max_len);
    }
    const int64_t bytes = base_in[(size_t)T];
    // the pinned buffer also holds copies of meta and offs after the varlenas: the upload copies all three from
    // pinned memory (pageable sources go through the HIP runtime's staging buffer, one copy at a time per process,
    // which serialised the uploads of concurrent pipeline slots: DESIGN.md §3b round 5)
    size_t n_holed = 0;
    for (const Part &q : part) n_holed += q.holed.size();
    const int64_t meta_at = (bytes + 15) & ~15ll, offs_at = meta_at + 8 * (int64_t)(2 * (n + 1) + n_holed);
    const int64_t need = offs_at + 8 * (int64_t)(n + 1);
    if (need > s.host_cap) {
        if (s.host) hipHostFree(s.host);
        s.host = nullptr;
        s.host_cap = 0;
        const int64_t cap = std::max<int64_t>(need + need / 4, 4096);
        if (hipHostMalloc((void **)&s.host, (size_t)cap) != hipSuccess) { s.host = nullptr; set_err("out of pinned host memory"); return BSQ_E_NOMEM; }
        s.host_cap = cap;
    }
    auto pass2 = [&](int t) {   // sizes -> offsets within the range, then the copy
        int64_t a = base_in[(size_t)t], c = base_pac[(size_t)t], d = base_b[(size_t)t];
        for (size_t i = lo[(size_t)t]; i < lo[(size_t)t + 1]; ++i) {
            const uint8_t *ns = static_cast<const uint8_t *>(reads[i]);
            const int64_t ni = in_off[i], pi = poff[i], bi = boff[i];
            in_off[i] = a; poff[i] = c; boff[i] = d;
            memcpy(s.host + a, ns, 12 + 16 * (size_t)ns_holes_num(ns) + (size_t)pi);
            a += ni; c += pi; d += bi;
        }
    };
    run(pass2);
    in_off[n] = bytes;
    poff[n] = base_pac[(size_t)T];
    boff[n] = base_b[(size_t)T];
    for (const Part &q : part) s.meta.insert(s.meta.end(), q.holed.begin(), q.holed.end());
    {   // pinned copies of meta and offs (by range on the staging threads)
        int64_t *pm = reinterpret_cast<int64_t *>(s.host + meta_at), *po = reinterpret_cast<int64_t *>(s.host + offs_at);
        const size_t nm = s.meta.size(), no = n + 1;
        run([&](int t) {
            const size_t a = nm * (size_t)t / (size_t)T, b = nm * (size_t)(t + 1) / (size_t)T;
            memcpy(pm + a, s.meta.data() + a, (b - a) * 8);
            const size_t c = no * (size_t)t / (size_t)T, d = no * (size_t)(t + 1) / (size_t)T;
            memcpy(po + c, s.offs.data() + c, (d - c) * 8);
        });
    }
    s.meta_at = meta_at;
    s.offs_at = offs_at;
    s.n = n_reads;
    s.max_len = max_len;
    s.bases = boff[n];
    s.host_bytes = bytes;
    return BSQ_OK;
}

int batch_upload_staged(bsq_batch *b, const NsStage &s, bool with_workspace)
{
    if (s.n > b->max_reads) { set_err("batch holds at most %d reads", b->max_reads); return BSQ_E_INVALID; }
    if (s.bases > b->max_bases) { set_err("batch holds at most %lld bases", (long long)b->max_bases); return BSQ_E_INVALID; }
    HIPCHK(hipSetDevice(b->device));
    const size_t n = (size_t)s.n;
    { const int rc = grow_dev(b->ns_dev, b->ns_dev_cap, std::max<int64_t>(s.host_bytes, 1)); if (rc) return rc; }
    { const int rc = grow_dev(b->ns_meta, b->ns_meta_cap, (int64_t)s.meta.size()); if (rc) return rc; }
    b->h_offs = s.offs;
    b->n_reads = s.n;
    b->max_len = s.max_len;
    hipStream_t st = b->stream;
    if (n) {
        HIPCHK(hipMemcpyAsync(b->ns_dev, s.host, (size_t)s.host_bytes, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(b->ns_meta, s.host + s.meta_at, s.meta.size() * 8, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(b->offs, s.host + s.offs_at, (n + 1) * 8, hipMemcpyHostToDevice, st));
        const DecView v{b->ns_dev, b->ns_meta, b->ns_meta + n + 1, b->offs, (int64_t)n, s.meta[2 * n + 1]};
        HIPCHK(launch_dec_codes(st, v, b->ns_meta + 2 * (n + 1), (int64_t)(s.meta.size() - 2 * (n + 1)), b->codes));
    }
    if (with_workspace) { const int rc = prepare_workspace(b, s.max_len); if (rc) return rc; }
    HIPCHK(hipStreamSynchronize(st));   // the staged buffers may be reused when this returns
    return BSQ_OK;
}

// A batch's workspaces (the main pass's and the retry levels') as a unit a pipeline lends to the batch whose
// alignment turn it is: up to run_cap alignments run at once, so a pipeline of 16 fetches needs run_cap sets of
// ~8.5 GB (262,144-read passes), not 16 (pipeline.cpp).
struct WsSet {
    Workspace main, retry[N_RETRY_LEVELS];
};

WsSet *batch_detach_workspaces(bsq_batch *b)
{
    hipSetDevice(b->device);
    hipStreamSynchronize(b->stream);   // nothing on the batch's stream may still use them
    WsSet *w = new (std::nothrow) WsSet();
    if (!w) return nullptr;
    std::swap(w->main, b->main);
    for (int i = 0; i < N_RETRY_LEVELS; ++i) std::swap(w->retry[i], b->retry[i]);
    return w;
}

bool batch_has_workspace(const bsq_batch *b) { return b->main.status != nullptr; }

void batch_attach_workspaces(bsq_batch *b, WsSet *w)
{
    if (!w) return;
    hipSetDevice(b->device);
    b->main.release();
    for (auto &r : b->retry) r.release();
    std::swap(w->main, b->main);
    for (int i = 0; i < N_RETRY_LEVELS; ++i) std::swap(w->retry[i], b->retry[i]);
    delete w;
}

void workspaces_free(WsSet *w)
{
    if (!w) return;
    w->main.release();
    for (auto &r : w->retry) r.release();
    delete w;
}

int batch_prepare_workspace(bsq_batch *b)
{
    HIPCHK(hipSetDevice(b->device));
    return prepare_workspace(b, std::max(b->max_len, 1));
}

}  // namespace bsq

extern "C" int bsq_batch_set_nuclseqs(bsq_batch *b, const void *const *reads, int32_t n_reads)
{
    if (!b || n_reads < 0 || (n_reads && !reads)) { set_err("invalid argument"); return BSQ_E_INVALID; }
    if (n_reads > b->max_reads) { set_err("batch holds at most %d reads", b->max_reads); return BSQ_E_INVALID; }
    { const int rc = stage_nuclseqs(b->stage, reads, n_reads); if (rc) return rc; }
    return batch_upload_staged(b, b->stage, true);
}


// Runs smem -> chain -> extend -> reg2aln on workspace w for n local reads.
// Seeding (mem_collect_intv) on workspace w: the main-pass LDS kernel, or the large-capacity kernel for
// the retry pass (sel != nullptr).
static int seed_stage(bsq_batch *b, Workspace &w, const DOpts &o, int n, const int32_t *sel)
{
    const DIndex &ix = b->idx->h.dev->view;
    hipStream_t st = b->stream;
    if (!sel && w.cp.max_len < 65536) {
        // main pass: LDS-resident SMEM lists (smem.hip); overflowing reads fall through to the retry pass
        // u32 rows: 15 entries in LDS = 9.6 KB per one-wave block, 16 waves per CU; longer lists spill.
        // 64-bit rows: 148 VGPRs allow 12 waves per CU.  With u32 interval sizes (l_pac < 2^32: 14-B entries)
        // 14 entries fill 12.5 KB per block at 12 waves (C4 seeding per 1M reads: 25.3 ms against 26.2 at 13,
        // 27.3 at 12); all-u64 entries (18 B) measured best at 12 (28.2 ms against 29.1 at 16 entries / 8 waves,
        // 29.0 at 11, 30.4 at 10).  BSQ_TEST_LCAP shrinks the LDS share so the spill path is tested
        // (tests/test_gpu_parity.py).
        const int lcap_env = getenv("BSQ_TEST_LCAP") ? atoi(getenv("BSQ_TEST_LCAP")) : 0;
        const int lcap = tiny_caps() ? 3 : lcap_env > 0 ? lcap_env : !ix.wide ? 15 : wide_z32(ix) ? 14 : 12;
        HIPCHK(launch_smem_lds(st, ix, o, w.cp, b->codes, (b->offs + b->lo), n, w.intv, w.n_intv, w.status, b->ctr, lcap,
                               w.lspill, tiny_caps() ? 0 : LSPILL, w.codes_t));
    } else {
        HIPCHK(launch_smem(w.grid, st, ix, o, w.cp, b->codes, (b->offs + b->lo), sel, n, w.intv, w.n_intv, w.status, w.scratch, b->ctr));
    }
    return BSQ_OK;
}

static int run_stages(bsq_batch *b, Workspace &w, const DOpts &o, int n, const int32_t *sel, bool timed)
{
    const DIndex &ix = b->idx->h.dev->view;
    hipStream_t st = b->stream;
    HIPCHK(hipMemsetAsync(w.status, 0, (size_t)std::max(n, 1) * 4, st));
    if (timed) HIPCHK(hipEventRecord(b->ev[STG_SMEM], st));
    Range rg("smem");
    { const int rc = seed_stage(b, w, o, n, sel); if (rc) return rc; }
    if (timed) HIPCHK(hipEventRecord(b->ev[STG_CHAIN], st));
    rg.next("chain");
    HIPCHK(launch_chain(w.grid, st, ix, o, w.cp, (b->offs + b->lo), sel, n, w.intv, w.n_intv, w.chains, w.seeds, w.n_chains, w.status,
                        w.scratch, b->ctr));
    if (w.sscore)   // long reads: mem_flt_chained_seeds (per read; shorter reads of the batch keep score = len)
        HIPCHK(launch_flt_seeds(w.grid, st, ix, o, w.cp, b->codes, (b->offs + b->lo), sel, n, w.chains, w.seeds,
                                w.n_chains, w.status, w.sscore, w.scratch, b->ctr));
    if (timed) HIPCHK(hipEventRecord(b->ev[STG_EXTEND], st));
    rg.next("extend");
    const int32_t *order = nullptr;
    if (!sel && w.ekey0 && n > 0) {
        // lane balance: run the extension in order of estimated DP work so each wave holds similar reads
        HIPCHK(launch_ext_key(st, w.cp, (b->offs + b->lo), sel, n, w.chains, w.seeds, w.n_chains, w.status, w.sscore,
                              w.ekey0, w.eidx0));
        size_t tb = w.esort_bytes;
        HIPCHK(hipcub::DeviceRadixSort::SortPairs(w.esort_tmp, tb, w.ekey0, w.ekey1, w.eidx0, w.eidx1, n, 0, 30, st));
        order = w.eidx1;
    }
    HIPCHK(launch_extend(w.grid, st, ix, o, w.cp, b->codes, (b->offs + b->lo), sel, (b->ids + b->lo), n, w.chains, w.seeds, w.n_chains, w.regs,
                         w.n_regs, w.status, w.scratch, b->ctr, order, w.sscore,
                         w.dcount && !ext_static() ? w.dcount + 5 : nullptr));
    if (timed) HIPCHK(hipEventRecord(b->ev[STG_REG2ALN], st));
    rg.next("reg2aln");
    if (!sel && w.cp.max_len <= 1024) {
        // main pass: one wave per read, DP rows across lanes, eh + traceback in LDS (dp_wave.hip)
        const size_t eh_bytes = ((size_t)(w.cp.max_len + 2) * 8 + 15) & ~(size_t)15;
        const int64_t q_bytes = ((int64_t)w.cp.max_len + 16) & ~15LL;
        const int zcap = (int)std::max<int64_t>(4096, (int64_t)(150 * 1024 / 12) - (int64_t)eh_bytes - q_bytes) & ~15;
        // persistent waves (3 blocks of 4 waves per CU); each owns a global traceback slab for big bands
        // The diagonal pass takes the reads in batch order and routes each one it does not decide to the kernel of its
        // widest first band.  (Ordering the pass by that band class first -- a key kernel and a 3-bit sort -- measured
        // level: C3 step 56.7 / 56.3 / 57.2 M against 56.7 / 56.4 / 57.5 M without; profiles/r06/r2a_order/.)
        HIPCHK(launch_reg2aln_chain(st, ix, o, w.cp, b->codes, (b->offs + b->lo), n, w.regs, w.n_regs, w.hits, w.cigars, w.n_cig,
                                    w.status, b->ctr, tiny_caps() ? 64 : zcap, w.zslab, w.zslab_bytes, w.zslab_blocks,
                                    w.dlist0, w.dlist1, w.dcount, nullptr, nullptr,
                                    w.eidx0 && !no_r2a_diag() ? w.eidx0 : nullptr));
        if (getenv("BSQ_R2A_COUNTS")) {   // diagnostics: reads handed on by each reg2aln kernel (host sync)
            int32_t dc[4] = {0, 0, 0, 0};
            HIPCHK(hipMemcpyAsync(dc, w.dcount, sizeof dc, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            fprintf(stderr, "bsq_r2a reads %d: to g16 %d, to g32 %d, to w %d\n", n, dc[3], dc[0], dc[1]);
        }
    } else {
        HIPCHK(launch_reg2aln(w.grid, st, ix, o, w.cp, b->codes, (b->offs + b->lo), sel, n, w.regs, w.n_regs, w.hits, w.cigars,
                              w.n_cig, w.status, w.scratch, b->ctr));
    }
    if (timed) HIPCHK(hipEventRecord(b->ev[STG_PACK], st));
    return BSQ_OK;
}

// Packs workspace w (n local reads) into host vectors hits/cig/off (hits with read_index = local).
static int pack_device(bsq_batch *b, Workspace &w, int n, bool allow_unresolved, int read_base, int64_t cig_base,
                       int64_t tot[2])
{
    hipStream_t st = b->stream;
    SlotView v{w.hits, w.cigars, w.n_regs, w.n_cig, w.cp};
    HIPCHK(hipMemsetAsync(b->unresolved, 0, 8, st));
    HIPCHK(hipMemsetAsync(b->cnt_hits + n, 0, 8, st));
    HIPCHK(hipMemsetAsync(b->cnt_cig + n, 0, 8, st));
    if (n) HIPCHK(launch_counts(st, n, v, v, nullptr, w.status, b->cnt_hits, b->cnt_cig, b->unresolved));
    size_t tb = b->cub_bytes;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(b->cub_tmp, tb, b->cnt_hits, b->off_hits, n + 1, st));
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(b->cub_tmp, tb, b->cnt_cig, b->off_cig, n + 1, st));
    unsigned long long unres = 0;
    HIPCHK(hipMemcpyAsync(&tot[0], b->off_hits + n, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(&tot[1], b->off_cig + n, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(&unres, b->unresolved, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (unres && !allow_unresolved) { set_err("%llu reads exceeded even the retry capacities", unres); return BSQ_E_UNSUPPORTED; }
    if (tot[0] > b->out_cap) {
        hipFree(b->d_out);
        b->out_cap = std::max<int64_t>(tot[0], 2 * b->out_cap);
        HIPCHK(hipMalloc(&b->d_out, (size_t)b->out_cap * sizeof(bsq_hit)));
    }
    if (tot[1] > b->out_cig_cap) {
        hipFree(b->d_out_cig);
        b->out_cig_cap = std::max<int64_t>(tot[1], 2 * b->out_cig_cap);
        HIPCHK(hipMalloc(&b->d_out_cig, (size_t)b->out_cig_cap * 4));
    }
    const DeviceIndex *d = b->idx->h.dev;
    if (n && tot[0])
        HIPCHK(launch_pack(st, n, v, v, nullptr, b->off_hits, b->off_cig, d->ann_off, d->ann_id, b->d_out, b->d_out_cig,
                           read_base, cig_base));
    return BSQ_OK;
}

// grows a pinned array to hold `need` elements, keeping the first `keep`
template <typename T>
static int grow_pinned(T *&p, int64_t &cap, int64_t need, int64_t keep)
{
    if (need <= cap) return BSQ_OK;
    const int64_t nc = std::max<int64_t>(need, 2 * cap);
    T *q = nullptr;
    HIPCHK(hipHostMalloc((void **)&q, (size_t)nc * sizeof(T)));
    if (keep > 0) memcpy(q, p, (size_t)keep * sizeof(T));
    hipHostFree(p);
    p = q;
    cap = nc;
    return BSQ_OK;
}

// The relayed record route: read offsets, hits and CIGARs of the packed chunk by peer DMA into relay_dev's HBM
// (one buffer, 256-B aligned parts), then D2H from there on relay_dev's stream into the same pinned arrays the
// direct route fills; the batch stream waits for the D2H, so the stage events and the view are unchanged.
static int relay_records(bsq_batch *b, int n, int lo, int64_t hit_dst, int64_t cig_dst, const int64_t tot[2])
{
    hipStream_t st = b->stream;
    auto al = [](int64_t x) { return (x + 255) & ~(int64_t)255; };
    const int64_t o_off = 0, o_hit = al((int64_t)(n + 1) * 8), o_cig = o_hit + al(tot[0] * (int64_t)sizeof(bsq_hit));
    const int64_t need = o_cig + al(tot[1] * 4);
    if (need > b->relay_cap) {
        HIPCHK(hipSetDevice(b->relay_dev));
        hipStreamSynchronize(b->relay_stream);
        hipFree(b->relay);
        b->relay = nullptr;
        b->relay_cap = 0;
        const int64_t cap = std::max<int64_t>(need + need / 4, 1 << 20);
        const hipError_t e = hipMalloc(&b->relay, (size_t)cap);
        hipSetDevice(b->device);
        if (e != hipSuccess) { set_err("relay buffer on device %d: %s", b->relay_dev, hipGetErrorString(e)); return BSQ_E_NOMEM; }
        b->relay_cap = cap;
    }
    uint8_t *r = b->relay;
    HIPCHK(hipMemcpyPeerAsync(r + o_off, b->relay_dev, b->off_hits, b->device, (size_t)(n + 1) * 8, st));
    if (tot[0]) HIPCHK(hipMemcpyPeerAsync(r + o_hit, b->relay_dev, b->d_out, b->device, (size_t)tot[0] * sizeof(bsq_hit), st));
    if (tot[1]) HIPCHK(hipMemcpyPeerAsync(r + o_cig, b->relay_dev, b->d_out_cig, b->device, (size_t)tot[1] * 4, st));
    HIPCHK(hipEventRecord(b->relay_in, st));
    HIPCHK(hipSetDevice(b->relay_dev));
    hipStream_t rs = b->relay_stream;
    hipError_t e = hipStreamWaitEvent(rs, b->relay_in, 0);
    if (e == hipSuccess) e = hipMemcpyAsync(b->h_pinned_off + lo, r + o_off, (size_t)(n + 1) * 8, hipMemcpyDeviceToHost, rs);
    if (e == hipSuccess && tot[0])
        e = hipMemcpyAsync(b->h_pinned + hit_dst, r + o_hit, (size_t)tot[0] * sizeof(bsq_hit), hipMemcpyDeviceToHost, rs);
    if (e == hipSuccess && tot[1])
        e = hipMemcpyAsync(b->h_pinned_cig + cig_dst, r + o_cig, (size_t)tot[1] * 4, hipMemcpyDeviceToHost, rs);
    if (e == hipSuccess) e = hipEventRecord(b->relay_out, rs);
    hipSetDevice(b->device);
    if (e != hipSuccess) { set_err("record relay: %s", hipGetErrorString(e)); return BSQ_E_HIP; }
    HIPCHK(hipStreamWaitEvent(st, b->relay_out, 0));
    return BSQ_OK;
}

extern "C" int bsq_batch_set_record_route(bsq_batch *b, int via_device)
{
    if (!b || via_device < -1) { set_err("invalid argument"); return BSQ_E_INVALID; }
    if (via_device == b->relay_dev) return BSQ_OK;
    int ndev = 0;
    if (via_device >= 0 && (hipGetDeviceCount(&ndev) != hipSuccess || via_device >= ndev)) {
        set_err("no HIP device %d", via_device);
        return BSQ_E_NODEV;
    }
    HIPCHK(hipSetDevice(b->device));
    HIPCHK(hipStreamSynchronize(b->stream));
    if (b->relay_dev >= 0) {   // drop the previous route's buffers
        hipSetDevice(b->relay_dev);
        hipStreamSynchronize(b->relay_stream);
        hipStreamDestroy(b->relay_stream);
        hipEventDestroy(b->relay_out);
        hipFree(b->relay);
        hipSetDevice(b->device);
        hipEventDestroy(b->relay_in);
        b->relay_stream = nullptr; b->relay_out = nullptr; b->relay = nullptr; b->relay_in = nullptr;
        b->relay_cap = 0;
        b->relay_dev = -1;
    }
    if (via_device < 0) return BSQ_OK;
    if (via_device != b->device) {   // peer DMA over xGMI (already enabled is fine)
        const hipError_t e = hipDeviceEnablePeerAccess(via_device, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) { set_err("peer access %d -> %d: %s", b->device, via_device, hipGetErrorString(e)); return BSQ_E_HIP; }
        (void)hipGetLastError();
    }
    HIPCHK(hipEventCreateWithFlags(&b->relay_in, hipEventDisableTiming));
    HIPCHK(hipSetDevice(via_device));
    hipError_t e = hipStreamCreateWithFlags(&b->relay_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&b->relay_out, hipEventDisableTiming);
    hipSetDevice(b->device);
    if (e != hipSuccess) { set_err("relay stream: %s", hipGetErrorString(e)); return BSQ_E_HIP; }
    b->relay_dev = via_device;
    return BSQ_OK;
}

// Main-pass chunk [lo, lo + n): records land in the batch-wide pinned arrays at hit_dst / cig_dst with
// batch-wide read indices and CIGAR offsets, read_off[lo .. lo + n] = batch-wide hit offsets.
static int pack_main(bsq_batch *b, Workspace &w, int n, int lo, int64_t hit_dst, int64_t cig_dst, int64_t tot[2])
{
    Range rg("pack+d2h");
    hipStream_t st = b->stream;
    { const int rc = pack_device(b, w, n, true, lo, cig_dst, tot); if (rc) return rc; }
    { int rc = grow_pinned(b->h_pinned, b->h_cap, hit_dst + tot[0], hit_dst); if (rc) return rc; }
    { int rc = grow_pinned(b->h_pinned_cig, b->h_cig_cap, cig_dst + tot[1], cig_dst); if (rc) return rc; }
    { int rc = grow_pinned(b->h_pinned_off, b->h_off_cap, (int64_t)b->n_reads + 1, lo); if (rc) return rc; }
    HIPCHK(launch_add_base(st, b->off_hits, n + 1, hit_dst));
    HIPCHK(hipEventRecord(b->ev[STG_D2H], st));
    if (b->relay_dev >= 0) {
        const int rc = relay_records(b, n, lo, hit_dst, cig_dst, tot);
        if (rc) return rc;
    } else {
        HIPCHK(hipMemcpyAsync(b->h_pinned_off + lo, b->off_hits, (size_t)(n + 1) * 8, hipMemcpyDeviceToHost, st));
        if (tot[0]) HIPCHK(hipMemcpyAsync(b->h_pinned + hit_dst, b->d_out, (size_t)tot[0] * sizeof(bsq_hit), hipMemcpyDeviceToHost, st));
        if (tot[1]) HIPCHK(hipMemcpyAsync(b->h_pinned_cig + cig_dst, b->d_out_cig, (size_t)tot[1] * 4, hipMemcpyDeviceToHost, st));
    }
    HIPCHK(hipEventRecord(b->ev[STG_N], st));
    HIPCHK(hipStreamSynchronize(st));
    return BSQ_OK;
}

// Retry-pass chunk: records (chunk-local indices) into host vectors.
static int pack_retry(bsq_batch *b, Workspace &w, int n, std::vector<bsq_hit> &hits, std::vector<uint32_t> &cig,
                      std::vector<int64_t> &off, bool last_level)
{
    hipStream_t st = b->stream;
    int64_t tot[2];
    { const int rc = pack_device(b, w, n, !last_level, 0, 0, tot); if (rc) return rc; }
    off.resize((size_t)n + 1);
    hits.resize((size_t)tot[0]);
    cig.resize((size_t)tot[1]);
    HIPCHK(hipMemcpyAsync(off.data(), b->off_hits, (size_t)(n + 1) * 8, hipMemcpyDeviceToHost, st));
    if (tot[0]) HIPCHK(hipMemcpyAsync(hits.data(), b->d_out, (size_t)tot[0] * sizeof(bsq_hit), hipMemcpyDeviceToHost, st));
    if (tot[1]) HIPCHK(hipMemcpyAsync(cig.data(), b->d_out_cig, (size_t)tot[1] * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return BSQ_OK;
}

// The retry workspace of `level`, (re)allocated for the batch's longest read.
static int ensure_retry(bsq_batch *b, int level)
{
    Workspace &r = b->retry[level];
    if (r.status && r.cp.max_len >= b->max_len) return BSQ_OK;
    r.release();
    const int ch = retry_chunk(level);
    return ws_alloc(r, retry_caps(std::max(b->max_len, 1), level), ch, ch, retry_zcap(level), true);
}

// One workspace pass over reads [b->lo, b->lo + n): main pass, packing into the batch-wide pinned arrays
// at (*hit_total, *cig_total), and the large-capacity retry for overflowing reads, merged in place.
static int run_chunk(bsq_batch *b, const DOpts &o, int n, int64_t &hit_total, int64_t &cig_total)
{
    hipStream_t st = b->stream;
    const int lo = b->lo;
    int rc = run_stages(b, b->main, o, n, nullptr, true);
    if (rc) return rc;
    // overflowing reads -> retry workspace with large capacities
    HIPCHK(hipMemsetAsync(b->ovf_count, 0, 4, st));
    HIPCHK(launch_collect_overflow(st, n, b->main.status, b->ovf_list, b->ovf_count));
    int32_t novf = 0;
    HIPCHK(hipMemcpyAsync(&novf, b->ovf_count, 4, hipMemcpyDeviceToHost, st));
    int64_t tot[2];
    rc = pack_main(b, b->main, n, lo, hit_total, cig_total, tot);
    if (rc) return rc;
    for (int s = 0; s < STG_N; ++s) {   // per-chunk device time (main pass), summed over chunks
        float ms = 0;
        hipEventElapsedTime(&ms, b->ev[s], b->ev[s + 1]);
        b->stage_ms[s] += ms;
    }
    if (novf == 0) { hit_total += tot[0]; cig_total += tot[1]; return BSQ_OK; }

    // chunk-local copy of the main results (the retry pass re-runs the pack machinery)
    b->retried += novf;
    b->main_off.resize((size_t)n + 1);
    for (int r = 0; r <= n; ++r) b->main_off[r] = b->h_pinned_off[lo + r] - hit_total;
    b->main_hits.assign(b->h_pinned + hit_total, b->h_pinned + hit_total + tot[0]);
    for (auto &x : b->main_hits) { x.read_index -= lo; x.cigar_off -= (uint32_t)cig_total; }
    b->main_cig.assign(b->h_pinned_cig + cig_total, b->h_pinned_cig + cig_total + tot[1]);
    std::vector<int32_t> list((size_t)novf);
    HIPCHK(hipMemcpy(list.data(), b->ovf_list, (size_t)novf * 4, hipMemcpyDeviceToHost));
    std::sort(list.begin(), list.end());
    // per-read replacement results, escalating through the retry levels
    std::vector<std::vector<bsq_hit>> rh((size_t)novf);
    std::vector<std::vector<uint32_t>> rcg((size_t)novf);
    std::vector<int32_t> pend((size_t)novf);   // positions in `list` still unresolved
    for (int k = 0; k < novf; ++k) pend[(size_t)k] = k;
    for (int level = 0; level < N_RETRY_LEVELS && !pend.empty(); ++level) {
        rc = ensure_retry(b, level);
        if (rc) return rc;
        Workspace &W = b->retry[level];
        const int CH = retry_chunk(level);
        const bool last = level + 1 == N_RETRY_LEVELS;
        std::vector<int32_t> next, sel((size_t)CH);
        std::vector<uint32_t> stt((size_t)CH);
        for (size_t s = 0; s < pend.size(); s += (size_t)CH) {
            const int m = (int)std::min<size_t>((size_t)CH, pend.size() - s);
            for (int j = 0; j < m; ++j) sel[(size_t)j] = list[(size_t)pend[s + (size_t)j]];
            HIPCHK(hipMemcpyAsync(W.sel, sel.data(), (size_t)m * 4, hipMemcpyHostToDevice, st));
            rc = run_stages(b, W, o, m, W.sel, false);
            if (rc) return rc;
            std::vector<bsq_hit> hh; std::vector<uint32_t> cc; std::vector<int64_t> oo;
            rc = pack_retry(b, W, m, hh, cc, oo, last);
            if (rc) return rc;
            HIPCHK(hipMemcpy(stt.data(), W.status, (size_t)m * 4, hipMemcpyDeviceToHost));
            for (int j = 0; j < m; ++j) {
                const int32_t li = pend[s + (size_t)j];
                if (stt[(size_t)j] & ST_OVERFLOW) { next.push_back(li); continue; }
                auto &dst = rh[(size_t)li];
                auto &dc = rcg[(size_t)li];
                for (int64_t k = oo[j]; k < oo[j + 1]; ++k) {
                    bsq_hit x = hh[(size_t)k];
                    uint32_t base = (uint32_t)dc.size();
                    dc.insert(dc.end(), cc.begin() + x.cigar_off, cc.begin() + x.cigar_off + x.n_cigar);
                    x.cigar_off = base;
                    dst.push_back(x);
                }
            }
        }
        pend.swap(next);
    }
    // merge into read order (chunk-local): bulk copies of the runs of main-pass reads between retried ones
    std::vector<bsq_hit> &mh = b->res_hits;
    std::vector<uint32_t> &mc = b->res_cig;
    std::vector<int64_t> &mo = b->res_off;
    mh.clear(); mc.clear(); mo.assign((size_t)n + 1, 0);
    const std::vector<int64_t> &MO = b->main_off;
    auto copy_run = [&](int r0, int r1) {   // main-pass reads [r0, r1)
        if (r0 >= r1) return;
        const int64_t h0 = MO[r0], h1 = MO[r1], hb = (int64_t)mh.size();
        for (int r = r0; r < r1; ++r) mo[r] = hb + (MO[r] - h0);
        if (h1 == h0) return;
        const uint32_t c0 = b->main_hits[h0].cigar_off;
        const uint32_t c1 = b->main_hits[h1 - 1].cigar_off + b->main_hits[h1 - 1].n_cigar;
        const uint32_t cb = (uint32_t)mc.size();
        mh.insert(mh.end(), b->main_hits.begin() + h0, b->main_hits.begin() + h1);
        for (int64_t k = hb; k < (int64_t)mh.size(); ++k) mh[k].cigar_off = mh[k].cigar_off - c0 + cb;
        mc.insert(mc.end(), b->main_cig.begin() + c0, b->main_cig.begin() + c1);
    };
    int prev = 0;
    for (size_t li = 0; li < list.size(); ++li) {
        const int r = list[li];
        copy_run(prev, r);
        mo[r] = (int64_t)mh.size();
        for (auto x : rh[li]) {
            uint32_t base = (uint32_t)mc.size();
            mc.insert(mc.end(), rcg[li].begin() + x.cigar_off, rcg[li].begin() + x.cigar_off + x.n_cigar);
            x.cigar_off = base; x.read_index = r;
            mh.push_back(x);
        }
        prev = r + 1;
    }
    copy_run(prev, n);
    mo[n] = (int64_t)mh.size();
    // write the merged chunk back into the batch-wide pinned arrays
    { int rc2 = grow_pinned(b->h_pinned, b->h_cap, hit_total + (int64_t)mh.size(), hit_total); if (rc2) return rc2; }
    { int rc2 = grow_pinned(b->h_pinned_cig, b->h_cig_cap, cig_total + (int64_t)mc.size(), cig_total); if (rc2) return rc2; }
    for (size_t k = 0; k < mh.size(); ++k) {
        bsq_hit x = mh[k];
        x.read_index += lo;
        x.cigar_off += (uint32_t)cig_total;
        b->h_pinned[hit_total + (int64_t)k] = x;
    }
    if (!mc.empty()) memcpy(b->h_pinned_cig + cig_total, mc.data(), mc.size() * 4);
    for (int r = 0; r <= n; ++r) b->h_pinned_off[lo + r] = hit_total + mo[r];
    hit_total += (int64_t)mh.size();
    cig_total += (int64_t)mc.size();
    return BSQ_OK;
}

extern "C" int bsq_batch_run(bsq_batch *b, const bsq_opts *opts, uint64_t first_call_seq)
{
    Range rg("bsq_batch_run");
    if (!b || !opts) { set_err("invalid argument"); return BSQ_E_INVALID; }
    if (opts->e_del <= 0 || opts->e_ins <= 0 || opts->max_occ <= 0 || opts->min_seed_len < 0) {
        set_err("gap extension penalties and max_occ must be positive, min_seed_len nonnegative");
        return BSQ_E_INVALID;
    }
    HIPCHK(hipSetDevice(b->device));
    b->dev_whole = false;   // set again only when this run completes with the whole view in d_out
    const int n = b->n_reads;
    const DOpts o = make_dopts(*opts);
    hipStream_t st = b->stream;
    // a batch whose workspaces a pipeline took back (pipeline.cpp: a group's held shares re-run by
    // bsq_batch_run_rounds) gets its own again; a no-op when they fit
    if (n > 0) { const int rc = prepare_workspace(b, std::max(b->max_len, 1)); if (rc) return rc; }
    // lrand48 ids: read i consumes call first_call_seq + i (computed on the device)
    if (n) hipLaunchKernelGGL(k_lrand_ids, dim3((n + 255) / 256), dim3(256), 0, st, (uint64_t)first_call_seq, n, b->ids);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemsetAsync(b->ctr, 0, sizeof(Counters) * STG_N, st));
    b->retried = 0;
    int rc = BSQ_OK;
    for (int s = 0; s < STG_N; ++s) b->stage_ms[s] = 0;
    { const int rc2 = grow_pinned(b->h_pinned_off, b->h_off_cap, (int64_t)n + 1, 0); if (rc2) return rc2; }
    int64_t hit_total = 0, cig_total = 0;
    if (n > 0 && b->idx->h.seq_len > 0) {
        // workspace-sized chunks; every chunk's records land in place in the batch-wide pinned arrays
        for (int lo = 0; lo < n; lo += b->chunk) {
            const int m = std::min(b->chunk, n - lo);
            b->lo = lo;
            rc = run_chunk(b, o, m, hit_total, cig_total);
            b->lo = 0;
            if (rc) return rc;
            if (cig_total > (int64_t)UINT32_MAX) {   // bsq_hit.cigar_off is u32: offsets would wrap
                set_err("batch holds more than 2^32 CIGAR operations; split it into smaller batches");
                return BSQ_E_UNSUPPORTED;
            }
        }
        // algorithmic bytes (stage times were summed over the chunks)
        Counters c[STG_N];
        HIPCHK(hipMemcpy(c, b->ctr, sizeof c, hipMemcpyDeviceToHost));
        b->stage_bytes[STG_SMEM] =
            32.0 * c[STG_SMEM].occ_blocks + 16.0 * c[STG_SMEM].kmer_hits + (double)b->h_offs[n] / 4.0 * 1.0;
        b->stage_bytes[STG_CHAIN] = 8.0 * c[STG_CHAIN].sa_values;
        b->stage_bytes[STG_EXTEND] = (double)c[STG_EXTEND].ref_bases;
        b->stage_bytes[STG_REG2ALN] = (double)c[STG_REG2ALN].ref_bases;
        b->stage_bytes[STG_PACK] = (double)hit_total * sizeof(bsq_hit) + 4.0 * (double)cig_total;
        b->stage_bytes[STG_D2H] = b->stage_bytes[STG_PACK];
        for (int s = 0; s < STG_N; ++s) b->stage_work[s] = (double)c[s].dp_cells;
        b->stage_work[STG_SMEM] = (double)c[STG_SMEM].kmer_hits + (double)c[STG_SMEM].occ_blocks / 2.0;
        {
            const int64_t g = (int64_t)(c[STG_CHAIN].sort_guard + c[STG_EXTEND].sort_guard);
            b->sort_guard += g;
            if (g) g_sort_guard.fetch_add(g);
        }
    } else {
        for (int s = 0; s < STG_N; ++s) { b->stage_ms[s] = 0; b->stage_bytes[s] = 0; b->stage_work[s] = 0; }
    }
    // the results stay in the batch-wide pinned arrays (zero-copy view, valid until the next run)
    if (n == 0 || b->idx->h.seq_len == 0) for (int r = 0; r <= n; ++r) b->h_pinned_off[r] = 0;
    b->dev_whole = n > 0 && b->chunk >= n && b->retried == 0 && b->idx->h.seq_len > 0;
    b->view.n_reads = n;
    b->view.n_hits = hit_total;
    b->view.hits = b->h_pinned;
    b->view.read_off = b->h_pinned_off;
    b->view.n_cigar = cig_total;
    b->view.cigar = b->h_pinned_cig;
    return BSQ_OK;
}

// ================================================================================================
// Seeding only (BASELINE.json configs[1]): libbwa mem_collect_intv for every read of the batch
// ================================================================================================
// Seeding pass over reads [b->lo, b->lo + n) of the main workspace; reads that overflow get the large-capacity
// kernel and keep their intervals in b->seed_retry (read index local to the chunk).
static int seed_chunk(bsq_batch *b, const DOpts &o, int n)
{
    hipStream_t st = b->stream;
    Workspace &w = b->main;
    b->seed_retry.clear();
    HIPCHK(hipMemsetAsync(w.status, 0, (size_t)n * 4, st));
    HIPCHK(hipEventRecord(b->ev[STG_SMEM], st));
    { const int rc = seed_stage(b, w, o, n, nullptr); if (rc) return rc; }
    HIPCHK(hipEventRecord(b->ev[STG_CHAIN], st));
    HIPCHK(hipMemsetAsync(b->ovf_count, 0, 4, st));
    HIPCHK(launch_collect_overflow(st, n, w.status, b->ovf_list, b->ovf_count));
    int32_t novf = 0;
    HIPCHK(hipMemcpyAsync(&novf, b->ovf_count, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (novf > 0) {   // large-capacity seeding for the reads whose lists or slots overflowed
        b->retried += novf;
        std::vector<int32_t> list((size_t)novf);
        HIPCHK(hipMemcpy(list.data(), b->ovf_list, (size_t)novf * 4, hipMemcpyDeviceToHost));
        std::sort(list.begin(), list.end());
        std::vector<int32_t> pend = list;
        for (int level = 0; level < N_RETRY_LEVELS && !pend.empty(); ++level) {
            { const int rc = ensure_retry(b, level); if (rc) return rc; }
            Workspace &r = b->retry[level];
            const int CH = retry_chunk(level);
            std::vector<int32_t> cnt((size_t)CH), next;
            std::vector<uint32_t> stt((size_t)CH);
            std::vector<Intv> slots((size_t)intv_slot_reads(CH) * r.cp.intv);
            for (size_t s0 = 0; s0 < pend.size(); s0 += (size_t)CH) {
                const int m = (int)std::min<size_t>((size_t)CH, pend.size() - s0);
                HIPCHK(hipMemcpyAsync(r.sel, pend.data() + s0, (size_t)m * 4, hipMemcpyHostToDevice, st));
                HIPCHK(hipMemsetAsync(r.status, 0, (size_t)m * 4, st));
                { const int rc = seed_stage(b, r, o, m, r.sel); if (rc) return rc; }
                HIPCHK(hipMemcpyAsync(cnt.data(), r.n_intv, (size_t)m * 4, hipMemcpyDeviceToHost, st));
                HIPCHK(hipMemcpyAsync(stt.data(), r.status, (size_t)m * 4, hipMemcpyDeviceToHost, st));
                HIPCHK(hipMemcpyAsync(slots.data(), r.intv, (size_t)intv_slot_reads(m) * r.cp.intv * sizeof(Intv),
                                      hipMemcpyDeviceToHost, st));
                HIPCHK(hipStreamSynchronize(st));
                for (int j = 0; j < m; ++j) {
                    if (stt[(size_t)j]) {
                        if (level + 1 < N_RETRY_LEVELS) { next.push_back(pend[s0 + (size_t)j]); continue; }
                        set_err("read %d exceeded even the retry seeding capacities", b->lo + pend[s0 + (size_t)j]);
                        return BSQ_E_UNSUPPORTED;
                    }
                    std::vector<uint64_t> v((size_t)cnt[(size_t)j] * 4);
                    for (int k = 0; k < cnt[(size_t)j]; ++k) {
                        const Intv &x = slots[(size_t)intv_slot_at(j, k, r.cp.intv)];
                        v[4 * k] = x.x[0]; v[4 * k + 1] = x.x[1]; v[4 * k + 2] = x.x[2]; v[4 * k + 3] = x.info;
                    }
                    b->seed_retry.emplace_back(pend[s0 + (size_t)j], std::move(v));
                }
            }
            pend.swap(next);
        }
        // pack_seed_chunk merges seed_retry with the main slots in read order
        std::sort(b->seed_retry.begin(), b->seed_retry.end(),
                  [](const std::pair<int32_t, std::vector<uint64_t>> &x, const std::pair<int32_t, std::vector<uint64_t>> &y) {
                      return x.first < y.first;
                  });
    }
    float ms = 0;
    hipEventElapsedTime(&ms, b->ev[STG_SMEM], b->ev[STG_CHAIN]);
    b->stage_ms[STG_SMEM] += ms;
    return BSQ_OK;
}

// Appends the intervals of the chunk just seeded (n reads, main slots + b->seed_retry) to seed_off /
// seed_intv, which hold the previous chunks.
static int pack_seed_chunk(bsq_batch *b, int n)
{
    hipStream_t st = b->stream;
    Workspace &w = b->main;
    HIPCHK(launch_intv_counts(st, n, w.n_intv, w.status, b->cnt_hits));
    size_t tb = b->cub_bytes;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(b->cub_tmp, tb, b->cnt_hits, b->off_hits, n + 1, st));
    std::vector<int64_t> off((size_t)n + 1);
    HIPCHK(hipMemcpyAsync(off.data(), b->off_hits, (size_t)(n + 1) * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const int64_t tot = off[n];
    if (tot > b->d_intv_cap) {
        hipFree(b->d_intv);
        b->d_intv_cap = std::max<int64_t>(tot, 1);
        HIPCHK(hipMalloc(&b->d_intv, (size_t)b->d_intv_cap * 32));
    }
    std::vector<uint64_t> packed((size_t)tot * 4);
    HIPCHK(launch_intv_pack(st, n, w.cp.intv, w.intv, w.n_intv, w.status, b->off_hits, b->d_intv));
    if (tot) HIPCHK(hipMemcpyAsync(packed.data(), b->d_intv, (size_t)tot * 32, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    size_t ri = 0;
    for (int li = 0; li < n; ++li) {
        b->seed_off.push_back((int64_t)(b->seed_intv.size() / 4));
        if (ri < b->seed_retry.size() && b->seed_retry[ri].first == li) {
            const auto &v = b->seed_retry[ri++].second;
            b->seed_intv.insert(b->seed_intv.end(), v.begin(), v.end());
        } else {
            b->seed_intv.insert(b->seed_intv.end(), packed.begin() + 4 * off[li], packed.begin() + 4 * off[li + 1]);
        }
    }
    return BSQ_OK;
}

extern "C" int bsq_batch_seed(bsq_batch *b, const bsq_opts *opts)
{
    Range rg("bsq_batch_seed");
    if (!b || !opts) { set_err("invalid argument"); return BSQ_E_INVALID; }
    if (opts->max_occ <= 0 || opts->min_seed_len < 0) {
        set_err("max_occ must be positive, min_seed_len nonnegative");
        return BSQ_E_INVALID;
    }
    HIPCHK(hipSetDevice(b->device));
    b->dev_whole = false;   // the seeding run reuses d_out's workspace: the records there are stale
    const int n = b->n_reads;
    const DOpts o = make_dopts(*opts);
    b->seeded = false;
    b->seed_packed = false;
    b->seed_retry.clear();
    b->seed_off.clear();
    b->seed_intv.clear();
    b->retried = 0;
    // a batch whose workspaces a pipeline took back (pipeline.cpp) gets its own again
    if (n > 0) { const int rc = prepare_workspace(b, std::max(b->max_len, 1)); if (rc) return rc; }
    HIPCHK(hipMemsetAsync(b->ctr, 0, sizeof(Counters) * STG_N, b->stream));
    for (int s = 0; s < STG_N; ++s) { b->stage_ms[s] = 0; b->stage_bytes[s] = 0; b->stage_work[s] = 0; }
    if (n > 0 && b->idx->h.seq_len > 0) {
        if (n <= b->chunk) {   // intervals stay in the workspace until bsq_batch_intervals
            b->lo = 0;
            const int rc = seed_chunk(b, o, n);
            if (rc) return rc;
        } else {               // the workspace is reused per chunk: pack each chunk's intervals as it finishes
            for (int lo = 0; lo < n; lo += b->chunk) {
                const int m = std::min(b->chunk, n - lo);
                b->lo = lo;
                int rc = seed_chunk(b, o, m);
                if (!rc) rc = pack_seed_chunk(b, m);
                b->lo = 0;
                if (rc) return rc;
            }
            b->seed_off.push_back((int64_t)(b->seed_intv.size() / 4));
            b->seed_packed = true;
        }
        Counters c[STG_N];
        HIPCHK(hipMemcpy(c, b->ctr, sizeof c, hipMemcpyDeviceToHost));
        b->stage_bytes[STG_SMEM] =
            32.0 * c[STG_SMEM].occ_blocks + 16.0 * c[STG_SMEM].kmer_hits + (double)b->h_offs[n] / 4.0 * 1.0;
        b->stage_work[STG_SMEM] = (double)c[STG_SMEM].kmer_hits + (double)c[STG_SMEM].occ_blocks / 2.0;
    }
    b->seeded = true;
    return BSQ_OK;
}

extern "C" int bsq_batch_intervals(bsq_batch *b, const int64_t **read_off, const uint64_t **intv, int64_t *n_intv)
{
    if (!b || !read_off || !intv || !n_intv) { set_err("invalid argument"); return BSQ_E_INVALID; }
    if (!b->seeded) { set_err("no seeding run on this batch (call bsq_batch_seed)"); return BSQ_E_INVALID; }
    HIPCHK(hipSetDevice(b->device));
    const int n = b->n_reads;
    if (!b->seed_packed) {
        b->seed_off.clear();
        b->seed_intv.clear();
        if (n > 0 && b->idx->h.seq_len > 0) {
            const int rc = pack_seed_chunk(b, n);
            if (rc) return rc;
        } else b->seed_off.assign((size_t)n, 0);
        b->seed_off.push_back((int64_t)(b->seed_intv.size() / 4));
        b->seed_packed = true;
    }
    *read_off = b->seed_off.data();
    *intv = b->seed_intv.data();
    *n_intv = b->seed_off[n];
    return BSQ_OK;
}

// The last run's records as one byte range in device memory (hits, then CIGAR words) -- the exchange step's
// send buffer of a sharded job (bench.py --gpus N): straight from the packed device arrays when they hold the
// whole view (one chunk, no retried read), else from the pinned host view.  dst == nullptr: size query.
extern "C" int bsq_batch_copy_records(const bsq_batch *b, void *dst, int64_t cap, int64_t *bytes)
{
    if (!b || !bytes) { set_err("invalid argument"); return BSQ_E_INVALID; }
    const int64_t nh = b->view.n_hits * (int64_t)sizeof(bsq_hit), nc = b->view.n_cigar * 4;
    *bytes = nh + nc;
    if (!dst || nh + nc == 0) return BSQ_OK;
    if (cap < nh + nc) { set_err("destination holds %lld bytes, records need %lld", (long long)cap, (long long)(nh + nc)); return BSQ_E_INVALID; }
    HIPCHK(hipSetDevice(b->device));
    const hipMemcpyKind k = b->dev_whole ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    const void *sh = b->dev_whole ? (const void *)b->d_out : (const void *)b->view.hits;
    const void *sc = b->dev_whole ? (const void *)b->d_out_cig : (const void *)b->view.cigar;
    uint8_t *d = static_cast<uint8_t *>(dst);
    if (nh) HIPCHK(hipMemcpyAsync(d, sh, (size_t)nh, k, b->stream));
    if (nc) HIPCHK(hipMemcpyAsync(d + nh, sc, (size_t)nc, k, b->stream));
    HIPCHK(hipStreamSynchronize(b->stream));
    return BSQ_OK;
}

extern "C" const bsq_hits *bsq_batch_hits(const bsq_batch *b) { return b ? &b->view : nullptr; }

namespace bsq {
BatchRecords batch_records(const bsq_batch *b)
{
    BatchRecords r;
    r.device = b->device;
    r.stream = b->stream;
    r.on_device = b->dev_whole;
    r.n_reads = b->view.n_reads;
    r.n_hits = b->view.n_hits;
    r.n_cigar = b->view.n_cigar;
    if (b->dev_whole) { r.off = b->off_hits; r.hits = b->d_out; r.cig = b->d_out_cig; }
    else { r.off = b->view.read_off; r.hits = b->view.hits; r.cig = b->view.cigar; }
    return r;
}
}  // namespace bsq

// Several batches in flight at once, one host thread and one stream each: the stages of one batch fill
// the tails and host gaps of the others (3 batches of 1/3 of the reads: +24 % reads/s at C3 on one
// MI355X, whose process gets 4 hardware queues).  first_call[i] is batch i's lrand48 position.
extern "C" int bsq_batch_run_rounds(bsq_batch *const *batches, int n, const bsq_opts *opts, const uint64_t *first_call,
                                    int rounds)
{
    if (n < 0 || rounds < 0 || (n > 0 && (!batches || !opts || !first_call))) { set_err("invalid argument"); return BSQ_E_INVALID; }
    std::vector<int> rc((size_t)n, BSQ_OK);
    std::vector<std::string> msg((size_t)n);
    auto one = [&](int i) {
        for (int r = 0; r < rounds && !rc[(size_t)i]; ++r) rc[(size_t)i] = bsq_batch_run(batches[i], opts, first_call[i]);
        if (rc[(size_t)i]) msg[(size_t)i] = g_err;   // the message is thread-local: carry it to the caller
    };
    std::vector<std::thread> th;
    for (int i = 1; i < n; ++i) th.emplace_back(one, i);
    if (n > 0) one(0);
    for (auto &t : th) t.join();
    for (int i = 0; i < n; ++i)
        if (rc[(size_t)i]) { g_err = "batch " + std::to_string(i) + ": " + msg[(size_t)i]; return rc[(size_t)i]; }
    return BSQ_OK;
}

extern "C" int bsq_batch_run_many(bsq_batch *const *batches, int n, const bsq_opts *opts, const uint64_t *first_call)
{
    return bsq_batch_run_rounds(batches, n, opts, first_call, 1);
}

// device buffer of at least `need` elements (contents not kept)
template <typename T>
static int grow_dev(T *&p, int64_t &cap, int64_t need)
{
    if (need <= cap) return BSQ_OK;
    hipFree(p);
    p = nullptr;
    cap = std::max<int64_t>(need, cap + cap / 2);
    HIPCHK(hipMalloc((void **)&p, (size_t)std::max<int64_t>(cap, 1) * sizeof(T)));
    return BSQ_OK;
}

// The reference's hole overlay as disjoint segments (bsq_index.h HoleIndex, shared with the host renderer), in
// HBM of the index's device: uploaded on first use, kept with the index.
static int index_render_holes(bsq_index *idx, const RenderHole **d, int64_t *n)
{
    std::lock_guard<std::mutex> lk(idx->rh_mu);
    if (idx->n_rh < 0) {
        std::vector<RenderHole> rh;
        for (const HoleRef &x : idx->holes().segs) rh.push_back(RenderHole{x.beg, x.end, x.order, (uint8_t)x.amb});
        if (!rh.empty()) {
            HIPCHK(hipMalloc(&idx->d_rh, rh.size() * sizeof(RenderHole)));
            HIPCHK(hipMemcpy(idx->d_rh, rh.data(), rh.size() * sizeof(RenderHole), hipMemcpyHostToDevice));
        }
        idx->n_rh = (int64_t)rh.size();
    }
    *d = static_cast<const RenderHole *>(idx->d_rh);
    *n = idx->n_rh;
    return BSQ_OK;
}

// Device inputs of the GPU renderers: the last run's records (still in HBM when the run was one chunk without
// retried reads, else uploaded from the host view), the reference holes, the reads' own holes.  Every buffer is
// the batch's or the index's (grow-only): nothing is allocated or freed in a steady loop.
static int render_inputs(bsq_batch *b, const void *const *reads, RenderView &v, hipStream_t st)
{
    const bsq_hits &H = b->view;
    const HostIndex &h = b->idx->h;
    const bsq_hit *dh = b->d_out;
    const uint32_t *dc = b->d_out_cig;
    if (!b->dev_whole) {
        { int rc = grow_dev(b->r_hits, b->r_hits_cap, H.n_hits); if (rc) return rc; }
        { int rc = grow_dev(b->r_cig, b->r_cig_cap, std::max<int64_t>(H.n_cigar, 1)); if (rc) return rc; }
        HIPCHK(hipMemcpyAsync(b->r_hits, H.hits, (size_t)H.n_hits * sizeof(bsq_hit), hipMemcpyHostToDevice, st));
        if (H.n_cigar) HIPCHK(hipMemcpyAsync(b->r_cig, H.cigar, (size_t)H.n_cigar * 4, hipMemcpyHostToDevice, st));
        dh = b->r_hits;
        dc = b->r_cig;
    }
    { int rc = grow_dev(b->r_len, b->r_len_cap, H.n_hits + 1); if (rc) return rc; }
    const RenderHole *d_rh = nullptr;
    int64_t n_rh = 0;
    { const int rc = index_render_holes(b->idx, &d_rh, &n_rh); if (rc) return rc; }
    // the reads' own hole symbols (nuclseq varlenas); without them, ambiguous bases print as N
    std::vector<int64_t> qoff;
    std::vector<RenderHole> qh;
    if (reads) {
        qoff.assign((size_t)H.n_reads + 1, 0);
        for (int32_t r = 0; r < H.n_reads; ++r) {
            const uint8_t *ns = static_cast<const uint8_t *>(reads[r]);
            const uint32_t nh = ns ? ns_holes_num(ns) : 0;
            for (uint32_t i = 0; i < nh; ++i) {
                const Hole x = ns_hole(ns, i);
                qh.push_back(RenderHole{x.offset, x.offset + x.len, i, (uint8_t)x.amb});
            }
            qoff[(size_t)r + 1] = (int64_t)qh.size();
        }
        if (qh.empty()) qoff.clear();
    }
    const RenderHole *d_qh = nullptr;
    const int64_t *d_qoff = nullptr;
    if (!qoff.empty()) {
        { int rc = grow_dev(b->r_qh, b->r_qh_cap, (int64_t)qh.size()); if (rc) return rc; }
        { int rc = grow_dev(b->r_qoff, b->r_qoff_cap, (int64_t)qoff.size()); if (rc) return rc; }
        HIPCHK(hipMemcpyAsync(b->r_qh, qh.data(), qh.size() * sizeof(RenderHole), hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(b->r_qoff, qoff.data(), qoff.size() * 8, hipMemcpyHostToDevice, st));
        HIPCHK(hipStreamSynchronize(st));   // the host vectors go out of scope
        d_qh = b->r_qh;
        d_qoff = b->r_qoff;
    }
    v = RenderView{dh, dc, H.n_hits, h.dev->pac, h.l_pac, d_rh, n_rh, b->codes, b->offs, d_qoff, d_qh};
    return BSQ_OK;
}

extern "C" int bsq_batch_render(bsq_batch *b, const void *const *reads, const char **text, int64_t *len)
{
    if (!b || !text || !len) { set_err("invalid argument"); return BSQ_E_INVALID; }
    *text = ""; *len = 0;
    const bsq_hits &H = b->view;
    if (H.n_hits <= 0) return BSQ_OK;
    HIPCHK(hipSetDevice(b->device));
    hipStream_t st = b->stream;
    RenderView v{};
    { const int rc = render_inputs(b, reads, v, st); if (rc) return rc; }
    HIPCHK(launch_row_len(st, v, b->r_len));
    HIPCHK(hipMemsetAsync(b->r_len + H.n_hits, 0, 8, st));
    size_t tb = 0;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, b->r_len, b->r_len, (int)(H.n_hits + 1), st));
    if (tb > b->r_tmp_bytes) {
        hipFree(b->r_tmp);
        b->r_tmp = nullptr;
        HIPCHK(hipMalloc(&b->r_tmp, tb));
        b->r_tmp_bytes = tb;
    }
    tb = b->r_tmp_bytes;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(b->r_tmp, tb, b->r_len, b->r_len, (int)(H.n_hits + 1), st));
    int64_t total = 0;
    HIPCHK(hipMemcpyAsync(&total, b->r_len + H.n_hits, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    { int rc = grow_dev(b->r_text, b->r_text_cap, total + 1); if (rc) return rc; }
    if (total + 1 > b->r_host_cap) {
        hipHostFree(b->r_host);
        b->r_host = nullptr;
        b->r_host_cap = std::max<int64_t>(total + 1, b->r_host_cap + b->r_host_cap / 2);
        HIPCHK(hipHostMalloc((void **)&b->r_host, (size_t)b->r_host_cap));
    }
    HIPCHK(launch_row_write(st, v, b->r_len, b->r_text));
    HIPCHK(hipMemcpyAsync(b->r_host, b->r_text, (size_t)total, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    b->r_host[total] = 0;
    *text = b->r_host;
    *len = total;
    return BSQ_OK;
}

extern "C" int bsq_batch_stage_ms(const bsq_batch *b, float *ms, int max)
{
    if (!b) return 0;
    for (int s = 0; s < STG_N && s < max; ++s) ms[s] = b->stage_ms[s];
    return STG_N;
}

extern "C" int bsq_batch_stage_bytes(const bsq_batch *b, double *bytes, int max)
{
    if (!b) return 0;
    for (int s = 0; s < STG_N && s < max; ++s) bytes[s] = b->stage_bytes[s];
    return STG_N;
}

extern "C" int64_t bsq_batch_sort_guard(const bsq_batch *b) { return b ? b->sort_guard : -1; }
extern "C" int64_t bsq_sort_guard_total(void) { return g_sort_guard.load(); }

extern "C" int bsq_batch_stage_work(const bsq_batch *b, double *work, int max)
{
    if (!b) return 0;
    for (int s = 0; s < STG_N && s < max; ++s) work[s] = b->stage_work[s];
    return STG_N;
}

extern "C" int64_t bsq_batch_retried(const bsq_batch *b) { return b ? b->retried : -1; }

// ================================================================================================
// one-shot API
// ================================================================================================
// Result arrays of the one-shot call.  A cursor calls bsq_align_batch fetch after fetch with results of similar
// size, and fresh malloc'd pages of ~90 MB per 1M reads cost more to fault in than the copy into them; freed
// result arrays are kept (a few, at most 2 GB) and handed to the next call that fits.  Each array carries its
// capacity in a 64-byte header.
namespace {
std::mutex g_out_mu;
std::vector<std::pair<size_t, void *>> g_out_cache;   // (capacity, header), most recently freed last
size_t g_out_bytes = 0;
constexpr size_t kOutCacheBytes = (size_t)2 << 30, kOutCacheN = 6, kOutHdr = 64;

void *out_alloc(size_t bytes)
{
    {
        std::lock_guard<std::mutex> lk(g_out_mu);
        size_t best = SIZE_MAX;
        for (size_t i = 0; i < g_out_cache.size(); ++i) {
            const size_t c = g_out_cache[i].first;
            if (c >= bytes && c <= 2 * bytes + (1 << 20) && (best == SIZE_MAX || c < g_out_cache[best].first)) best = i;
        }
        if (best != SIZE_MAX) {
            void *hdr = g_out_cache[best].second;
            g_out_bytes -= g_out_cache[best].first;
            g_out_cache.erase(g_out_cache.begin() + (long)best);
            return static_cast<uint8_t *>(hdr) + kOutHdr;
        }
    }
    void *hdr = malloc(bytes + kOutHdr);
    if (!hdr) return nullptr;
    *static_cast<size_t *>(hdr) = bytes;
    return static_cast<uint8_t *>(hdr) + kOutHdr;
}

void out_cache_drain()
{
    std::lock_guard<std::mutex> lk(g_out_mu);
    for (auto &c : g_out_cache) free(c.second);
    g_out_cache.clear();
    g_out_bytes = 0;
}

void out_free(void *p)
{
    if (!p) return;
    void *hdr = static_cast<uint8_t *>(p) - kOutHdr;
    const size_t cap = *static_cast<size_t *>(hdr);
    std::lock_guard<std::mutex> lk(g_out_mu);
    g_out_cache.emplace_back(cap, hdr);
    g_out_bytes += cap;
    while (g_out_cache.size() > kOutCacheN || g_out_bytes > kOutCacheBytes) {
        g_out_bytes -= g_out_cache.front().first;
        free(g_out_cache.front().second);
        g_out_cache.erase(g_out_cache.begin());
    }
}
}  // namespace

extern "C" int bsq_align_batch(bsq_index *idx, const bsq_opts *opts, const void *const *reads, int32_t n_reads,
                               uint64_t first_call_seq, bsq_hits **out)
{
    if (!idx || !opts || !out || n_reads < 0 || (n_reads && !reads)) { set_err("invalid argument"); return BSQ_E_INVALID; }
    *out = nullptr;
    for (int i = 0; i < n_reads; ++i)
        if (!reads[i]) { set_err("read %d is NULL", i); return BSQ_E_INVALID; }
    bsq_hits *h = (bsq_hits *)calloc(1, sizeof(bsq_hits));
    if (!h) { set_err("out of memory"); return BSQ_E_NOMEM; }
    h->n_reads = n_reads;
    if (!idx->h.built) { free(h); set_err("index not built"); return BSQ_E_INVALID; }
    if (idx->h.seq_len == 0 || n_reads == 0) {   // empty reference: align_sequence returns {} (bwa.cpp:142-143)
        h->read_off = (int64_t *)out_alloc(((size_t)n_reads + 1) * 8);
        if (!h->read_off) { free(h); set_err("out of host memory"); return BSQ_E_NOMEM; }
        memset(h->read_off, 0, ((size_t)n_reads + 1) * 8);
        *out = h;
        return BSQ_OK;
    }
    if (!idx->h.dev) { free(h); set_err("index not uploaded to a device (call bsq_index_upload)"); return BSQ_E_NODEV; }
    // The call runs as up to `slots` concurrent sub-batches of the index's pipeline (pipeline.cpp): each slot's
    // worker stages, uploads and aligns its share on its own stream, so the stages of one fill the tails of the
    // others and the host staging runs in parallel.  The pipeline (and its workspaces) is kept across calls; a
    // concurrent caller that finds it busy runs on a pipeline of its own.
    const int slots = []() { const char *e = getenv("BSQ_PIPE_SLOTS"); const int v = e ? atoi(e) : 0; return v > 0 ? std::min(v, 16) : 4; }();
    const int64_t min_chunk = 32768;   // smaller shares lose more to the stage tails than concurrency gains
    const int k = (int)std::max<int64_t>(1, std::min<int64_t>(slots, ((int64_t)n_reads + min_chunk - 1) / min_chunk));
    std::unique_lock<std::mutex> lk(idx->pool_mu, std::try_to_lock);
    const bool pooled = lk.owns_lock();
    bsq_pipeline *p = nullptr;
    int rc = BSQ_OK;
    if (pooled) {
        if (!idx->pipe || bsq_pipeline_slots(idx->pipe) < k) {
            bsq_pipeline_free(idx->pipe);
            idx->pipe = nullptr;
            rc = bsq_pipeline_create(idx, std::max(k, slots), &idx->pipe);
        }
        p = idx->pipe;
    } else rc = bsq_pipeline_create(idx, k, &p);
    std::vector<int32_t> lo((size_t)k + 1);
    for (int j = 0; j <= k; ++j) lo[(size_t)j] = (int32_t)((int64_t)n_reads * j / k);
    int submitted = 0;
    for (int j = 0; j < k && rc == BSQ_OK; ++j) {
        rc = pipeline_submit_ex(p, opts, reads + lo[(size_t)j], lo[(size_t)j + 1] - lo[(size_t)j],
                                first_call_seq + (uint64_t)lo[(size_t)j], 0, PipeMode::DEFER);
        if (rc == BSQ_OK) ++submitted;
    }
    std::vector<const bsq_hits *> v((size_t)k, nullptr);
    std::string err;
    for (int j = 0; j < submitted; ++j) {   // every submission is taken, failed or not
        const int r = pipeline_next_ex(p, &v[(size_t)j], nullptr, nullptr, nullptr);
        if (r && rc == BSQ_OK) { rc = r; err = g_err; }
    }
    auto release_all = [&] {
        for (int j = 0; j < submitted; ++j) if (v[(size_t)j]) bsq_pipeline_release(p);
        if (!pooled) bsq_pipeline_free(p);
    };
    if (rc != BSQ_OK) {
        if (!err.empty()) g_err = err;
        const std::string m = g_err;
        release_all();
        if (pooled) { bsq_pipeline_free(idx->pipe); idx->pipe = nullptr; }
        g_err = m;
        free(h);
        return rc;
    }
    std::vector<int64_t> hb((size_t)k + 1, 0), cb((size_t)k + 1, 0);
    for (int j = 0; j < k; ++j) {
        hb[(size_t)j + 1] = hb[(size_t)j] + v[(size_t)j]->n_hits;
        cb[(size_t)j + 1] = cb[(size_t)j] + v[(size_t)j]->n_cigar;
    }
    if (cb[(size_t)k] > (int64_t)UINT32_MAX) {
        release_all();
        free(h);
        set_err("call holds more than 2^32 CIGAR operations; split it into smaller batches");
        return BSQ_E_UNSUPPORTED;
    }
    h->n_hits = hb[(size_t)k];
    h->n_cigar = cb[(size_t)k];
    h->hits = (bsq_hit *)out_alloc(sizeof(bsq_hit) * (size_t)std::max<int64_t>(h->n_hits, 1));
    h->cigar = (uint32_t *)out_alloc(4 * (size_t)std::max<int64_t>(h->n_cigar, 1));
    h->read_off = (int64_t *)out_alloc(8 * ((size_t)n_reads + 1));
    if (!h->hits || !h->cigar || !h->read_off) {
        release_all();
        bsq_hits_free(h);
        set_err("out of host memory for the hit records");
        return BSQ_E_NOMEM;
    }
    // merge in read order, one host thread per share: call-wide read indices and CIGAR offsets
    auto copy_share = [&](int j) {
        const bsq_hits &x = *v[(size_t)j];
        bsq_hit *dst = h->hits + hb[(size_t)j];
        if (x.n_hits) memcpy(dst, x.hits, sizeof(bsq_hit) * (size_t)x.n_hits);
        for (int64_t i = 0; i < x.n_hits; ++i) {
            dst[i].read_index += lo[(size_t)j];
            dst[i].cigar_off += (uint32_t)cb[(size_t)j];
        }
        if (x.n_cigar) memcpy(h->cigar + cb[(size_t)j], x.cigar, 4 * (size_t)x.n_cigar);
        for (int32_t r = 0; r < x.n_reads; ++r) h->read_off[lo[(size_t)j] + r] = hb[(size_t)j] + x.read_off[r] - x.read_off[0];
    };
    {
        std::vector<std::thread> th;
        for (int j = 1; j < k; ++j) th.emplace_back(copy_share, j);
        copy_share(0);
        for (auto &t : th) t.join();
    }
    h->read_off[n_reads] = h->n_hits;
    release_all();
    *out = h;
    return BSQ_OK;
}

extern "C" int bsq_index_release_pool(bsq_index *idx)
{
    if (!idx) { set_err("invalid argument"); return BSQ_E_INVALID; }
    std::unique_lock<std::mutex> lk(idx->pool_mu, std::try_to_lock);
    if (!lk.owns_lock()) { set_err("the index's pooled pipeline is in use"); return BSQ_E_INVALID; }
    bsq_pipeline_free(idx->pipe);
    idx->pipe = nullptr;
    out_cache_drain();   // the recycled result arrays of the one-shot calls (up to 2 GB) go back too
    return BSQ_OK;
}

extern "C" void bsq_hits_free(bsq_hits *h)
{
    if (!h) return;
    out_free(h->hits); out_free(h->cigar); out_free(h->read_off); free(h);
}

// ================================================================================================
// bulk nuclseq codec on the GPU (codec_gpu.hip)
// ================================================================================================
namespace {
struct DevAllocs {   // device buffers of one call, released on every return path
    std::vector<void *> p;
    ~DevAllocs() { for (void *q : p) hipFree(q); }
    template <typename T>
    hipError_t get(T *&out, size_t count)
    {
        void *q = nullptr;
        const hipError_t e = hipMalloc(&q, std::max<size_t>(count, 1) * sizeof(T));
        if (e == hipSuccess) p.push_back(q);
        out = static_cast<T *>(q);
        return e;
    }
};
struct OwnStream {
    hipStream_t s = nullptr;
    ~OwnStream() { if (s) hipStreamDestroy(s); }
};
thread_local double g_codec_ms[2];   // last call: kernels, whole call

double now_ms()
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

bool allowed_host(unsigned char c) { return c && strchr("ACGTNWSMKRYBDHV", c) != nullptr; }

int codec_device(int device)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
    if (device < 0 || device >= ndev) {
        set_err("no HIP device %d (found %d); the bulk codec has no CPU fallback (bsq_nuclseq_from_text / _to_text "
                "are the per-value host path)", device, ndev);
        return BSQ_E_NODEV;
    }
    HIPCHK(hipSetDevice(device));
    return BSQ_OK;
}
}  // namespace

// nuclseq_from_text of n texts already in HBM (text i at d_text + toff[i], pac bytes poff[]): the varlenas
// are written to *d_out at the device offsets *d_off (n+1, 8-byte aligned), *total bytes.  With validate,
// a character nuclseq_in rejects stops before the write pass: *first_bad = its text offset (else ~0).
// d_toff / d_poff: the texts' offsets and pac-byte offsets (n + 1 each) already on the device; slots = d_poff[n].
template <class Alloc>
static int encode_device_core(hipStream_t st, Alloc &da, const uint8_t *d_text, const int64_t *d_toff,
                              const int64_t *d_poff, int64_t slots, int64_t n, bool validate, uint8_t **d_out,
                              int64_t **d_off, int64_t *total, unsigned long long *first_bad, double *kernel_ms)
{
    const int64_t ntiles = (slots + 255) / 256;
    if (ntiles + 1 >= INT32_MAX || n + 1 >= INT32_MAX) { set_err("batch too large (%lld pac bytes)", (long long)slots); return BSQ_E_INVALID; }
    int64_t *tile_first, *tile_hb, *tile_hs, *hb_base, *hs_base, *off;
    uint32_t *loc;
    unsigned long long *bad;
    HIPCHK(da.get(tile_first, (size_t)ntiles + 1));
    HIPCHK(da.get(tile_hb, (size_t)ntiles + 1));
    HIPCHK(da.get(tile_hs, (size_t)ntiles + 1));
    HIPCHK(da.get(hb_base, (size_t)n + 1));
    HIPCHK(da.get(hs_base, (size_t)n + 1));
    HIPCHK(da.get(off, (size_t)n + 1));
    HIPCHK(da.get(loc, (size_t)n + 1));
    HIPCHK(da.get(bad, 1));
    HIPCHK(hipMemsetAsync(tile_hb, 0, ((size_t)ntiles + 1) * 8, st));
    HIPCHK(hipMemsetAsync(tile_hs, 0, ((size_t)ntiles + 1) * 8, st));
    HIPCHK(hipMemsetAsync(bad, 0xff, 8, st));
    hipEvent_t ev[4];
    for (auto &e : ev) HIPCHK(hipEventCreate(&e));
    struct EvFree { hipEvent_t *e; ~EvFree() { for (int i = 0; i < 4; ++i) hipEventDestroy(e[i]); } } evf{ev};
    const EncView v{d_text, d_toff, d_poff, n, slots, validate ? 1 : 0};
    HIPCHK(hipEventRecord(ev[0], st));
    HIPCHK(launch_enc_count(st, v, ntiles, tile_first, tile_hb, tile_hs, loc, bad));
    size_t tb = 0, tb2 = 0;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, tile_hb, tile_hb, (int)(ntiles + 1), st));
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, off, off, (int)(n + 1), st));
    uint8_t *cub = nullptr;
    HIPCHK(da.get(cub, std::max(tb, tb2)));
    tb = std::max(tb, tb2);
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(cub, tb, tile_hb, tile_hb, (int)(ntiles + 1), st));
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(cub, tb, tile_hs, tile_hs, (int)(ntiles + 1), st));
    HIPCHK(launch_enc_meta(st, v, tile_hb, tile_hs, ntiles, loc, hb_base, hs_base, off));
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(cub, tb, off, off, (int)(n + 1), st));
    int64_t tot[2] = {0, 0};
    HIPCHK(hipEventRecord(ev[1], st));
    HIPCHK(hipMemcpyAsync(&tot[0], off + n, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(&tot[1], hs_base + n, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(first_bad, bad, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    *d_out = nullptr; *d_off = off; *total = tot[0];
    if (validate && *first_bad != ~0ull) return BSQ_OK;
    uint8_t *out;
    HIPCHK(da.get(out, (size_t)tot[0]));
    HIPCHK(hipEventRecord(ev[2], st));
    HIPCHK(launch_enc_write(st, v, ntiles, tile_first, tile_hb, tile_hs, hb_base, hs_base, off, tot[1], out));
    HIPCHK(hipEventRecord(ev[3], st));
    HIPCHK(hipStreamSynchronize(st));
    float a = 0, c = 0;
    hipEventElapsedTime(&a, ev[0], ev[1]);
    hipEventElapsedTime(&c, ev[2], ev[3]);
    *kernel_ms = a + c;
    *d_out = out;
    return BSQ_OK;
}

// the same with the offsets in host vectors (uploaded first)
template <class Alloc>
static int encode_device(hipStream_t st, Alloc &da, const uint8_t *d_text, const std::vector<int64_t> &toff,
                         const std::vector<int64_t> &poff, int64_t n, bool validate, uint8_t **d_out, int64_t **d_off,
                         int64_t *total, unsigned long long *first_bad, double *kernel_ms)
{
    int64_t *d_toff, *d_poff;
    HIPCHK(da.get(d_toff, (size_t)n + 1));
    HIPCHK(da.get(d_poff, (size_t)n + 1));
    HIPCHK(hipMemcpyAsync(d_toff, toff.data(), ((size_t)n + 1) * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_poff, poff.data(), ((size_t)n + 1) * 8, hipMemcpyHostToDevice, st));
    return encode_device_core(st, da, d_text, d_toff, d_poff, poff[(size_t)n], n, validate, d_out, d_off, total,
                              first_bad, kernel_ms);
}

// copies n+1 offsets and the bytes they span from the device into malloc'd host arrays
static int download(hipStream_t st, const uint8_t *d_buf, const int64_t *d_off, int64_t n, int64_t total, uint8_t **buf,
                    int64_t **offs)
{
    uint8_t *h_buf = static_cast<uint8_t *>(malloc((size_t)std::max<int64_t>(total, 1)));
    int64_t *h_off = static_cast<int64_t *>(malloc(((size_t)n + 1) * 8));
    if (!h_buf || !h_off) { free(h_buf); free(h_off); set_err("out of host memory"); return BSQ_E_NOMEM; }
    hipError_t e = total ? hipMemcpyAsync(h_buf, d_buf, (size_t)total, hipMemcpyDeviceToHost, st) : hipSuccess;
    if (e == hipSuccess) e = hipMemcpyAsync(h_off, d_off, ((size_t)n + 1) * 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) { free(h_buf); free(h_off); set_err("download: %s", hipGetErrorString(e)); return BSQ_E_HIP; }
    *buf = h_buf;
    *offs = h_off;
    return BSQ_OK;
}

extern "C" int bsq_nuclseq_encode_batch(int device, const char *text, const int64_t *offs, int64_t n, int validate,
                                        uint8_t **out, int64_t **out_off)
{
    if (!offs || n < 0 || n >= INT32_MAX || !out || !out_off) { set_err("invalid argument"); return BSQ_E_INVALID; }
    *out = nullptr; *out_off = nullptr;
    const double t_call = now_ms();
    std::vector<int64_t> toff((size_t)n + 1, 0), poff((size_t)n + 1, 0);
    int64_t first_long = -1;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t len = offs[i + 1] - offs[i];
        if (len < 0) { set_err("text offsets decrease at text %lld", (long long)i); return BSQ_E_INVALID; }
        if (len > INT32_MAX / 4 && first_long < 0) first_long = i;
        toff[(size_t)i + 1] = toff[(size_t)i] + len;
        poff[(size_t)i + 1] = poff[(size_t)i] + (len + 3) / 4;
    }
    if (toff[(size_t)n] && !text) { set_err("invalid argument"); return BSQ_E_INVALID; }
    if (first_long >= 0) {   // nuclseq_in checks the length before the alphabet (extension.cpp:50-58)
        for (int64_t i = 0; validate && i < first_long; ++i)
            for (int64_t j = offs[i]; j < offs[i + 1]; ++j)
                if (!allowed_host((unsigned char)text[j])) {
                    set_err("invalid nucleotide in nuclseq_in: '%c'", text[j]);
                    return BSQ_E_INVALID;
                }
        set_err("provided sequence is too long");
        return BSQ_E_INVALID;
    }
    { const int rc = codec_device(device); if (rc) return rc; }
    OwnStream os;
    HIPCHK(hipStreamCreateWithFlags(&os.s, hipStreamNonBlocking));
    hipStream_t st = os.s;
    DevAllocs da;
    uint8_t *d_text;
    HIPCHK(da.get(d_text, (size_t)toff[(size_t)n]));
    if (toff[(size_t)n]) HIPCHK(hipMemcpyAsync(d_text, text + offs[0], (size_t)toff[(size_t)n], hipMemcpyHostToDevice, st));
    uint8_t *d_out = nullptr;
    int64_t *d_off = nullptr, total = 0;
    unsigned long long first_bad = ~0ull;
    double kms = 0;
    { const int rc = encode_device(st, da, d_text, toff, poff, n, validate != 0, &d_out, &d_off, &total, &first_bad, &kms);
      if (rc) return rc; }
    if (validate && first_bad != ~0ull) {   // the first text (in order) with a character nuclseq_in rejects
        set_err("invalid nucleotide in nuclseq_in: '%c'", text[offs[0] + (int64_t)first_bad]);
        return BSQ_E_INVALID;
    }
    { const int rc = download(st, d_out, d_off, n, total, out, out_off); if (rc) return rc; }
    g_codec_ms[0] = kms;
    g_codec_ms[1] = now_ms() - t_call;
    return BSQ_OK;
}

// build_tuple_bwa's two nuclseq columns for every row of the last run (extension.cpp:282-305, which calls
// nuclseq_from_text on ref_subseq and query_subseq per row, :285,290) into the batch's pinned buffers (borrowed
// until the next render or run of the batch): varlena 2k = ref_subseq of row k, 2k+1 = its query_subseq.  Texts
// without holes are packed straight from the reference pac / the read codes (render_gpu.hip k_col_direct); the
// few with holes are rendered as text and encoded by the bulk codec; one D2H.
namespace bsq {
int batch_render_cols(bsq_batch *b, const void *const *reads, const uint8_t **out, const int64_t **out_off)
{
    const double t_call = now_ms();
    const bsq_hits &H = b->view;
    const int64_t n = 2 * H.n_hits;
    HIPCHK(hipSetDevice(b->device));
    // The columns run after the batch's alignment, while the pipeline's other slots align: on a stream of the
    // device's greatest priority their small kernels are dispatched ahead of the queued alignment workgroups,
    // so the oldest fetch's rows (the ones the backend waits for) are not held behind the younger fetches'
    // seeding (BSQ_COLS_PRIORITY=0: the batch's own stream)
    if (!b->cstream) {
        const char *e = getenv("BSQ_COLS_PRIORITY");
        if (e && *e == '0') b->cstream = b->stream;
        else {
            int lo = 0, hi = 0;
            HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
            HIPCHK(hipStreamCreateWithPriority(&b->cstream, hipStreamNonBlocking, hi));
        }
    }
    hipStream_t st = b->cstream;
    b->arena.reset();
    int64_t *size, *hpos;
    HIPCHK(b->arena.get(size, (size_t)n + 1));
    HIPCHK(b->arena.get(hpos, (size_t)n + 1));
    uint8_t *d_out = nullptr;
    int64_t total = 0;
    double kms = 0;
    if (H.n_hits) {
        // (1) hole-free texts get their varlena size directly; (2) the texts with holes (reference N runs over the
        // window, reads with ambiguous bases) are rendered and encoded by the generic codec as a compacted subset;
        // (3) one scan of the sizes gives every varlena's offset; (4) the hole-free varlenas are written straight from
        // the pac / the read codes and the generic ones copied into place.
        RenderView v{};
        { const int rc = render_inputs(b, reads, v, st); if (rc) return rc; }
        hipEvent_t ev[2];
        for (auto &e : ev) HIPCHK(hipEventCreate(&e));
        struct EvFree { hipEvent_t *e; ~EvFree() { hipEventDestroy(e[0]); hipEventDestroy(e[1]); } } evf{ev};
        HIPCHK(hipEventRecord(ev[0], st));
        HIPCHK(launch_col_class(st, v, size, hpos));
        size_t tb = 0;
        HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, hpos, hpos, (int)(n + 1), st));
        uint8_t *cub = nullptr;
        HIPCHK(b->arena.get(cub, tb));
        HIPCHK(hipcub::DeviceScan::ExclusiveSum(cub, tb, hpos, hpos, (int)(n + 1), st));
        int64_t nh = 0;
        HIPCHK(hipMemcpyAsync(&nh, hpos + n, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        int64_t *hl = nullptr, *enc_off = nullptr;
        uint8_t *enc = nullptr;
        double ekms = 0;
        if (nh) {
            int64_t *tl, *pl;
            HIPCHK(b->arena.get(hl, (size_t)nh));
            HIPCHK(b->arena.get(tl, (size_t)nh + 1));
            HIPCHK(b->arena.get(pl, (size_t)nh + 1));
            HIPCHK(launch_col_holed(st, v, hpos, nh, hl, tl, pl));
            size_t tb2 = 0;
            HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, tl, tl, (int)(nh + 1), st));
            uint8_t *cub2 = nullptr;
            HIPCHK(b->arena.get(cub2, tb2));
            HIPCHK(hipcub::DeviceScan::ExclusiveSum(cub2, tb2, tl, tl, (int)(nh + 1), st));
            HIPCHK(hipcub::DeviceScan::ExclusiveSum(cub2, tb2, pl, pl, (int)(nh + 1), st));
            int64_t tot[2] = {0, 0};
            HIPCHK(hipMemcpyAsync(&tot[0], tl + nh, 8, hipMemcpyDeviceToHost, st));
            HIPCHK(hipMemcpyAsync(&tot[1], pl + nh, 8, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            char *d_text;
            HIPCHK(b->arena.get(d_text, (size_t)std::max<int64_t>(tot[0], 1)));
            HIPCHK(launch_sub_write_sel(st, v, hl, nh, tl, d_text));
            int64_t etotal = 0;
            unsigned long long first_bad = ~0ull;
            { const int rc = encode_device_core(st, b->arena, reinterpret_cast<const uint8_t *>(d_text), tl, pl, tot[1], nh,
                                                false, &enc, &enc_off, &etotal, &first_bad, &ekms);
              if (rc) return rc; }
            HIPCHK(launch_col_holed_size(st, hl, nh, enc_off, size));
        }
        HIPCHK(hipcub::DeviceScan::ExclusiveSum(cub, tb, size, size, (int)(n + 1), st));
        HIPCHK(hipMemcpyAsync(&total, size + n, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        HIPCHK(b->arena.get(d_out, (size_t)std::max<int64_t>(total, 1)));
        HIPCHK(launch_col_write(st, v, size, hpos, hl, nh, enc_off, enc, d_out));
        HIPCHK(hipEventRecord(ev[1], st));
        HIPCHK(hipStreamSynchronize(st));
        float ms = 0;
        hipEventElapsedTime(&ms, ev[0], ev[1]);
        kms = ms;
        (void)ekms;
    } else {
        HIPCHK(hipMemsetAsync(size, 0, 8, st));
    }
    { int rc = grow_pinned(b->c_host, b->c_host_cap, std::max<int64_t>(total, 1), 0); if (rc) return rc; }
    { int rc = grow_pinned(b->c_off, b->c_off_cap, n + 1, 0); if (rc) return rc; }
    if (total) HIPCHK(hipMemcpyAsync(b->c_host, d_out, (size_t)total, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(b->c_off, size, ((size_t)n + 1) * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    *out = b->c_host;
    *out_off = b->c_off;
    g_codec_ms[0] = kms;
    g_codec_ms[1] = now_ms() - t_call;
    return BSQ_OK;
}
}  // namespace bsq

extern "C" int bsq_batch_render_nuclseqs(bsq_batch *b, const void *const *reads, uint8_t **out, int64_t **out_off)
{
    if (!b || !out || !out_off) { set_err("invalid argument"); return BSQ_E_INVALID; }
    *out = nullptr; *out_off = nullptr;
    const uint8_t *c = nullptr;
    const int64_t *o = nullptr;
    { const int rc = batch_render_cols(b, reads, &c, &o); if (rc) return rc; }
    const int64_t n = 2 * b->view.n_hits, total = o[n];
    uint8_t *h_buf = static_cast<uint8_t *>(malloc((size_t)std::max<int64_t>(total, 1)));
    int64_t *h_off = static_cast<int64_t *>(malloc(((size_t)n + 1) * 8));
    if (!h_buf || !h_off) { free(h_buf); free(h_off); set_err("out of host memory"); return BSQ_E_NOMEM; }
    if (total) memcpy(h_buf, c, (size_t)total);
    memcpy(h_off, o, ((size_t)n + 1) * 8);
    *out = h_buf;
    *out_off = h_off;
    return BSQ_OK;
}

extern "C" int bsq_nuclseq_decode_batch(int device, const void *const *nuclseqs, int64_t n, char **text,
                                        int64_t **text_off)
{
    if (n < 0 || (n > 0 && !nuclseqs) || !text || !text_off) { set_err("invalid argument"); return BSQ_E_INVALID; }
    *text = nullptr; *text_off = nullptr;
    const double t_call = now_ms();
    std::vector<int64_t> in_off((size_t)n + 1, 0), poff((size_t)n + 1, 0), toff((size_t)n + 1, 0), holed;
    for (int64_t s = 0; s < n; ++s) {
        const uint8_t *ns = static_cast<const uint8_t *>(nuclseqs[s]);
        if (!ns) { set_err("nuclseq %lld is NULL", (long long)s); return BSQ_E_INVALID; }
        uint32_t vl; memcpy(&vl, ns, 4);
        const uint64_t size = vl >> 2, nh = ns_holes_num(ns), len = ns_len(ns);
        const uint64_t need = 12 + 16 * nh + pac_byte_size(len);
        if (size < need) {
            set_err("nuclseq %lld: varlena of %llu bytes, %llu needed", (long long)s, (unsigned long long)size,
                    (unsigned long long)need);
            return BSQ_E_INVALID;
        }
        if (nh) holed.push_back(s);
        in_off[(size_t)s + 1] = in_off[(size_t)s] + (int64_t)((need + 7) & ~7ull);
        poff[(size_t)s + 1] = poff[(size_t)s] + (int64_t)pac_byte_size(len);
        toff[(size_t)s + 1] = toff[(size_t)s] + (int64_t)len;
    }
    { const int rc = codec_device(device); if (rc) return rc; }
    OwnStream os;
    HIPCHK(hipStreamCreateWithFlags(&os.s, hipStreamNonBlocking));
    hipStream_t st = os.s;
    std::vector<uint8_t> packed((size_t)in_off[(size_t)n]);
    for (int64_t s = 0; s < n; ++s)
        memcpy(packed.data() + in_off[(size_t)s], nuclseqs[s],
               12 + 16 * (size_t)ns_holes_num(static_cast<const uint8_t *>(nuclseqs[s])) +
                   (size_t)(poff[(size_t)s + 1] - poff[(size_t)s]));
    DevAllocs da;
    uint8_t *d_in;
    int64_t *d_in_off, *d_poff, *d_toff, *d_holed;
    char *d_text;
    HIPCHK(da.get(d_in, packed.size()));
    HIPCHK(da.get(d_in_off, (size_t)n + 1));
    HIPCHK(da.get(d_poff, (size_t)n + 1));
    HIPCHK(da.get(d_toff, (size_t)n + 1));
    HIPCHK(da.get(d_holed, holed.size()));
    HIPCHK(da.get(d_text, (size_t)toff[(size_t)n]));
    if (!packed.empty()) HIPCHK(hipMemcpyAsync(d_in, packed.data(), packed.size(), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_in_off, in_off.data(), ((size_t)n + 1) * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_poff, poff.data(), ((size_t)n + 1) * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_toff, toff.data(), ((size_t)n + 1) * 8, hipMemcpyHostToDevice, st));
    if (!holed.empty()) HIPCHK(hipMemcpyAsync(d_holed, holed.data(), holed.size() * 8, hipMemcpyHostToDevice, st));
    hipEvent_t ev[2];
    for (auto &e : ev) HIPCHK(hipEventCreate(&e));
    struct EvFree { hipEvent_t *e; ~EvFree() { hipEventDestroy(e[0]); hipEventDestroy(e[1]); } } evf{ev};
    const DecView v{d_in, d_in_off, d_poff, d_toff, n, poff[(size_t)n]};
    HIPCHK(hipEventRecord(ev[0], st));
    HIPCHK(launch_dec(st, v, d_holed, (int64_t)holed.size(), d_text));
    HIPCHK(hipEventRecord(ev[1], st));
    char *h_text = static_cast<char *>(malloc((size_t)toff[(size_t)n] + 1));
    int64_t *h_off = static_cast<int64_t *>(malloc(((size_t)n + 1) * 8));
    if (!h_text || !h_off) { free(h_text); free(h_off); set_err("out of host memory"); return BSQ_E_NOMEM; }
    hipError_t e = toff[(size_t)n] ? hipMemcpyAsync(h_text, d_text, (size_t)toff[(size_t)n], hipMemcpyDeviceToHost, st)
                                   : hipSuccess;
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) { free(h_text); free(h_off); set_err("decode: %s", hipGetErrorString(e)); return BSQ_E_HIP; }
    h_text[toff[(size_t)n]] = 0;
    memcpy(h_off, toff.data(), ((size_t)n + 1) * 8);
    float a = 0;
    hipEventElapsedTime(&a, ev[0], ev[1]);
    g_codec_ms[0] = a;
    g_codec_ms[1] = now_ms() - t_call;
    *text = h_text;
    *text_off = h_off;
    return BSQ_OK;
}

extern "C" int bsq_nuclseq_codec_ms(double *kernel_ms, double *call_ms)
{
    if (kernel_ms) *kernel_ms = g_codec_ms[0];
    if (call_ms) *call_ms = g_codec_ms[1];
    return BSQ_OK;
}
