// group.cpp -- one host process driving several MI355X devices (include/bsq.h bsq_group_*).
//
// a Postgres backend is one process, so the multi-GPU form of the SQL path is one process
// with one RCCL communicator per device (ncclCommInitAll over xGMI), not one process per GPU.  The index is
// built once (on member 0) and its device tables are broadcast to the other members; the reads of a cursor
// batch are sharded into contiguous ranges, one member each, every member on its own host thread and HIP
// stream; the records come back to the backend over each member's own PCIe link and are merged in read
// order.  This replaces the per-read loop of nuclseq_multi_search_bwa (bioseqdb/extension.cpp:362-370).
//
// Why the records are not gathered over xGMI first: the consumer is host memory (the backend's tuplestore).
// Pulling each shard over its own device's PCIe link uses all n links at once; an RCCL gather into member 0
// would then funnel every byte through member 0's single link.  The one-process-per-GPU driver
// (bioseqdb_amd/dist.py, bench.py --gpus N) is different -- there the other ranks cannot hand host memory to
// the caller, so its exchange step is an RCCL gather.
//
// Built only on the public C-ABI of bsq_api.cpp plus RCCL.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../../include/bsq.h"

extern "C" void bsq_internal_set_error(const char *msg);   // bsq_api.cpp: the message bsq_last_error() returns

namespace {

int fail(int rc, const std::string &m)
{
    bsq_internal_set_error(m.c_str());
    return rc;
}

int hip_fail(const char *what, hipError_t e) { return fail(BSQ_E_HIP, std::string(what) + ": " + hipGetErrorString(e)); }

struct Member {
    int device = 0;
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;
    bsq_index *index = nullptr;          // member 0: the caller's index; others: imported replica
    std::vector<void *> bufs;            // replica tables (owned, members >= 1)
    bsq_batch *batch = nullptr;
    int32_t cap_reads = 0;
    int64_t cap_bases = 0;
    int32_t lo = 0, n = 0;               // shard of the last run
};

}  // namespace

struct bsq_group {
    std::vector<Member> m;
    bool rccl = false;                   // distinct devices: RCCL communicators; a repeated device: D2D copies
    bsq_index *src = nullptr;
    int32_t n_reads = 0;
    std::vector<bsq_hit> hits;
    std::vector<uint32_t> cigar;
    std::vector<int64_t> read_off;
    bsq_hits view{};
};

namespace {

void drop_replicas(bsq_group *g)
{
    for (size_t k = 0; k < g->m.size(); ++k) {
        Member &x = g->m[k];
        bsq_batch_free(x.batch);
        x.batch = nullptr;
        x.cap_reads = 0;
        x.cap_bases = 0;
        if (k > 0) {
            bsq_index_free(x.index);
            hipSetDevice(x.device);
            for (void *p : x.bufs) hipFree(p);
        }
        x.bufs.clear();
        x.index = nullptr;
    }
    g->src = nullptr;
}

// Runs f(k) for every member on its own host thread (member 0 on the caller's); the first failure wins,
// with its message.
template <class F>
int for_members(bsq_group *g, F f)
{
    const size_t n = g->m.size();
    std::vector<int> rc(n, BSQ_OK);
    std::vector<std::string> msg(n);
    auto one = [&](size_t k) {
        rc[k] = f((int)k);
        if (rc[k]) msg[k] = bsq_last_error();
    };
    std::vector<std::thread> th;
    for (size_t k = 1; k < n; ++k) th.emplace_back(one, k);
    one(0);
    for (auto &t : th) t.join();
    for (size_t k = 0; k < n; ++k)
        if (rc[k]) return fail(rc[k], "member " + std::to_string(k) + " (device " + std::to_string(g->m[k].device) +
                                          "): " + msg[k]);
    return BSQ_OK;
}

}  // namespace

extern "C" int bsq_group_create(const int *devices, int n_devices, bsq_group **out)
{
    if (!devices || n_devices < 1 || !out) return fail(BSQ_E_INVALID, "invalid argument");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return fail(BSQ_E_NODEV, "no HIP device; the alignment path has no CPU fallback");
    std::vector<int> dl(devices, devices + n_devices);
    for (int d : dl)
        if (d < 0 || d >= ndev) return fail(BSQ_E_NODEV, "no HIP device " + std::to_string(d) + " (found " + std::to_string(ndev) + ")");
    std::unique_ptr<bsq_group> g(new (std::nothrow) bsq_group());
    if (!g) return fail(BSQ_E_NOMEM, "out of memory");
    g->m.resize((size_t)n_devices);
    std::vector<int> sorted = dl;
    std::sort(sorted.begin(), sorted.end());
    g->rccl = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    for (int k = 0; k < n_devices; ++k) {
        Member &x = g->m[(size_t)k];
        x.device = dl[(size_t)k];
        hipError_t e = hipSetDevice(x.device);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&x.stream, hipStreamNonBlocking);
        if (e != hipSuccess) { bsq_group_free(g.release()); return hip_fail("member stream", e); }
    }
    if (g->rccl) {
        std::vector<ncclComm_t> comms((size_t)n_devices, nullptr);
        const ncclResult_t r = ncclCommInitAll(comms.data(), n_devices, dl.data());
        if (r != ncclSuccess) {
            bsq_group_free(g.release());
            return fail(BSQ_E_HIP, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
        }
        for (int k = 0; k < n_devices; ++k) g->m[(size_t)k].comm = comms[(size_t)k];
    }
    *out = g.release();
    return BSQ_OK;
}

extern "C" void bsq_group_free(bsq_group *g)
{
    if (!g) return;
    drop_replicas(g);
    for (Member &x : g->m) {
        hipSetDevice(x.device);
        if (x.comm) ncclCommDestroy(x.comm);
        if (x.stream) hipStreamDestroy(x.stream);
    }
    delete g;
}

extern "C" int bsq_group_size(const bsq_group *g) { return g ? (int)g->m.size() : 0; }

extern "C" int bsq_group_replicate(bsq_group *g, bsq_index *idx, double *broadcast_ms)
{
    if (!g || !idx) return fail(BSQ_E_INVALID, "invalid argument");
    drop_replicas(g);
    const int dev0 = g->m[0].device;
    bsq_table src[BSQ_N_TABLES];
    int on = -1;
    if (bsq_index_device_tables(idx, &on, src, BSQ_N_TABLES) != BSQ_OK) {   // not on a device yet: upload to member 0
        const int rc = bsq_index_upload(idx, dev0);
        if (rc) return rc;
        if (bsq_index_device_tables(idx, &on, src, BSQ_N_TABLES) != BSQ_OK) return fail(BSQ_E_INVALID, bsq_last_error());
    }
    if (on != dev0) return fail(BSQ_E_INVALID, "index is on device " + std::to_string(on) + ", the group's first member is " +
                                                   std::to_string(dev0));
    uint64_t meta_bytes = 0;
    if (bsq_index_layout(idx, nullptr, nullptr, &meta_bytes) != BSQ_OK) return fail(BSQ_E_INVALID, bsq_last_error());
    std::vector<uint8_t> meta((size_t)meta_bytes);
    if (bsq_index_layout(idx, nullptr, meta.data(), &meta_bytes) != BSQ_OK) return fail(BSQ_E_INVALID, bsq_last_error());
    g->src = idx;
    g->m[0].index = idx;
    const size_t G = g->m.size();
    // receive buffers on the other members
    for (size_t k = 1; k < G; ++k) {
        Member &x = g->m[k];
        hipError_t e = hipSetDevice(x.device);
        if (e != hipSuccess) { drop_replicas(g); return hip_fail("hipSetDevice", e); }
        x.bufs.assign(BSQ_N_TABLES, nullptr);
        for (int t = 0; t < BSQ_N_TABLES; ++t) {
            if (!src[t].bytes) continue;
            e = hipMalloc(&x.bufs[(size_t)t], src[t].bytes);
            if (e != hipSuccess) { drop_replicas(g); return fail(BSQ_E_NOMEM, "replica table " + std::to_string(t) + ": " + hipGetErrorString(e)); }
        }
    }
    const auto t0 = std::chrono::steady_clock::now();
    roctxRangePushA("bsq_group_broadcast");
    struct PopAtExit { ~PopAtExit() { roctxRangePop(); } } pop_at_exit;
    if (G > 1) {
        if (g->rccl) {   // every table from member 0, all broadcasts in one group call
            ncclResult_t r = ncclGroupStart();
            for (int t = 0; t < BSQ_N_TABLES && r == ncclSuccess; ++t) {
                if (!src[t].bytes) continue;
                for (size_t k = 0; k < G && r == ncclSuccess; ++k) {
                    void *buf = k == 0 ? src[t].ptr : g->m[k].bufs[(size_t)t];
                    r = ncclBroadcast(buf, buf, (size_t)src[t].bytes, ncclUint8, 0, g->m[k].comm, g->m[k].stream);
                }
            }
            const ncclResult_t r2 = ncclGroupEnd();
            if (r == ncclSuccess) r = r2;
            if (r != ncclSuccess) { drop_replicas(g); return fail(BSQ_E_HIP, std::string("ncclBroadcast: ") + ncclGetErrorString(r)); }
        } else {         // replicas on a repeated device: plain device-to-device copies
            for (size_t k = 1; k < G; ++k)
                for (int t = 0; t < BSQ_N_TABLES; ++t) {
                    if (!src[t].bytes) continue;
                    const hipError_t e = hipMemcpyPeerAsync(g->m[k].bufs[(size_t)t], g->m[k].device, src[t].ptr, dev0,
                                                            src[t].bytes, g->m[k].stream);
                    if (e != hipSuccess) { drop_replicas(g); return hip_fail("replica copy", e); }
                }
        }
        for (size_t k = 0; k < G; ++k) {
            hipSetDevice(g->m[k].device);
            const hipError_t e = hipStreamSynchronize(g->m[k].stream);
            if (e != hipSuccess) { drop_replicas(g); return hip_fail("broadcast", e); }
        }
    }
    if (broadcast_ms) *broadcast_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    for (size_t k = 1; k < G; ++k) {
        Member &x = g->m[k];
        bsq_table tab[BSQ_N_TABLES];
        for (int t = 0; t < BSQ_N_TABLES; ++t) tab[t] = bsq_table{x.bufs[(size_t)t], src[t].bytes};
        const int rc = bsq_index_import(meta.data(), meta_bytes, x.device, tab, BSQ_N_TABLES, &x.index);
        if (rc) { const std::string m = bsq_last_error(); drop_replicas(g); return fail(rc, m); }
    }
    return BSQ_OK;
}

extern "C" int bsq_group_run(bsq_group *g, const bsq_opts *opts, const void *const *reads, int32_t n_reads,
                             uint64_t first_call_seq)
{
    if (!g || !opts) return fail(BSQ_E_INVALID, "invalid argument");
    if (!g->src) return fail(BSQ_E_INVALID, "no index replicated on the group (bsq_group_replicate)");
    const size_t G = g->m.size();
    if (reads) {
        if (n_reads < 0) return fail(BSQ_E_INVALID, "invalid argument");
        for (int32_t i = 0; i < n_reads; ++i)
            if (!reads[i]) return fail(BSQ_E_INVALID, "read " + std::to_string(i) + " is NULL");
        g->n_reads = n_reads;
        for (size_t k = 0; k < G; ++k) {
            g->m[k].lo = (int32_t)((int64_t)n_reads * (int64_t)k / (int64_t)G);
            g->m[k].n = (int32_t)((int64_t)n_reads * (int64_t)(k + 1) / (int64_t)G) - g->m[k].lo;
        }
    } else if (n_reads != g->n_reads) return fail(BSQ_E_INVALID, "re-run of a different read count");
    const int rc = for_members(g, [&](int k) -> int {
        Member &x = g->m[(size_t)k];
        if (x.n == 0) return BSQ_OK;
        if (reads) {
            int64_t bases = 0;
            for (int32_t i = 0; i < x.n; ++i) {
                uint32_t len;
                memcpy(&len, static_cast<const uint8_t *>(reads[x.lo + i]) + 8, 4);   // sequence.h:18-38 len
                bases += len;
            }
            if (!x.batch || x.cap_reads < x.n || x.cap_bases < bases) {
                bsq_batch_free(x.batch);
                x.batch = nullptr;
                x.cap_reads = std::max(x.n, 2 * x.cap_reads);
                x.cap_bases = std::max(bases, 2 * x.cap_bases);
                const int r = bsq_batch_create(x.index, x.cap_reads, x.cap_bases, &x.batch);
                if (r) { x.cap_reads = 0; x.cap_bases = 0; return r; }
            }
            const int r = bsq_batch_set_nuclseqs(x.batch, reads + x.lo, x.n);
            if (r) return r;
        }
        return bsq_batch_run(x.batch, opts, first_call_seq + (uint64_t)x.lo);
    });
    if (rc) return rc;
    // merge in member (= read) order: batch-wide read indices and CIGAR offsets
    int64_t nh = 0, nc = 0;
    std::vector<int64_t> hb(G + 1, 0), cb(G + 1, 0);
    for (size_t k = 0; k < G; ++k) {
        const bsq_hits *v = g->m[k].n ? bsq_batch_hits(g->m[k].batch) : nullptr;
        hb[k + 1] = hb[k] + (v ? v->n_hits : 0);
        cb[k + 1] = cb[k] + (v ? v->n_cigar : 0);
    }
    nh = hb[G];
    nc = cb[G];
    try {
        g->hits.resize((size_t)nh);
        g->cigar.resize((size_t)nc);
        g->read_off.resize((size_t)g->n_reads + 1);
    } catch (const std::bad_alloc &) {
        return fail(BSQ_E_NOMEM, "out of host memory for the merged records");
    }
    g->read_off[0] = 0;
    for (size_t k = 0; k < G; ++k) {
        const Member &x = g->m[k];
        if (!x.n) continue;
        const bsq_hits *v = bsq_batch_hits(x.batch);
        if ((uint64_t)cb[k] + (uint64_t)v->n_cigar > UINT32_MAX)
            return fail(BSQ_E_UNSUPPORTED, "more than 2^32 CIGAR operations in one call");
        bsq_hit *dst = g->hits.data() + hb[k];
        if (v->n_hits) memcpy(dst, v->hits, sizeof(bsq_hit) * (size_t)v->n_hits);
        for (int64_t i = 0; i < v->n_hits; ++i) {
            dst[i].read_index += x.lo;
            dst[i].cigar_off += (uint32_t)cb[k];
        }
        if (v->n_cigar) memcpy(g->cigar.data() + cb[k], v->cigar, 4 * (size_t)v->n_cigar);
        for (int32_t i = 1; i <= x.n; ++i) g->read_off[(size_t)x.lo + (size_t)i] = hb[k] + v->read_off[i] - v->read_off[0];
    }
    g->view.n_reads = g->n_reads;
    g->view.n_hits = nh;
    g->view.hits = g->hits.data();
    g->view.read_off = g->read_off.data();
    g->view.n_cigar = nc;
    g->view.cigar = g->cigar.data();
    return BSQ_OK;
}

extern "C" const bsq_hits *bsq_group_hits(const bsq_group *g) { return g ? &g->view : nullptr; }

extern "C" int bsq_group_render_nuclseqs(bsq_group *g, const void *const *reads, uint8_t **out, int64_t **out_off)
{
    if (!g || !out || !out_off || (g->n_reads && !reads)) return fail(BSQ_E_INVALID, "invalid argument");
    *out = nullptr;
    *out_off = nullptr;
    const size_t G = g->m.size();
    std::vector<uint8_t *> part(G, nullptr);
    std::vector<int64_t *> poff(G, nullptr);
    const int rc = for_members(g, [&](int k) -> int {
        const Member &x = g->m[(size_t)k];
        if (!x.n) return BSQ_OK;
        return bsq_batch_render_nuclseqs(x.batch, reads + x.lo, &part[(size_t)k], &poff[(size_t)k]);
    });
    auto release = [&] { for (size_t k = 0; k < G; ++k) { bsq_free(part[k]); bsq_free(poff[k]); } };
    if (rc) { release(); return rc; }
    const int64_t nv = 2 * g->view.n_hits;
    std::vector<int64_t> base(G + 1, 0);   // byte offset of member k's varlenas (8-byte aligned)
    for (size_t k = 0; k < G; ++k) {
        const int64_t nk = g->m[k].n ? 2 * bsq_batch_hits(g->m[k].batch)->n_hits : 0;
        const int64_t bytes = nk ? poff[k][nk] : 0;
        base[k + 1] = base[k] + ((bytes + 7) & ~7LL);
    }
    uint8_t *buf = static_cast<uint8_t *>(malloc((size_t)std::max<int64_t>(base[G], 1)));
    int64_t *off = static_cast<int64_t *>(malloc(((size_t)nv + 1) * 8));
    if (!buf || !off) { free(buf); free(off); release(); return fail(BSQ_E_NOMEM, "out of host memory"); }
    int64_t v0 = 0;
    for (size_t k = 0; k < G; ++k) {
        const int64_t nk = g->m[k].n ? 2 * bsq_batch_hits(g->m[k].batch)->n_hits : 0;
        if (!nk) continue;
        memcpy(buf + base[k], part[k], (size_t)poff[k][nk]);
        for (int64_t i = 0; i < nk; ++i) off[v0 + i] = base[k] + poff[k][i];
        v0 += nk;
    }
    off[nv] = base[G];
    release();
    *out = buf;
    *out_off = off;
    return BSQ_OK;
}
