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
// Every member aligns its shard as up to `slots` concurrent shares on a pipeline of its own (pipeline.cpp), so a
// member keeps its device as busy as the one-GPU bench's concurrent batches do.  The records stay where the
// members' pipelines put them -- pinned host memory, one segment per share, in read order -- until the caller
// asks for the merged view (bsq_group_hits merges on first use, one host thread per segment) or walks the
// segments itself (bsq_group_segments, zero-copy).
//
// Built on the public C-ABI of bsq_api.cpp plus RCCL and the pipeline internals (bsq_internal.h).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../../include/bsq.h"
#include "bsq_internal.h"

extern "C" void bsq_internal_set_error(const char *msg);   // bsq_api.cpp: the message bsq_last_error() returns

using bsq::PipeMode;
using bsq::pipeline_next_ex;
using bsq::pipeline_submit_ex;
using bsq::pipeline_rewind;
using bsq::pipeline_set_record_route;

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
    bsq_pipeline *pipe = nullptr;        // this member's concurrent shares (created at replicate)
    int32_t lo = 0, n = 0;               // shard of the last run
    std::vector<int32_t> slo;            // shares of the shard: [slo[j], slo[j+1]) relative to lo
    std::vector<const bsq_hits *> views; // taken (held) results of the shares, until the next run
    std::vector<bsq_batch *> batches;    // the batch holding each share's records (NULL: no rows)
};

}  // namespace

struct bsq_group {
    std::vector<Member> m;
    bool rccl = false;                   // distinct devices: RCCL communicators; a repeated device: D2D copies
    bsq_index *src = nullptr;
    int slots = 4;                       // concurrent shares per member (bsq_group_set_slots)
    int exchange = BSQ_XCHG_LINKS;       // how the records reach the host (bsq_group_set_exchange)
    int32_t n_reads = 0;
    bool merged = false;                 // hits/cigar/read_off hold the last run's segments
    std::vector<bsq_hit> hits;
    std::vector<uint32_t> cigar;
    std::vector<int64_t> read_off;
    bsq_hits view{};
};

namespace {

void release_held(Member &x)
{
    for (size_t j = 0; j < x.views.size(); ++j) bsq_pipeline_release(x.pipe);
    x.views.clear();
    x.batches.clear();
}

void drop_replicas(bsq_group *g)
{
    g->merged = false;
    g->view = bsq_hits{};
    for (size_t k = 0; k < g->m.size(); ++k) {
        Member &x = g->m[k];
        release_held(x);
        bsq_pipeline_free(x.pipe);
        x.pipe = nullptr;
        x.n = 0;
        x.slo.clear();
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
    if (const char *e = getenv("BSQ_GROUP_RCCL")) g->rccl = g->rccl && atoi(e) != 0;   // 0: peer copies only
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
    for (size_t k = 0; k < G; ++k) {
        int rc = bsq_pipeline_create(g->m[k].index, g->slots, &g->m[k].pipe);
        if (!rc) rc = pipeline_set_record_route(g->m[k].pipe, g->exchange == BSQ_XCHG_VIA_FIRST && k > 0 ? dev0 : -1);
        if (rc) { const std::string m = bsq_last_error(); drop_replicas(g); return fail(rc, m); }
    }
    return BSQ_OK;
}

extern "C" int bsq_group_set_exchange(bsq_group *g, int mode)
{
    if (!g || (mode != BSQ_XCHG_LINKS && mode != BSQ_XCHG_VIA_FIRST)) return fail(BSQ_E_INVALID, "invalid argument");
    g->merged = false;
    g->view = bsq_hits{};
    for (Member &x : g->m) release_held(x);   // the held views' slots must be free to re-route
    g->exchange = mode;
    for (Member &x : g->m) {
        if (!x.pipe) continue;   // not replicated yet: applied at bsq_group_replicate
        // member 0's records take its own link either way (the relay would copy them onto the same device)
        const int rc = pipeline_set_record_route(x.pipe, mode == BSQ_XCHG_VIA_FIRST && &x != &g->m[0] ? g->m[0].device : -1);
        if (rc) return rc;
    }
    return BSQ_OK;
}

extern "C" int bsq_group_set_slots(bsq_group *g, int slots)
{
    if (!g || slots < 1 || slots > 16) return fail(BSQ_E_INVALID, "invalid argument");
    if (g->src) return fail(BSQ_E_INVALID, "set the slots before bsq_group_replicate");
    g->slots = slots;
    return BSQ_OK;
}

static int finish_run(bsq_group *g, int rc);

// One round of a member's shard: share j submitted to slot j (staged from `reads`, or re-run from the slot's
// staging when reads == NULL), then every share taken in order and held.
static int member_round(Member &x, const bsq_opts *opts, const void *const *reads, uint64_t first_call_seq)
{
    if (x.n == 0) return BSQ_OK;
    const int s = (int)x.slo.size() - 1;
    int rc = pipeline_rewind(x.pipe), submitted = 0;   // share j on slot j (a re-run finds its staging there)
    for (int j = 0; j < s && rc == BSQ_OK; ++j) {
        const int32_t a = x.lo + x.slo[(size_t)j], n = x.slo[(size_t)j + 1] - x.slo[(size_t)j];
        rc = reads ? pipeline_submit_ex(x.pipe, opts, reads + a, n, first_call_seq + (uint64_t)a, 0, PipeMode::DEFER)
                   : pipeline_submit_ex(x.pipe, opts, nullptr, n, first_call_seq + (uint64_t)a, 0, PipeMode::RERUN);
        if (rc == BSQ_OK) ++submitted;
    }
    std::string err;
    for (int j = 0; j < submitted; ++j) {   // every submission is taken, failed or not
        const bsq_hits *v = nullptr;
        bsq_batch *b = nullptr;
        const int r = pipeline_next_ex(x.pipe, &v, nullptr, nullptr, &b);
        if (r) { if (rc == BSQ_OK) { rc = r; err = bsq_last_error(); } continue; }
        x.views.push_back(v);
        x.batches.push_back(b);
    }
    if (rc != BSQ_OK) {
        if (!err.empty()) bsq_internal_set_error(err.c_str());
        const std::string m = bsq_last_error();
        release_held(x);
        bsq_internal_set_error(m.c_str());
    }
    return rc;
}

extern "C" int bsq_group_run(bsq_group *g, const bsq_opts *opts, const void *const *reads, int32_t n_reads,
                             uint64_t first_call_seq)
{
    if (!g || !opts) return fail(BSQ_E_INVALID, "invalid argument");
    if (!g->src) return fail(BSQ_E_INVALID, "no index replicated on the group (bsq_group_replicate)");
    const size_t G = g->m.size();
    g->merged = false;
    g->view = bsq_hits{};
    for (Member &x : g->m) release_held(x);
    if (reads) {
        if (n_reads < 0) return fail(BSQ_E_INVALID, "invalid argument");
        for (int32_t i = 0; i < n_reads; ++i)
            if (!reads[i]) return fail(BSQ_E_INVALID, "read " + std::to_string(i) + " is NULL");
        g->n_reads = n_reads;
        const int64_t min_share = 32768;   // smaller shares lose more to stage tails than concurrency gains
        for (size_t k = 0; k < G; ++k) {
            Member &x = g->m[k];
            x.lo = (int32_t)((int64_t)n_reads * (int64_t)k / (int64_t)G);
            x.n = (int32_t)((int64_t)n_reads * (int64_t)(k + 1) / (int64_t)G) - x.lo;
            const int s = (int)std::max<int64_t>(1, std::min<int64_t>(g->slots, ((int64_t)x.n + min_share - 1) / min_share));
            x.slo.assign((size_t)s + 1, 0);
            for (int j = 0; j <= s; ++j) x.slo[(size_t)j] = (int32_t)((int64_t)x.n * j / s);
        }
    } else if (n_reads != g->n_reads) return fail(BSQ_E_INVALID, "re-run of a different read count");
    const int rc = for_members(g, [&](int k) -> int { return member_round(g->m[(size_t)k], opts, reads, first_call_seq); });
    return finish_run(g, rc);
}

extern "C" int bsq_group_run_rounds(bsq_group *g, const bsq_opts *opts, int32_t n_reads, uint64_t first_call_seq, int rounds)
{
    if (!g || !opts || rounds < 1) return fail(BSQ_E_INVALID, "invalid argument");
    if (!g->src) return fail(BSQ_E_INVALID, "no index replicated on the group (bsq_group_replicate)");
    if (n_reads != g->n_reads) return fail(BSQ_E_INVALID, "re-run of a different read count");
    g->merged = false;
    g->view = bsq_hits{};
    const int rc = for_members(g, [&](int k) -> int {
        Member &x = g->m[(size_t)k];
        const int s = (int)x.slo.size() - 1;
        if (x.n == 0 || s < 1) return BSQ_OK;
        int todo = rounds;
        bool held = (int)x.batches.size() == s;
        for (bsq_batch *b : x.batches) held = held && b;
        if (!held) {   // the previous run's shares are not all held on their batches: one staged round first
            release_held(x);
            const int r = member_round(x, opts, nullptr, first_call_seq);
            if (r || --todo == 0) return r;
        }
        // The shares' batches (held since the last run, reads resident) run bsq_batch_run_rounds' schedule: each
        // share's thread starts its next round as soon as its last one ends, so the shares drift out of phase and
        // one's seeding overlaps the others' DP stages (the pipeline's in-order turns would keep them in step).
        std::vector<uint64_t> fc((size_t)s);
        for (int j = 0; j < s; ++j) fc[(size_t)j] = first_call_seq + (uint64_t)(x.lo + x.slo[(size_t)j]);
        const int r = bsq_batch_run_rounds(x.batches.data(), s, opts, fc.data(), todo);
        if (r) release_held(x);
        return r;
    });
    return finish_run(g, rc);
}

static int finish_run(bsq_group *g, int rc)
{
    if (rc) {
        for (Member &x : g->m) release_held(x);
        return rc;
    }
    int64_t nc = 0;
    for (const Member &x : g->m)
        for (const bsq_hits *v : x.views) nc += v->n_cigar;
    if ((uint64_t)nc > UINT32_MAX) {
        for (Member &x : g->m) release_held(x);
        return fail(BSQ_E_UNSUPPORTED, "more than 2^32 CIGAR operations in one call");
    }
    return BSQ_OK;
}

extern "C" int bsq_group_segments(const bsq_group *g, const bsq_hits **views, int32_t *read_lo, int max)
{
    if (!g || max < 0 || (max > 0 && (!views || !read_lo))) return fail(BSQ_E_INVALID, "invalid argument");
    int n = 0;
    for (const Member &x : g->m)
        for (size_t j = 0; j < x.views.size(); ++j, ++n)
            if (n < max) { views[n] = x.views[j]; read_lo[n] = x.lo + x.slo[j]; }
    return n;
}

// the merged view of the last run (segments concatenated in read order; one host thread per segment)
static int merge(bsq_group *g)
{
    std::vector<const bsq_hits *> v;
    std::vector<int32_t> rlo;
    for (const Member &x : g->m)
        for (size_t j = 0; j < x.views.size(); ++j) { v.push_back(x.views[j]); rlo.push_back(x.lo + x.slo[j]); }
    const size_t S = v.size();
    std::vector<int64_t> hb(S + 1, 0), cb(S + 1, 0);
    for (size_t j = 0; j < S; ++j) { hb[j + 1] = hb[j] + v[j]->n_hits; cb[j + 1] = cb[j] + v[j]->n_cigar; }
    try {
        g->hits.resize((size_t)hb[S]);
        g->cigar.resize((size_t)cb[S]);
        g->read_off.assign((size_t)g->n_reads + 1, 0);
    } catch (const std::bad_alloc &) {
        return fail(BSQ_E_NOMEM, "out of host memory for the merged records");
    }
    auto one = [&](size_t j) {
        const bsq_hits &x = *v[j];
        bsq_hit *dst = g->hits.data() + hb[j];
        if (x.n_hits) memcpy(dst, x.hits, sizeof(bsq_hit) * (size_t)x.n_hits);
        for (int64_t i = 0; i < x.n_hits; ++i) {
            dst[i].read_index += rlo[j];
            dst[i].cigar_off += (uint32_t)cb[j];
        }
        if (x.n_cigar) memcpy(g->cigar.data() + cb[j], x.cigar, 4 * (size_t)x.n_cigar);
        for (int32_t i = 0; i < x.n_reads; ++i) g->read_off[(size_t)rlo[j] + (size_t)i] = hb[j] + x.read_off[i] - x.read_off[0];
    };
    std::vector<std::thread> th;
    for (size_t j = 1; j < S; ++j) th.emplace_back(one, j);
    if (S) one(0);
    for (auto &t : th) t.join();
    g->read_off[(size_t)g->n_reads] = hb[S];
    g->view.n_reads = g->n_reads;
    g->view.n_hits = hb[S];
    g->view.hits = g->hits.data();
    g->view.read_off = g->read_off.data();
    g->view.n_cigar = cb[S];
    g->view.cigar = g->cigar.data();
    g->merged = true;
    return BSQ_OK;
}

extern "C" const bsq_hits *bsq_group_hits(const bsq_group *cg)
{
    if (!cg) return nullptr;
    bsq_group *g = const_cast<bsq_group *>(cg);   // the merge is a cache of the segments
    if (!g->merged && g->src && merge(g) != BSQ_OK) return nullptr;
    return &g->view;
}

extern "C" int bsq_group_render_nuclseqs(bsq_group *g, const void *const *reads, uint8_t **out, int64_t **out_off)
{
    if (!g || !out || !out_off || (g->n_reads && !reads)) return fail(BSQ_E_INVALID, "invalid argument");
    *out = nullptr;
    *out_off = nullptr;
    const size_t G = g->m.size();
    struct Part { uint8_t *buf = nullptr; int64_t *off = nullptr; int64_t nv = 0; };
    std::vector<std::vector<Part>> part(G);
    for (size_t k = 0; k < G; ++k) part[k].resize(g->m[k].views.size());
    const int rc = for_members(g, [&](int k) -> int {
        const Member &x = g->m[(size_t)k];
        for (size_t j = 0; j < x.views.size(); ++j) {
            if (!x.batches[j] || !x.views[j]->n_hits) continue;
            Part &q = part[(size_t)k][j];
            q.nv = 2 * x.views[j]->n_hits;
            const int r = bsq_batch_render_nuclseqs(x.batches[j], reads + x.lo + x.slo[j], &q.buf, &q.off);
            if (r) return r;
        }
        return BSQ_OK;
    });
    auto release = [&] { for (auto &v : part) for (Part &q : v) { bsq_free(q.buf); bsq_free(q.off); } };
    if (rc) { release(); return rc; }
    int64_t nv = 0, bytes = 0;
    for (auto &v : part)
        for (Part &q : v) { nv += q.nv; bytes += q.nv ? ((q.off[q.nv] + 7) & ~7LL) : 0; }
    uint8_t *buf = static_cast<uint8_t *>(malloc((size_t)std::max<int64_t>(bytes, 1)));
    int64_t *off = static_cast<int64_t *>(malloc(((size_t)nv + 1) * 8));
    if (!buf || !off) { free(buf); free(off); release(); return fail(BSQ_E_NOMEM, "out of host memory"); }
    int64_t v0 = 0, base = 0;
    for (auto &v : part)
        for (Part &q : v) {
            if (!q.nv) continue;
            memcpy(buf + base, q.buf, (size_t)q.off[q.nv]);
            for (int64_t i = 0; i < q.nv; ++i) off[v0 + i] = base + q.off[i];
            v0 += q.nv;
            base += (q.off[q.nv] + 7) & ~7LL;
        }
    off[nv] = base;
    release();
    *out = buf;
    *out_off = off;
    return BSQ_OK;
}
