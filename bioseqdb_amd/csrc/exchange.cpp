// exchange.cpp -- the record exchange of the one-process-per-GPU driver (include/bsq.h bsq_xchg_*).
//
// SURVEY.md 8(e) / north_star: a cursor batch is sharded read-parallel over the GPUs of a node and every rank's hit
// records return to the caller -- the backend that runs nuclseq_multi_search_bwa (bioseqdb/extension.cpp:362-370
// puts every row into its tuplestore), here rank 0.  Under torchrun each rank is a process, so the records cross
// between processes by RCCL over xGMI.
//
// The orchestration -- one exchange thread per rank issuing every (round, lane)'s header all-gather and send/recv in
// one fixed global order, failure propagation through the header's status word -- is exchange_core.h's Core, shared
// with the host-memory simulation of tests/xchg_sim.cpp.  This file is its RCCL transport: ONE communicator and ONE
// HIP stream per rank (every collective of the rank in one order on one queue), per-lane receive buffers (rank 0's
// view of each lane's last round), per-lane `packed`/`sent` events that order a send after its batch's pack and the
// batch's next round after the send.  Host waits on the exchange stream poll with a deadline (BSQ_XCHG_TIMEOUT_S,
// default 600 s); on a timeout, a transport error or a failure any rank reports, the communicator is aborted
// (ncclCommAbort), so a broken rank ends the job instead of hanging it.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/bsq.h"
#include "bsq_internal.h"
#include "bsq_index.h"
#include "exchange_core.h"

extern "C" void bsq_internal_set_error(const char *msg);

namespace {

using bsq::xchg::Parts;
using bsq::xchg::Records;

int fail(int rc, const std::string &m)
{
    bsq_internal_set_error(m.c_str());
    return rc;
}

#define XHIP(x)                                                                                              \
    do {                                                                                                     \
        const hipError_t e_ = (x);                                                                           \
        if (e_ != hipSuccess) return fail(BSQ_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_));        \
    } while (0)
#define XNCCL(x)                                                                                             \
    do {                                                                                                     \
        const ncclResult_t r_ = (x);                                                                         \
        if (r_ != ncclSuccess) return fail(BSQ_E_HIP, std::string(#x) + ": " + ncclGetErrorString(r_));      \
    } while (0)
// inside the transport: the message goes to the Core's error string
#define THIP(x)                                                                                              \
    do {                                                                                                     \
        const hipError_t e_ = (x);                                                                           \
        if (e_ != hipSuccess) { err = std::string(#x) + ": " + hipGetErrorString(e_); return BSQ_E_HIP; }    \
    } while (0)
#define TNCCL(x)                                                                                             \
    do {                                                                                                     \
        const ncclResult_t r_ = (x);                                                                         \
        if (r_ != ncclSuccess) { err = std::string(#x) + ": " + ncclGetErrorString(r_); return BSQ_E_HIP; }  \
    } while (0)

struct Lane {
    hipStream_t bs = nullptr;        // the lane's batch stream (set by every round's produce)
    hipEvent_t packed = nullptr;     // on bs: the round's records are final
    hipEvent_t sent = nullptr;       // on xs: the send buffers may be overwritten
    bool has_sent = false;
    uint8_t *send_dev = nullptr;     // the round's wire form (bsq_internal.h WireHit): header + counts, hits, CIGAR words
    int64_t send_cap = 0;
    uint8_t *stage_dev = nullptr;    // a host-resident view (a round with retried reads) copied to HBM before packing
    int64_t stage_cap = 0;
    uint8_t *recv_dev = nullptr;     // rank 0: every other rank's parts
    int64_t recv_cap = 0;
    uint8_t *recv_host = nullptr;    // rank 0: the same, pinned (the caller's view of the last round)
    int64_t recv_host_cap = 0;
};

template <typename T>
int grow(T *&p, int64_t &cap, int64_t need, bool pinned, std::string &err)
{
    if (need <= cap) return BSQ_OK;
    const int64_t c = std::max<int64_t>(need + need / 4, 1 << 20);
    if (pinned) { hipHostFree(p); p = nullptr; THIP(hipHostMalloc((void **)&p, (size_t)c)); }
    else { hipFree(p); p = nullptr; THIP(hipMalloc((void **)&p, (size_t)c)); }
    cap = c;
    return BSQ_OK;
}

class RcclTransport final : public bsq::xchg::Transport {
  public:
    int world_ = 1, rank_ = 0, device_ = 0;
    ncclComm_t comm = nullptr;
    hipStream_t xs = nullptr;
    int64_t *hdr_dev = nullptr;    // world x 4
    int64_t *hdr_host = nullptr;   // pinned
    std::vector<Lane> lanes;
    double timeout_s = 600;
    bool aborted = false;

    int world() const override { return world_; }
    int rank() const override { return rank_; }

    // host wait for everything issued on xs so far, with a deadline (a peer that never joins must not hang us)
    int sync_xs(std::string &err)
    {
        const auto t0 = std::chrono::steady_clock::now();
        for (int spin = 0;; ++spin) {
            const hipError_t e = hipStreamQuery(xs);
            if (e == hipSuccess) return BSQ_OK;
            if (e != hipErrorNotReady) { err = std::string("exchange stream: ") + hipGetErrorString(e); return BSQ_E_HIP; }
            ncclResult_t async = ncclSuccess;
            if (ncclCommGetAsyncError(comm, &async) == ncclSuccess && async != ncclSuccess && async != ncclInProgress) {
                err = std::string("RCCL: ") + ncclGetErrorString(async);
                return BSQ_E_HIP;
            }
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) {
                err = "timed out after " + std::to_string((int)timeout_s) + " s waiting for the other ranks (BSQ_XCHG_TIMEOUT_S)";
                return BSQ_E_HIP;
            }
            if (spin < 2000) std::this_thread::yield();
            else std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
    }

    // the exchange thread waiting for a lane to publish: RCCL's asynchronous error, and the same deadline as sync_xs
    // (a lane whose stream waits on an unmatched send blocks in its next HIP call; abort() then releases it)
    int poll(double waited_s, std::string &err) override
    {
        ncclResult_t async = ncclSuccess;
        if (comm && ncclCommGetAsyncError(comm, &async) == ncclSuccess && async != ncclSuccess && async != ncclInProgress) {
            err = std::string("RCCL: ") + ncclGetErrorString(async);
            return BSQ_E_HIP;
        }
        if (waited_s > timeout_s) {
            err = "timed out after " + std::to_string((int)timeout_s) +
                  " s waiting for a local batch (its stream may wait on a send no other rank matched; BSQ_XCHG_TIMEOUT_S)";
            return BSQ_E_HIP;
        }
        return BSQ_OK;
    }

    int all_gather(int, const int64_t mine[4], int64_t *all, std::string &err) override
    {
        THIP(hipSetDevice(device_));
        int64_t *h = hdr_host + 4 * rank_;
        memcpy(h, mine, 32);
        THIP(hipMemcpyAsync(hdr_dev + 4 * rank_, h, 32, hipMemcpyHostToDevice, xs));
        TNCCL(ncclAllGather(hdr_dev + 4 * rank_, hdr_dev, 4, ncclInt64, comm, xs));
        THIP(hipMemcpyAsync(hdr_host, hdr_dev, (size_t)world_ * 32, hipMemcpyDeviceToHost, xs));
        if (const int rc = sync_xs(err)) return rc;
        memcpy(all, hdr_host, (size_t)world_ * 32);
        return BSQ_OK;
    }

    // The round's records go out in the wire form (bsq_internal.h WireHit, 32 B per hit + 4 B per read instead of
    // 72 + 8): k_wire_pack on the exchange stream turns the batch's packed records into it, and rank 0 expands it on
    // its host (bsq_xchg_view).  The bytes through rank 0's one PCIe link are what the 8-rank exchange funnels.
    int send(int li, const Records &r, const Parts &p, std::string &err) override
    {
        Lane &l = lanes[(size_t)li];
        THIP(hipSetDevice(device_));
        if (p.total() > l.send_cap) { if (const int rc = sync_xs(err)) return rc; }   // the old buffer may be in flight
        if (const int rc = grow(l.send_dev, l.send_cap, p.total(), false, err)) return rc;
        const void *off = r.off, *hits = r.hits, *cig = r.cig;
        if (!r.on_device) {   // the view is in pinned host memory: copy it to HBM first (same stream)
            const int64_t ob = (r.n_reads + 1) * 8, need = bsq::xchg::al(ob) + r.n_hits * (int64_t)sizeof(bsq_hit);
            if (need > l.stage_cap) { if (const int rc = sync_xs(err)) return rc; }
            if (const int rc = grow(l.stage_dev, l.stage_cap, need, false, err)) return rc;
            THIP(hipMemcpyAsync(l.stage_dev, r.off, (size_t)ob, hipMemcpyHostToDevice, xs));
            if (p.n_hits) THIP(hipMemcpyAsync(l.stage_dev + bsq::xchg::al(ob), r.hits, (size_t)(r.n_hits * sizeof(bsq_hit)),
                                              hipMemcpyHostToDevice, xs));
            if (p.n_cigar) THIP(hipMemcpyAsync(l.send_dev + p.o_cig(), r.cig, (size_t)p.cig_bytes(), hipMemcpyHostToDevice, xs));
            off = l.stage_dev; hits = l.stage_dev + bsq::xchg::al(ob); cig = l.send_dev + p.o_cig();
        } else {   // straight from the batch's packed arrays: the pack waits for the batch stream's pack
            THIP(hipStreamWaitEvent(xs, l.packed, 0));
        }
        if (bsq::launch_wire_pack(xs, (int32_t)p.n_reads, static_cast<const int64_t *>(off), static_cast<const bsq_hit *>(hits),
                                  l.send_dev, reinterpret_cast<bsq::WireHit *>(l.send_dev + p.o_hit())) != BSQ_OK) {
            err = "k_wire_pack launch failed";
            return BSQ_E_HIP;
        }
        // the batch's next run may regrow (free) the pinned view the staging copies read
        if (!r.on_device) { if (const int rc = sync_xs(err)) return rc; }
        TNCCL(ncclGroupStart());
        TNCCL(ncclSend(l.send_dev, (size_t)p.off_bytes(), ncclUint8, 0, comm, xs));
        if (p.n_hits) TNCCL(ncclSend(l.send_dev + p.o_hit(), (size_t)p.hits_bytes(), ncclUint8, 0, comm, xs));
        if (p.n_cigar) TNCCL(ncclSend(cig, (size_t)p.cig_bytes(), ncclUint8, 0, comm, xs));
        TNCCL(ncclGroupEnd());
        THIP(hipEventRecord(l.sent, xs));
        l.has_sent = true;
        return BSQ_OK;
    }

    int recv(int li, const std::vector<Parts> &parts, const std::vector<int64_t> &at, int64_t total, std::string &err) override
    {
        Lane &l = lanes[(size_t)li];
        THIP(hipSetDevice(device_));
        if (total > l.recv_cap || total > l.recv_host_cap) { if (const int rc = sync_xs(err)) return rc; }
        if (const int rc = grow(l.recv_dev, l.recv_cap, total, false, err)) return rc;
        if (const int rc = grow(l.recv_host, l.recv_host_cap, total, true, err)) return rc;
        TNCCL(ncclGroupStart());
        for (int k = 1; k < world_; ++k) {
            const Parts &p = parts[(size_t)k];
            uint8_t *d = l.recv_dev + at[(size_t)k];
            TNCCL(ncclRecv(d, (size_t)p.off_bytes(), ncclUint8, k, comm, xs));
            if (p.n_hits) TNCCL(ncclRecv(d + p.o_hit(), (size_t)p.hits_bytes(), ncclUint8, k, comm, xs));
            if (p.n_cigar) TNCCL(ncclRecv(d + p.o_cig(), (size_t)p.cig_bytes(), ncclUint8, k, comm, xs));
        }
        TNCCL(ncclGroupEnd());
        if (total) THIP(hipMemcpyAsync(l.recv_host, l.recv_dev, (size_t)total, hipMemcpyDeviceToHost, xs));
        return BSQ_OK;
    }

    int batch_resume(int li, std::string &err) override
    {
        Lane &l = lanes[(size_t)li];
        if (l.has_sent && l.bs) THIP(hipStreamWaitEvent(l.bs, l.sent, 0));   // the next round overwrites the sent arrays
        return BSQ_OK;
    }

    void abort() override
    {
        if (comm && !aborted) ncclCommAbort(comm);
        aborted = true;
        comm = nullptr;
    }

    ~RcclTransport()
    {
        hipSetDevice(device_);
        if (xs && !aborted) hipStreamSynchronize(xs);
        if (comm) ncclCommDestroy(comm);
        for (Lane &l : lanes) {
            hipFree(l.send_dev); hipFree(l.stage_dev); hipFree(l.recv_dev); hipHostFree(l.recv_host);
            if (l.packed) hipEventDestroy(l.packed);
            if (l.sent) hipEventDestroy(l.sent);
        }
        hipFree(hdr_dev); hipHostFree(hdr_host);
        if (xs) hipStreamDestroy(xs);
    }
};

}  // namespace

struct bsq_xchg {
    std::unique_ptr<RcclTransport> t;
    std::unique_ptr<bsq::xchg::Core> core;
    // rank 0: the index's anns (bsq_xchg_set_index) and the views expanded from the wire form, per (lane, rank)
    std::vector<int64_t> ann_off, ann_id;
    struct View { int64_t round = -1; std::vector<int64_t> off; std::vector<bsq_hit> hits; };
    mutable std::mutex view_mu;
    mutable std::vector<View> views;   // lane * world + rank
};

extern "C" int bsq_xchg_unique_id(void *id)
{
    if (!id) return fail(BSQ_E_INVALID, "invalid argument");
    ncclUniqueId u;
    XNCCL(ncclGetUniqueId(&u));
    memcpy(id, &u, sizeof u);
    return BSQ_OK;
}

extern "C" int bsq_xchg_create(int world, int rank, int device, const void *id, int lanes, bsq_xchg **out)
{
    if (!out || !id || world < 1 || rank < 0 || rank >= world || lanes < 1 || lanes > 64)
        return fail(BSQ_E_INVALID, "invalid argument");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return fail(BSQ_E_NODEV, "no HIP device " + std::to_string(device));
    std::unique_ptr<bsq_xchg> x(new (std::nothrow) bsq_xchg());
    if (!x) return fail(BSQ_E_NOMEM, "out of memory");
    x->t.reset(new RcclTransport());
    RcclTransport &t = *x->t;
    t.world_ = world; t.rank_ = rank; t.device_ = device;
    if (const char *s = getenv("BSQ_XCHG_TIMEOUT_S")) { const double v = atof(s); if (v > 0) t.timeout_s = v; }
    XHIP(hipSetDevice(device));
    XHIP(hipStreamCreateWithFlags(&t.xs, hipStreamNonBlocking));
    XHIP(hipMalloc(&t.hdr_dev, (size_t)world * 32));
    XHIP(hipHostMalloc((void **)&t.hdr_host, (size_t)world * 32));
    t.lanes.resize((size_t)lanes);
    for (Lane &l : t.lanes) {
        XHIP(hipEventCreateWithFlags(&l.packed, hipEventDisableTiming));
        XHIP(hipEventCreateWithFlags(&l.sent, hipEventDisableTiming));
    }
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    XNCCL(ncclCommInitRank(&t.comm, world, u, rank));
    x->core.reset(new bsq::xchg::Core(t, lanes, (int64_t)sizeof(bsq::WireHit), 4, bsq::kWireHead));
    x->views.resize((size_t)lanes * (size_t)world);
    *out = x.release();
    return BSQ_OK;
}

extern "C" void bsq_xchg_free(bsq_xchg *x)
{
    if (!x) return;
    x->core.reset();
    x->t.reset();
    delete x;
}

extern "C" int bsq_batch_run_rounds_x(bsq_batch *const *batches, int n, const bsq_opts *opts, const uint64_t *first_call,
                                      int rounds, bsq_xchg *x)
{
    if (!x) return bsq_batch_run_rounds(batches, n, opts, first_call, rounds);
    if (n < 1 || rounds < 0 || !batches || !opts || !first_call) return fail(BSQ_E_INVALID, "invalid argument");
    if (n != x->core->n_lanes()) return fail(BSQ_E_INVALID, "one exchange lane per batch expected");
    if (x->core->aborted()) return fail(BSQ_E_INVALID, "the exchange was aborted by an earlier failure");
    RcclTransport &t = *x->t;
    std::vector<std::string> msg((size_t)n);
    // fault injection for the failure path's tests: BSQ_XCHG_TEST_FAIL="lane:round" fails that batch run on this rank
    int fail_lane = -1, fail_round = -1;
    if (const char *f = getenv("BSQ_XCHG_TEST_FAIL")) sscanf(f, "%d:%d", &fail_lane, &fail_round);
    auto produce = [&](int i, int k, Records &rec) -> int {
        roctxRangePushA("bsq_batch_round_x");
        int rc = (i == fail_lane && k == fail_round) ? (bsq_internal_set_error("injected failure (BSQ_XCHG_TEST_FAIL)"), BSQ_E_INVALID)
                                                     : bsq_batch_run(batches[i], opts, first_call[i]);
        if (!rc) {
            const bsq::BatchRecords r = bsq::batch_records(batches[i]);
            Lane &l = t.lanes[(size_t)i];
            l.bs = static_cast<hipStream_t>(r.stream);
            if (hipEventRecord(l.packed, l.bs) != hipSuccess) { rc = BSQ_E_HIP; bsq_internal_set_error("hipEventRecord(packed)"); }
            rec.n_reads = r.n_reads; rec.n_hits = r.n_hits; rec.n_cigar = r.n_cigar;
            rec.off = r.off; rec.hits = r.hits; rec.cig = r.cig; rec.on_device = r.on_device;
        }
        if (rc) msg[(size_t)i] = bsq_last_error();
        roctxRangePop();
        return rc;
    };
    std::string err;
    const int rc = x->core->run(rounds, produce, err);
    if (rc) {
        for (int i = 0; i < n; ++i)
            if (!msg[(size_t)i].empty()) err += "; local batch " + std::to_string(i) + ": " + msg[(size_t)i];
        return fail(rc, err);
    }
    return BSQ_OK;
}

extern "C" int bsq_xchg_finish(bsq_xchg *x, int64_t *bytes_moved, double *wait_ms)
{
    if (!x) return fail(BSQ_E_INVALID, "invalid argument");
    RcclTransport &t = *x->t;
    XHIP(hipSetDevice(t.device_));
    if (!x->core->aborted()) {
        std::string err;
        if (const int rc = t.sync_xs(err)) { t.abort(); return fail(rc, err); }
    }
    int64_t moved = 0;
    for (int i = 0; i < x->core->n_lanes(); ++i) moved += x->core->lane(i).bytes;
    if (bytes_moved) *bytes_moved = moved;
    if (wait_ms) *wait_ms = x->core->wait_ms();
    return BSQ_OK;
}

extern "C" int bsq_xchg_view(const bsq_xchg *x, int lane, int src_rank, bsq_hits *out)
{
    if (!x || !out || lane < 0 || lane >= x->core->n_lanes() || src_rank < 0 || src_rank >= x->t->world_)
        return fail(BSQ_E_INVALID, "invalid argument");
    if (x->t->rank_ != 0 || src_rank == 0) return fail(BSQ_E_INVALID, "rank 0 holds the other ranks' records (its own are in its batches)");
    const bsq::xchg::LaneState &ls = x->core->lane(lane);
    if (!ls.rounds) return fail(BSQ_E_INVALID, "no round exchanged yet");
    if (x->ann_off.empty()) return fail(BSQ_E_INVALID, "bsq_xchg_view: no index set (bsq_xchg_set_index) to expand the records with");
    const Parts &p = ls.parts[(size_t)src_rank];
    uint8_t *h = x->t->lanes[(size_t)lane].recv_host + ls.at[(size_t)src_rank];
    std::lock_guard<std::mutex> lk(x->view_mu);
    bsq_xchg::View &v = x->views[(size_t)lane * (size_t)x->t->world_ + (size_t)src_rank];
    if (v.round != ls.rounds) {   // expanded once per exchanged round
        v.off.resize((size_t)p.n_reads + 1);
        v.hits.resize((size_t)std::max<int64_t>(p.n_hits, 1));
        bsq::wire_expand(h, reinterpret_cast<const bsq::WireHit *>(h + p.o_hit()), (int32_t)p.n_reads, x->ann_off.data(),
                         x->ann_id.data(), (int64_t)x->ann_off.size(), v.off.data(), v.hits.data());
        v.round = ls.rounds;
    }
    *out = bsq_hits{};
    out->n_reads = (int32_t)p.n_reads;
    out->n_hits = p.n_hits;
    out->read_off = v.off.data();
    out->hits = v.hits.data();
    out->n_cigar = p.n_cigar;
    out->cigar = reinterpret_cast<uint32_t *>(h + p.o_cig());
    return BSQ_OK;
}

extern "C" int bsq_xchg_set_index(bsq_xchg *x, const bsq_index *idx)
{
    if (!x || !idx) return fail(BSQ_E_INVALID, "invalid argument");
    const std::vector<bsq::Ann> &a = idx->h.anns;
    x->ann_off.assign(std::max<size_t>(a.size(), 1), 0);
    x->ann_id.assign(std::max<size_t>(a.size(), 1), 0);
    for (size_t i = 0; i < a.size(); ++i) { x->ann_off[i] = a[i].offset; x->ann_id[i] = a[i].id; }
    return BSQ_OK;
}

namespace bsq {

void wire_expand(const uint8_t *off_part, const WireHit *wire, int32_t n_reads, const int64_t *ann_off, const int64_t *ann_id,
                 int64_t n_anns, int64_t *read_off, bsq_hit *hits)
{
    int64_t read_base = 0, cig = 0;
    memcpy(&read_base, off_part, 8);
    memcpy(&cig, off_part + 8, 8);
    const uint8_t *cnt = off_part + kWireHead;
    int64_t g = 0;
    read_off[0] = 0;
    for (int32_t i = 0; i < n_reads; ++i) {
        int32_t c;
        memcpy(&c, cnt + 4 * (size_t)i, 4);
        for (int32_t k = 0; k < c; ++k, ++g) {
            const WireHit &w = wire[g];
            bsq_hit &b = hits[g];
            memset(&b, 0, sizeof b);   // k_pack zeroes the padding: records compare byte for byte
            const int64_t roff = w.rid >= 0 && w.rid < n_anns ? ann_off[w.rid] : 0;
            b.ref_id = w.rid >= 0 && w.rid < n_anns ? ann_id[w.rid] : 0;
            b.rb = w.rb;
            b.re = w.rb + w.len;
            b.ref_match_start = (int32_t)(b.rb - roff);
            b.ref_match_end = (int32_t)(b.re - roff);
            b.ref_match_len = w.len;
            b.qb = w.qb; b.qe = w.qe; b.score = w.score; b.rid = w.rid;
            b.is_primary = (uint8_t)(w.ncig >> 29 & 1); b.is_secondary = (uint8_t)(w.ncig >> 30 & 1);
            b.is_reverse = (uint8_t)(w.ncig >> 31 & 1);
            b.read_index = (int32_t)(read_base + i);
            b.n_cigar = w.ncig & ((1u << 29) - 1);
            b.cigar_off = (uint32_t)cig;
            cig += b.n_cigar;
        }
        read_off[i + 1] = g;
    }
}

}  // namespace bsq

// The wire form checked on one GPU (the exchange's send half runs only with peers): the batch's last records through
// the same k_wire_pack the send path launches, back to the host, expanded as rank 0's views are, and compared byte
// for byte with the batch's own view.  *wire_bytes / *raw_bytes: what one (round, lane) puts on the link now / as
// bsq_hit records with int64 offsets.
extern "C" int bsq_xchg_wire_check(bsq_batch *b, const bsq_index *idx, int64_t *wire_bytes, int64_t *raw_bytes,
                                   int64_t *mismatches)
{
    if (!b || !idx || !mismatches) return fail(BSQ_E_INVALID, "invalid argument");
    const bsq::BatchRecords r = bsq::batch_records(b);
    const bsq_hits *view = bsq_batch_hits(b);
    if (!view) return fail(BSQ_E_INVALID, "the batch has no records");
    XHIP(hipSetDevice(r.device));
    hipStream_t st = static_cast<hipStream_t>(r.stream);
    Parts p;
    p.n_reads = r.n_reads; p.n_hits = r.n_hits; p.n_cigar = r.n_cigar;
    p.hit_bytes = (int64_t)sizeof(bsq::WireHit); p.off_per_read = 4; p.off_fixed = bsq::kWireHead;
    const int64_t ob = (r.n_reads + 1) * 8, hb = r.n_hits * (int64_t)sizeof(bsq_hit);
    uint8_t *dev = nullptr, *stage = nullptr;
    std::vector<uint8_t> host((size_t)p.o_cig());
    auto done = [&](int rc) { hipFree(dev); hipFree(stage); return rc; };
    if (hipMalloc(&dev, (size_t)std::max<int64_t>(p.o_cig(), 1)) != hipSuccess) return done(fail(BSQ_E_NOMEM, "hipMalloc"));
    const void *off = r.off, *hits = r.hits;
    if (!r.on_device) {
        if (hipMalloc(&stage, (size_t)(bsq::xchg::al(ob) + std::max<int64_t>(hb, 1))) != hipSuccess) return done(fail(BSQ_E_NOMEM, "hipMalloc"));
        if (hipMemcpyAsync(stage, r.off, (size_t)ob, hipMemcpyHostToDevice, st) != hipSuccess ||
            (hb && hipMemcpyAsync(stage + bsq::xchg::al(ob), r.hits, (size_t)hb, hipMemcpyHostToDevice, st) != hipSuccess))
            return done(fail(BSQ_E_HIP, "staging copy"));
        off = stage; hits = stage + bsq::xchg::al(ob);
    }
    if (bsq::launch_wire_pack(st, (int32_t)p.n_reads, static_cast<const int64_t *>(off), static_cast<const bsq_hit *>(hits),
                              dev, reinterpret_cast<bsq::WireHit *>(dev + p.o_hit())) != BSQ_OK)
        return done(fail(BSQ_E_HIP, "k_wire_pack"));
    if (hipMemcpyAsync(host.data(), dev, host.size(), hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
        return done(fail(BSQ_E_HIP, "wire copy"));
    std::vector<int64_t> ann_off(std::max<size_t>(idx->h.anns.size(), 1), 0), ann_id(ann_off.size(), 0);
    for (size_t i = 0; i < idx->h.anns.size(); ++i) { ann_off[i] = idx->h.anns[i].offset; ann_id[i] = idx->h.anns[i].id; }
    std::vector<int64_t> ro((size_t)p.n_reads + 1);
    std::vector<bsq_hit> hx((size_t)std::max<int64_t>(p.n_hits, 1));
    bsq::wire_expand(host.data(), reinterpret_cast<const bsq::WireHit *>(host.data() + p.o_hit()), (int32_t)p.n_reads,
                     ann_off.data(), ann_id.data(), (int64_t)ann_off.size(), ro.data(), hx.data());
    int64_t bad = 0;
    for (int64_t i = 0; i <= p.n_reads; ++i) bad += ro[(size_t)i] != view->read_off[i] - view->read_off[0];
    for (int64_t g = 0; g < p.n_hits; ++g) bad += memcmp(&hx[(size_t)g], &view->hits[g], sizeof(bsq_hit)) != 0;
    *mismatches = bad;
    if (wire_bytes) *wire_bytes = p.payload();
    if (raw_bytes) *raw_bytes = ob + hb + p.cig_bytes();
    return done(BSQ_OK);
}
