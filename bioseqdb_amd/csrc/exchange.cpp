// exchange.cpp -- the record exchange of the one-process-per-GPU driver (include/bsq.h bsq_xchg_*).
//
// SURVEY.md 8(e) / north_star: a cursor batch is sharded read-parallel over the GPUs of a node and every rank's hit
// records return to the caller -- the backend that runs nuclseq_multi_search_bwa (bioseqdb/extension.cpp:362-370
// puts every row into its tuplestore), here rank 0.  Under torchrun each rank is a process, so the records cross
// between processes by RCCL over xGMI.
//
// A rank aligns its shard as S concurrent batches, each a stream of rounds (bsq_batch_run_rounds' schedule: a batch
// starts its next round as soon as its previous one ends).  Batch i of every rank is bound to lane i: one RCCL
// communicator, one exchange stream.  After each round of batch i, lane i (1) all-gathers every rank's record
// counts (4 x int64 per rank) and reads them on the host, then (2) each rank r > 0 sends its read offsets, hit
// records and CIGAR words to rank 0 (ncclSend x3 in one group) while rank 0 receives all of them into HBM
// (ncclRecv x3 per rank in one group) and copies them to pinned host memory on the lane's stream.  A lane's
// operations are issued by its batch's host thread only, in the same order on every rank, so lanes never wait on
// each other; the batch's next round waits (on the device) only for its own send to drain.  Rank 0's own records
// reach its host memory inside bsq_batch_run as on one GPU.
//
// Built on the public C-ABI of bsq_api.cpp, bsq_internal.h's batch_records and RCCL.
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
#include "bsq_internal.h"

extern "C" void bsq_internal_set_error(const char *msg);

namespace {

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

constexpr int64_t kAlign = 256;
int64_t al(int64_t x) { return (x + kAlign - 1) & ~(kAlign - 1); }

// One rank's records of one round: read offsets (n_reads + 1), hits, CIGAR words; each part 256-B aligned.
struct Parts {
    int64_t n_reads = 0, n_hits = 0, n_cigar = 0;
    int64_t off_bytes() const { return (n_reads + 1) * 8; }
    int64_t hit_bytes() const { return n_hits * (int64_t)sizeof(bsq_hit); }
    int64_t cig_bytes() const { return n_cigar * 4; }
    int64_t o_hit() const { return al(off_bytes()); }
    int64_t o_cig() const { return o_hit() + al(hit_bytes()); }
    int64_t total() const { return o_cig() + al(cig_bytes()); }
};

struct Lane {
    ncclComm_t comm = nullptr;
    hipStream_t xs = nullptr;
    hipEvent_t packed = nullptr;     // on the batch stream: this round's records are final
    hipEvent_t sent = nullptr;       // on xs: the send buffers may be overwritten
    int64_t *hdr_dev = nullptr;      // world x {n_reads, n_hits, n_cigar, 0}
    int64_t *hdr_host = nullptr;     // pinned
    uint8_t *send_dev = nullptr;     // staging of a host-resident view (a round with retried reads)
    int64_t send_cap = 0;
    uint8_t *recv_dev = nullptr;     // rank 0: every other rank's parts
    int64_t recv_cap = 0;
    uint8_t *recv_host = nullptr;    // rank 0: the same, pinned (the caller's view of the last round)
    int64_t recv_host_cap = 0;
    std::vector<Parts> parts;        // per rank, last round
    std::vector<int64_t> at;         // per rank: offset of its parts in recv_dev / recv_host
    int64_t bytes = 0, rounds = 0;   // bytes received (rank 0) or sent (other ranks) over all rounds
};

}  // namespace

struct bsq_xchg {
    int world = 1, rank = 0, device = 0;
    std::vector<Lane> lanes;
    double wait_ms = 0;               // host time the batch threads spent in the exchange (all lanes)
};

namespace {

void free_lane(Lane &l)
{
    if (l.xs) hipStreamSynchronize(l.xs);
    if (l.comm) ncclCommDestroy(l.comm);
    hipFree(l.hdr_dev); hipHostFree(l.hdr_host); hipFree(l.send_dev); hipFree(l.recv_dev); hipHostFree(l.recv_host);
    if (l.packed) hipEventDestroy(l.packed);
    if (l.sent) hipEventDestroy(l.sent);
    if (l.xs) hipStreamDestroy(l.xs);
    l = Lane{};
}

template <typename T>
int grow(T *&p, int64_t &cap, int64_t need, bool pinned)
{
    if (need <= cap) return BSQ_OK;
    const int64_t c = std::max<int64_t>(need + need / 4, 1 << 20);
    if (pinned) { hipHostFree(p); p = nullptr; XHIP(hipHostMalloc((void **)&p, (size_t)c)); }
    else { hipFree(p); p = nullptr; XHIP(hipMalloc((void **)&p, (size_t)c)); }
    cap = c;
    return BSQ_OK;
}

// The exchange of one round of lane `li`'s batch (called by that batch's host thread right after bsq_batch_run).
int lane_round(bsq_xchg *x, int li, bsq_batch *b)
{
    Lane &l = x->lanes[(size_t)li];
    const bsq::BatchRecords r = bsq::batch_records(b);
    hipStream_t bs = static_cast<hipStream_t>(r.stream);
    XHIP(hipSetDevice(x->device));
    // (1) every rank's counts, on the host of every rank
    int64_t *mine = l.hdr_host + 4 * x->rank;
    mine[0] = r.n_reads; mine[1] = r.n_hits; mine[2] = r.n_cigar; mine[3] = 0;
    XHIP(hipMemcpyAsync(l.hdr_dev + 4 * x->rank, mine, 32, hipMemcpyHostToDevice, l.xs));
    XNCCL(ncclAllGather(l.hdr_dev + 4 * x->rank, l.hdr_dev, 4, ncclInt64, l.comm, l.xs));
    XHIP(hipMemcpyAsync(l.hdr_host, l.hdr_dev, (size_t)x->world * 32, hipMemcpyDeviceToHost, l.xs));
    XHIP(hipStreamSynchronize(l.xs));
    int64_t total = 0;
    for (int k = 0; k < x->world; ++k) {
        Parts &p = l.parts[(size_t)k];
        p.n_reads = l.hdr_host[4 * k]; p.n_hits = l.hdr_host[4 * k + 1]; p.n_cigar = l.hdr_host[4 * k + 2];
        l.at[(size_t)k] = total;
        if (k != 0) total += p.total();
    }
    ++l.rounds;
    if (x->world == 1) return BSQ_OK;
    const ncclDataType_t u8 = ncclUint8;
    if (x->rank != 0) {   // (2) send this rank's parts to rank 0
        const Parts &p = l.parts[(size_t)x->rank];
        const void *off = r.off, *hits = r.hits, *cig = r.cig;
        if (!r.on_device) {   // the view is in pinned host memory: stage it in HBM first (same stream)
            { const int rc = grow(l.send_dev, l.send_cap, p.total(), false); if (rc) return rc; }
            XHIP(hipMemcpyAsync(l.send_dev, r.off, (size_t)p.off_bytes(), hipMemcpyHostToDevice, l.xs));
            if (p.n_hits) XHIP(hipMemcpyAsync(l.send_dev + p.o_hit(), r.hits, (size_t)p.hit_bytes(), hipMemcpyHostToDevice, l.xs));
            if (p.n_cigar) XHIP(hipMemcpyAsync(l.send_dev + p.o_cig(), r.cig, (size_t)p.cig_bytes(), hipMemcpyHostToDevice, l.xs));
            off = l.send_dev; hits = l.send_dev + p.o_hit(); cig = l.send_dev + p.o_cig();
            XHIP(hipStreamSynchronize(l.xs));   // the next run may regrow (free) the pinned view it copies from
        } else {   // straight from the batch's packed arrays: the lane waits for the batch stream's pack
            XHIP(hipEventRecord(l.packed, bs));
            XHIP(hipStreamWaitEvent(l.xs, l.packed, 0));
        }
        XNCCL(ncclGroupStart());
        XNCCL(ncclSend(off, (size_t)p.off_bytes(), u8, 0, l.comm, l.xs));
        if (p.n_hits) XNCCL(ncclSend(hits, (size_t)p.hit_bytes(), u8, 0, l.comm, l.xs));
        if (p.n_cigar) XNCCL(ncclSend(cig, (size_t)p.cig_bytes(), u8, 0, l.comm, l.xs));
        XNCCL(ncclGroupEnd());
        XHIP(hipEventRecord(l.sent, l.xs));
        XHIP(hipStreamWaitEvent(bs, l.sent, 0));   // the batch's next round overwrites the sent arrays
        l.bytes += p.off_bytes() + p.hit_bytes() + p.cig_bytes();
        return BSQ_OK;
    }
    // rank 0: receive every other rank's parts into HBM, then into pinned host memory
    { const int rc = grow(l.recv_dev, l.recv_cap, total, false); if (rc) return rc; }
    { const int rc = grow(l.recv_host, l.recv_host_cap, total, true); if (rc) return rc; }
    XNCCL(ncclGroupStart());
    for (int k = 1; k < x->world; ++k) {
        const Parts &p = l.parts[(size_t)k];
        uint8_t *d = l.recv_dev + l.at[(size_t)k];
        XNCCL(ncclRecv(d, (size_t)p.off_bytes(), u8, k, l.comm, l.xs));
        if (p.n_hits) XNCCL(ncclRecv(d + p.o_hit(), (size_t)p.hit_bytes(), u8, k, l.comm, l.xs));
        if (p.n_cigar) XNCCL(ncclRecv(d + p.o_cig(), (size_t)p.cig_bytes(), u8, k, l.comm, l.xs));
    }
    XNCCL(ncclGroupEnd());
    if (total) XHIP(hipMemcpyAsync(l.recv_host, l.recv_dev, (size_t)total, hipMemcpyDeviceToHost, l.xs));
    l.bytes += total;
    return BSQ_OK;
}

}  // namespace

extern "C" int bsq_xchg_unique_id(void *id)
{
    if (!id) return fail(BSQ_E_INVALID, "invalid argument");
    ncclUniqueId u;
    XNCCL(ncclGetUniqueId(&u));
    memcpy(id, &u, sizeof u);
    return BSQ_OK;
}

extern "C" int bsq_xchg_create(int world, int rank, int device, const void *ids, int lanes, bsq_xchg **out)
{
    if (!out || !ids || world < 1 || rank < 0 || rank >= world || lanes < 1 || lanes > 64)
        return fail(BSQ_E_INVALID, "invalid argument");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return fail(BSQ_E_NODEV, "no HIP device " + std::to_string(device));
    std::unique_ptr<bsq_xchg> x(new (std::nothrow) bsq_xchg());
    if (!x) return fail(BSQ_E_NOMEM, "out of memory");
    x->world = world; x->rank = rank; x->device = device;
    x->lanes.resize((size_t)lanes);
    XHIP(hipSetDevice(device));
    auto cleanup = [&] { for (Lane &l : x->lanes) free_lane(l); };
    for (Lane &l : x->lanes) {
        l.parts.resize((size_t)world);
        l.at.resize((size_t)world);
        hipError_t e = hipStreamCreateWithFlags(&l.xs, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&l.packed, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&l.sent, hipEventDisableTiming);
        if (e == hipSuccess) e = hipMalloc(&l.hdr_dev, (size_t)world * 32);
        if (e == hipSuccess) e = hipHostMalloc((void **)&l.hdr_host, (size_t)world * 32);
        if (e != hipSuccess) { cleanup(); return fail(BSQ_E_HIP, std::string("exchange lane: ") + hipGetErrorString(e)); }
    }
    // every lane's communicator in one group (the ranks join lane by lane in the same order)
    ncclResult_t r = ncclGroupStart();
    for (int k = 0; k < lanes && r == ncclSuccess; ++k) {
        ncclUniqueId u;
        memcpy(&u, static_cast<const uint8_t *>(ids) + (size_t)k * sizeof u, sizeof u);
        r = ncclCommInitRank(&x->lanes[(size_t)k].comm, world, u, rank);
    }
    const ncclResult_t r2 = ncclGroupEnd();
    if (r == ncclSuccess) r = r2;
    if (r != ncclSuccess) { cleanup(); return fail(BSQ_E_HIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r)); }
    *out = x.release();
    return BSQ_OK;
}

extern "C" void bsq_xchg_free(bsq_xchg *x)
{
    if (!x) return;
    hipSetDevice(x->device);
    for (Lane &l : x->lanes) free_lane(l);
    delete x;
}

extern "C" int bsq_batch_run_rounds_x(bsq_batch *const *batches, int n, const bsq_opts *opts, const uint64_t *first_call,
                                      int rounds, bsq_xchg *x)
{
    if (!x) return bsq_batch_run_rounds(batches, n, opts, first_call, rounds);
    if (n < 1 || rounds < 0 || !batches || !opts || !first_call) return fail(BSQ_E_INVALID, "invalid argument");
    if (n != (int)x->lanes.size()) return fail(BSQ_E_INVALID, "one exchange lane per batch expected");
    std::vector<int> rc((size_t)n, BSQ_OK);
    std::vector<std::string> msg((size_t)n);
    std::vector<double> wait((size_t)n, 0.0);
    auto one = [&](int i) {
        roctxRangePushA("bsq_batch_rounds_x");
        for (int k = 0; k < rounds && !rc[(size_t)i]; ++k) {
            rc[(size_t)i] = bsq_batch_run(batches[i], opts, first_call[i]);
            if (rc[(size_t)i]) break;
            const auto t0 = std::chrono::steady_clock::now();
            rc[(size_t)i] = lane_round(x, i, batches[i]);
            wait[(size_t)i] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        }
        if (rc[(size_t)i]) msg[(size_t)i] = bsq_last_error();
        roctxRangePop();
    };
    std::vector<std::thread> th;
    for (int i = 1; i < n; ++i) th.emplace_back(one, i);
    one(0);
    for (auto &t : th) t.join();
    for (double w : wait) x->wait_ms += w;
    for (int i = 0; i < n; ++i)
        if (rc[(size_t)i]) return fail(rc[(size_t)i], "batch " + std::to_string(i) + ": " + msg[(size_t)i]);
    return BSQ_OK;
}

extern "C" int bsq_xchg_finish(bsq_xchg *x, int64_t *bytes_moved, double *wait_ms)
{
    if (!x) return fail(BSQ_E_INVALID, "invalid argument");
    XHIP(hipSetDevice(x->device));
    int64_t moved = 0;
    for (Lane &l : x->lanes) {
        XHIP(hipStreamSynchronize(l.xs));
        moved += l.bytes;
    }
    if (bytes_moved) *bytes_moved = moved;
    if (wait_ms) *wait_ms = x->wait_ms;
    return BSQ_OK;
}

extern "C" int bsq_xchg_view(const bsq_xchg *x, int lane, int src_rank, bsq_hits *out)
{
    if (!x || !out || lane < 0 || lane >= (int)x->lanes.size() || src_rank < 0 || src_rank >= x->world)
        return fail(BSQ_E_INVALID, "invalid argument");
    if (x->rank != 0 || src_rank == 0) return fail(BSQ_E_INVALID, "rank 0 holds the other ranks' records (its own are in its batches)");
    const Lane &l = x->lanes[(size_t)lane];
    if (!l.rounds) return fail(BSQ_E_INVALID, "no round exchanged yet");
    const Parts &p = l.parts[(size_t)src_rank];
    uint8_t *h = l.recv_host + l.at[(size_t)src_rank];
    *out = bsq_hits{};
    out->n_reads = (int32_t)p.n_reads;
    out->n_hits = p.n_hits;
    out->read_off = reinterpret_cast<int64_t *>(h);
    out->hits = reinterpret_cast<bsq_hit *>(h + p.o_hit());
    out->n_cigar = p.n_cigar;
    out->cigar = reinterpret_cast<uint32_t *>(h + p.o_cig());
    return BSQ_OK;
}
