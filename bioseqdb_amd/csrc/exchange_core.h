// exchange_core.h -- the orchestration of the record exchange (bsq_xchg, exchange.cpp), transport-agnostic.
//
// SURVEY.md 8(e) / north_star: a cursor batch is sharded read-parallel over the ranks (one process per GPU) and
// every rank's hit records return to the caller -- the backend that runs nuclseq_multi_search_bwa, whose
// tuplestore takes every row (bioseqdb/extension.cpp:362-370) -- here rank 0.
//
// A rank aligns its shard as L concurrent batches ("lanes"), each a stream of rounds on its own host thread.
// After round k of lane i, every rank (1) all-gathers the header {n_reads, n_hits, n_cigar, status} of that
// (round, lane), then (2) each rank r > 0 sends its read offsets, hit records and CIGAR words to rank 0, which
// receives them into one buffer, rank after rank (Parts layout below).
//
// Deadlock freedom.  Every collective of every (round, lane) is issued by ONE exchange thread per rank, in the
// same global order on every rank: round-major, lane-minor -- (0,0), (0,1), ..., (0,L-1), (1,0), ...  A rank's
// lanes finish their rounds in whatever order their batches happen to take, and the exchange thread simply waits
// (on the host) for the next (round, lane) in the fixed order; operations therefore match one-to-one across ranks
// on one communicator and one stream, and no rank can wait on an operation another rank issues later.  A lane's
// batch thread publishes round k's records and blocks until the exchange thread has issued that round's send
// (its buffers may be overwritten only after it); lanes can drift up to one round apart, which is what lets one
// batch's seeding overlap another's DP stages.
//
// Failure.  The header's fourth word is the lane's batch status.  A batch that fails publishes its status
// instead of records; the all-gather carries it to every rank, and every rank stops the exchange at that same
// (round, lane): all batch threads return, nothing more is sent, and the transport is aborted.  A transport
// error (or a transport-level timeout) aborts the same way on the rank that sees it.
//
// No HIP here: exchange.cpp plugs in RCCL, tests/xchg_sim.cpp a host-memory transport with threads as ranks.
#pragma once
#include <stdint.h>

#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace bsq {
namespace xchg {

constexpr int64_t kAlign = 256;
inline int64_t al(int64_t x) { return (x + kAlign - 1) & ~(kAlign - 1); }

// One rank's records of one round: read offsets (n_reads x off_per_read + off_fixed bytes: the RCCL transport's wire
// form is a 16-B header and one int32 count per read, the host simulation sends n_reads + 1 int64 offsets), hits
// (n_hits x hit_bytes), CIGAR words (n_cigar u32); each part 256-B aligned inside the rank's slice of rank 0's
// receive buffer.
struct Parts {
    int64_t n_reads = 0, n_hits = 0, n_cigar = 0, hit_bytes = 0, off_per_read = 8, off_fixed = 8;
    int64_t off_bytes() const { return n_reads * off_per_read + off_fixed; }
    int64_t hits_bytes() const { return n_hits * hit_bytes; }
    int64_t cig_bytes() const { return n_cigar * 4; }
    int64_t o_hit() const { return al(off_bytes()); }
    int64_t o_cig() const { return o_hit() + al(hits_bytes()); }
    int64_t total() const { return o_cig() + al(cig_bytes()); }
    int64_t payload() const { return off_bytes() + hits_bytes() + cig_bytes(); }
};

// One lane's records of one round as its batch left them.
struct Records {
    int64_t n_reads = 0, n_hits = 0, n_cigar = 0;
    const void *off = nullptr, *hits = nullptr, *cig = nullptr;
    bool on_device = false;   // false: the view lives in (pinned) host memory and is staged by the transport
};

class Transport {
  public:
    virtual ~Transport() = default;
    virtual int world() const = 0;
    virtual int rank() const = 0;
    // 4 x int64 per rank; on return `all` (world x 4) is on this host.  Blocking.
    virtual int all_gather(int lane, const int64_t mine[4], int64_t *all, std::string &err) = 0;
    // rank > 0: `r`'s parts `p` to rank 0.  May return before the bytes have left; the lane's batch must not
    // overwrite them before batch_resume(lane).
    virtual int send(int lane, const Records &r, const Parts &p, std::string &err) = 0;
    // rank 0: every other rank's parts into the lane's receive buffer (`total` bytes; rank k's at at[k]).
    virtual int recv(int lane, const std::vector<Parts> &parts, const std::vector<int64_t> &at, int64_t total,
                     std::string &err) = 0;
    // batch thread, before its lane's next round: order the batch's next writes after the lane's last send
    // (RCCL: a device-side wait -- the batch's next blocking HIP call can then wait on that send indefinitely)
    virtual int batch_resume(int lane, std::string &err) = 0;
    // exchange thread, while it has waited `waited_s` for a lane to publish its next round: nonzero (with `err`)
    // ends the wait as a failure -- a transport error, or a deadline.  A lane blocked behind a send that no peer
    // will ever match (rank 0 died, or its receive failed locally) publishes nothing, so without this the exchange
    // thread would wait forever; the failure aborts the transport, which releases the blocked device waits.
    virtual int poll(double waited_s, std::string &err) { (void)waited_s; (void)err; return 0; }
    // every rank stops (a failure reported by some rank, or this rank's transport error)
    virtual void abort() {}
};

struct LaneState {
    std::vector<Parts> parts;   // per rank, last exchanged round
    std::vector<int64_t> at;    // per rank: offset of its parts in rank 0's receive buffer
    int64_t total = 0;          // bytes of that buffer
    int64_t bytes = 0;          // payload received (rank 0) or sent (others) over all rounds
    int64_t rounds = 0;
};

// produce(lane, round, &records) runs the lane's batch for one round and returns its status (0 = ok).
using Produce = std::function<int(int, int, Records &)>;

class Core {
  public:
    Core(Transport &t, int lanes, int64_t hit_bytes, int64_t off_per_read = 8, int64_t off_fixed = 8)
        : t_(t), hit_bytes_(hit_bytes), off_per_read_(off_per_read), off_fixed_(off_fixed), lanes_((size_t)lanes)
    {
        for (LaneState &l : lanes_) { l.parts.resize((size_t)t.world()); l.at.resize((size_t)t.world()); }
    }
    int n_lanes() const { return (int)lanes_.size(); }
    const LaneState &lane(int i) const { return lanes_[(size_t)i]; }
    double wait_ms() const { return wait_ms_; }
    bool aborted() const { return aborted_; }

    // Runs `rounds` rounds of every lane (lane i's batch thread calls produce(i, k, .)), exchanging after each.
    // The calling thread is the exchange thread.  Returns 0 or the first failure (err names rank, lane, round).
    int run(int rounds, const Produce &produce, std::string &err)
    {
        const int L = n_lanes(), W = t_.world(), R = t_.rank();
        std::mutex mu;
        std::condition_variable cv;
        struct Pub { int round = -1, status = 0; Records rec; int released = -1; };
        std::vector<Pub> pub((size_t)L);
        bool stop = false;
        std::string first;
        std::vector<double> wait((size_t)L, 0.0);
        std::vector<std::string> lane_err((size_t)L);
        auto batch = [&](int i) {
            bool resume_failed = false;   // the next round publishes a failure instead of running
            for (int k = 0; k < rounds; ++k) {
                Records rec;
                const int st = resume_failed ? -3 : produce(i, k, rec);
                const auto t0 = std::chrono::steady_clock::now();
                std::unique_lock<std::mutex> lk(mu);
                if (stop) return;
                Pub &p = pub[(size_t)i];
                p.round = k; p.status = st; p.rec = rec;
                cv.notify_all();
                if (st) return;   // the exchange thread carries the failure to every rank
                cv.wait(lk, [&] { return stop || p.released >= k; });
                wait[(size_t)i] += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                if (stop) return;
                lk.unlock();
                std::string e;
                if (t_.batch_resume(i, e)) {   // a local transport error: carried to every rank by the next header
                    lk.lock();
                    if (lane_err[(size_t)i].empty()) lane_err[(size_t)i] = e;
                    lk.unlock();
                    resume_failed = true;
                }
            }
        };
        std::vector<std::thread> th;
        th.reserve((size_t)L);
        for (int i = 0; i < L; ++i) th.emplace_back(batch, i);
        int rc = 0;
        std::vector<int64_t> all((size_t)W * 4);
        for (int k = 0; k < rounds && !rc; ++k) {
            for (int i = 0; i < L && !rc; ++i) {
                Records rec;
                int st = 0;
                std::string e;
                {
                    std::unique_lock<std::mutex> lk(mu);
                    Pub &p = pub[(size_t)i];
                    const auto t0 = std::chrono::steady_clock::now();
                    while (!cv.wait_for(lk, std::chrono::milliseconds(5), [&] { return p.round >= k; })) {
                        lk.unlock();
                        const double waited = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                        const int prc = t_.poll(waited, e);
                        lk.lock();
                        if (prc) { if (e.empty()) e = "transport poll failed"; break; }
                    }
                    if (!e.empty()) {
                        rc = fail(-3, "exchange (round " + std::to_string(k) + ", lane " + std::to_string(i) +
                                  ") waiting for the lane's batch: " + e, first);
                        break;
                    }
                    rec = p.rec;
                    st = p.status;
                }
                const int64_t mine[4] = {st ? 0 : rec.n_reads, st ? 0 : rec.n_hits, st ? 0 : rec.n_cigar, (int64_t)st};
                if (t_.all_gather(i, mine, all.data(), e)) {
                    rc = fail(-3, "exchange all-gather (round " + std::to_string(k) + ", lane " + std::to_string(i) + "): " + e, first);
                    break;
                }
                for (int r = 0; r < W; ++r)
                    if (all[(size_t)r * 4 + 3]) {
                        rc = fail((int)all[(size_t)r * 4 + 3], "rank " + std::to_string(r) + " lane " + std::to_string(i) +
                                  " round " + std::to_string(k) + " failed (status " + std::to_string(all[(size_t)r * 4 + 3]) + ")", first);
                        break;
                    }
                if (rc) break;
                LaneState &l = lanes_[(size_t)i];
                int64_t total = 0;
                for (int r = 0; r < W; ++r) {
                    Parts &p = l.parts[(size_t)r];
                    p.n_reads = all[(size_t)r * 4]; p.n_hits = all[(size_t)r * 4 + 1]; p.n_cigar = all[(size_t)r * 4 + 2];
                    p.hit_bytes = hit_bytes_; p.off_per_read = off_per_read_; p.off_fixed = off_fixed_;
                    l.at[(size_t)r] = total;
                    if (r != 0) total += p.total();
                }
                l.total = total;
                ++l.rounds;
                if (W > 1) {
                    if (R != 0) {
                        if (t_.send(i, rec, l.parts[(size_t)R], e)) { rc = fail(-3, "exchange send: " + e, first); break; }
                        l.bytes += l.parts[(size_t)R].payload();
                    } else {
                        if (t_.recv(i, l.parts, l.at, total, e)) { rc = fail(-3, "exchange receive: " + e, first); break; }
                        for (int r = 1; r < W; ++r) l.bytes += l.parts[(size_t)r].payload();
                    }
                }
                std::lock_guard<std::mutex> lk(mu);
                pub[(size_t)i].released = k;
                cv.notify_all();
            }
        }
        {
            std::lock_guard<std::mutex> lk(mu);
            if (rc) stop = true;
            cv.notify_all();
        }
        if (rc) { aborted_ = true; t_.abort(); }
        for (auto &x : th) x.join();
        for (double w : wait) wait_ms_ += w;
        if (!rc)
            for (int i = 0; i < L; ++i)
                if (!lane_err[(size_t)i].empty()) { rc = fail(-3, "lane " + std::to_string(i) + ": " + lane_err[(size_t)i], first); break; }
        if (rc) err = first;
        return rc;
    }

  private:
    static int fail(int rc, const std::string &m, std::string &first)
    {
        if (first.empty()) first = m;
        return rc < 0 ? rc : -3;
    }
    Transport &t_;
    int64_t hit_bytes_, off_per_read_, off_fixed_;
    std::vector<LaneState> lanes_;
    double wait_ms_ = 0;
    bool aborted_ = false;
};

}  // namespace xchg
}  // namespace bsq
