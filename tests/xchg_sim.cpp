// xchg_sim.cpp -- the record exchange's real orchestration (bioseqdb_amd/csrc/exchange_core.h, the Core that
// exchange.cpp drives over RCCL) run on the host: ranks are threads, the transport is host memory with NCCL's
// matching rules (collectives match by issue order on a communicator; send/recv match in order per peer pair, and
// the byte counts of a matched pair must agree).  TEST INFRASTRUCTURE (tests/test_xchg_sim.py builds and runs it).
//
// What it checks, for world sizes and schedules the one-GPU box cannot run (the driver's 8-GPU curve,
// SURVEY.md 8(e); the reference's loop being sharded is bioseqdb/extension.cpp:362-370):
//   * every rank issues its collectives in the same order: the transport asserts that the k-th all-gather of
//     every rank is for the same lane, and that the k-th send of rank r matches rank 0's k-th receive from r in
//     lane and size -- with lanes finishing their rounds in a shuffled order (per-round sleeps);
//   * rank 0's receive buffer holds, for every (round, lane), every other rank's read offsets, hits and CIGAR words
//     at the offsets the Core computed (Parts), byte for byte -- ragged ranks, zero-read and zero-hit ranks,
//     the staged (host-resident view) branch;
//   * a batch failure on one rank stops every rank at the same (round, lane) with an error naming it, and nothing
//     hangs (every wait in the transport has a deadline that fails the run instead);
//   * a lane's next round waits for its previous send to be matched (batch_resume blocks, as the batch stream's
//     wait on the RCCL `sent` event does), and when rank 0's receive fails locally (mode "recv") the other ranks'
//     exchange threads, waiting for a lane that can never publish, give up through Transport::poll's deadline.
//   Aborts are local to a rank (ncclCommAbort does not wake a peer).
// Usage: xchg_sim <world> <lanes> <rounds> [fail_rank fail_lane fail_round [recv]]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../bioseqdb_amd/csrc/exchange_core.h"

using namespace bsq::xchg;

constexpr int64_t HIT = 72;   // sizeof(bsq_hit)
constexpr double DEADLINE_S = 20.0;
constexpr double POLL_DEADLINE_S = 3.0;   // the exchange thread's wait for a lane to publish (BSQ_XCHG_TIMEOUT_S)

// ---- the records a (rank, lane, round) produces: deterministic, ragged, some empty ----
struct Gen {
    int64_t n_reads, n_hits, n_cigar;
    std::vector<int64_t> off;
    std::vector<uint8_t> hits;
    std::vector<uint32_t> cig;
    bool on_device;
};
static uint64_t mix(uint64_t x)
{
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}
static Gen gen(int r, int i, int k)
{
    Gen g;
    const uint64_t h = mix((uint64_t)r * 1000003 + (uint64_t)i * 10007 + (uint64_t)k * 101 + 7);
    g.n_reads = (h % 7 == 0) ? 0 : (int64_t)(h % 97) + 1;            // some shares are empty
    const bool zero_hits = (h >> 8) % 5 == 0;                         // some ranks find nothing
    g.off.assign((size_t)g.n_reads + 1, 0);
    for (int64_t j = 0; j < g.n_reads; ++j)
        g.off[(size_t)j + 1] = g.off[(size_t)j] + (zero_hits ? 0 : (int64_t)(mix(h + (uint64_t)j) % 4));
    g.n_hits = g.off[(size_t)g.n_reads];
    g.hits.resize((size_t)(g.n_hits * HIT));
    for (size_t b = 0; b < g.hits.size(); ++b) g.hits[b] = (uint8_t)mix(h ^ (b * 0x9e3779b97f4a7c15ull));
    g.n_cigar = g.n_hits * 2 + (int64_t)((h >> 16) % 3) * (g.n_hits > 0);
    g.cig.resize((size_t)g.n_cigar);
    for (size_t c = 0; c < g.cig.size(); ++c) g.cig[c] = (uint32_t)mix(h + 77 + c);
    g.on_device = (h >> 24) % 4 != 0;                                  // 1 in 4 rounds: the staged branch
    return g;
}

// ---- the fabric: host-memory "RCCL" shared by the rank threads ----
struct Fabric {
    int world;
    std::mutex mu;
    std::condition_variable cv;
    std::vector<char> aborted;   // per rank
    std::vector<std::string> violations;
    // all-gathers by issue index: lane + headers per rank
    struct AG { int lane = -1; int arrived = 0; std::vector<int64_t> hdr; };
    std::map<int64_t, AG> ag;
    // per source rank: FIFO of sends to rank 0 (lane, bytes)
    std::vector<std::deque<std::pair<int, std::vector<uint8_t>>>> q;
    // per (source rank, lane): sends issued and sends matched by rank 0's receive
    std::map<std::pair<int, int>, int64_t> issued, matched;
    std::atomic<int64_t> staged{0}, sends{0}, recvs{0};
    explicit Fabric(int w) : world(w), aborted((size_t)w, 0), q((size_t)w) {}
    void violate(const std::string &m) { std::lock_guard<std::mutex> lk(mu); violations.push_back(m); }
    template <class P> bool wait(int rank, std::unique_lock<std::mutex> &lk, P pred, std::string &err, const char *what)
    {
        if (!cv.wait_for(lk, std::chrono::duration<double>(DEADLINE_S), [&] { return aborted[(size_t)rank] || pred(); })) {
            err = std::string("deadline: ") + what + " never matched (a deadlock on real RCCL)";
            return false;
        }
        if (aborted[(size_t)rank] && !pred()) { err = "aborted"; return false; }
        return true;
    }
};

class FakeTransport final : public Transport {
  public:
    FakeTransport(Fabric &f, int rank, int lanes, int fail_lane = -1, int fail_round = -1)
        : f_(f), rank_(rank), recv_buf_((size_t)lanes), n_recv_((size_t)lanes, 0), fail_lane_(fail_lane), fail_round_(fail_round) {}
    int world() const override { return f_.world; }
    int rank() const override { return rank_; }
    int all_gather(int lane, const int64_t mine[4], int64_t *all, std::string &err) override
    {
        std::unique_lock<std::mutex> lk(f_.mu);
        Fabric::AG &a = f_.ag[n_ag_];
        if (a.hdr.empty()) a.hdr.assign((size_t)f_.world * 4, 0);
        if (a.lane < 0) a.lane = lane;
        else if (a.lane != lane)
            f_.violations.push_back("all-gather #" + std::to_string(n_ag_) + ": rank " + std::to_string(rank_) + " lane " +
                                    std::to_string(lane) + " vs lane " + std::to_string(a.lane));
        memcpy(&a.hdr[(size_t)rank_ * 4], mine, 32);
        ++a.arrived;
        f_.cv.notify_all();
        const int64_t me = n_ag_++;
        if (!f_.wait(rank_, lk, [&] { return f_.ag[me].arrived == f_.world; }, err, "an all-gather")) return -3;
        memcpy(all, f_.ag[me].hdr.data(), (size_t)f_.world * 32);
        return 0;
    }
    int send(int lane, const Records &r, const Parts &p, std::string &) override
    {
        // what the RCCL transport puts on the wire: the three parts back to back (the receiver places them)
        std::vector<uint8_t> w((size_t)p.payload());
        const uint8_t *src_off = static_cast<const uint8_t *>(r.off);
        if (!r.on_device) {   // the staged branch: the host view is copied into a staging buffer first
            staging_.assign(src_off, src_off + p.off_bytes());
            src_off = staging_.data();
            ++f_.staged;
        }
        memcpy(w.data(), src_off, (size_t)p.off_bytes());
        if (p.n_hits) memcpy(w.data() + p.off_bytes(), r.hits, (size_t)p.hits_bytes());
        if (p.n_cigar) memcpy(w.data() + p.off_bytes() + p.hits_bytes(), r.cig, (size_t)p.cig_bytes());
        std::lock_guard<std::mutex> lk(f_.mu);
        f_.q[(size_t)rank_].emplace_back(lane, std::move(w));
        ++f_.issued[{rank_, lane}];
        ++f_.sends;
        f_.cv.notify_all();
        return 0;
    }
    int recv(int lane, const std::vector<Parts> &parts, const std::vector<int64_t> &at, int64_t total, std::string &err) override
    {
        if (lane == fail_lane_ && n_recv_[(size_t)lane] == fail_round_) { err = "injected receive failure"; return -3; }
        ++n_recv_[(size_t)lane];
        std::vector<uint8_t> &buf = recv_buf_[(size_t)lane];
        buf.assign((size_t)total, 0xEE);
        for (int k = 1; k < f_.world; ++k) {
            std::unique_lock<std::mutex> lk(f_.mu);
            if (!f_.wait(rank_, lk, [&] { return !f_.q[(size_t)k].empty(); }, err, "a receive")) return -3;
            auto item = std::move(f_.q[(size_t)k].front());
            f_.q[(size_t)k].pop_front();
            ++f_.matched[{k, item.first}];
            f_.cv.notify_all();
            lk.unlock();
            const Parts &p = parts[(size_t)k];
            if (item.first != lane || (int64_t)item.second.size() != p.payload()) {
                f_.violate("receive from rank " + std::to_string(k) + ": lane " + std::to_string(item.first) + " (" +
                           std::to_string(item.second.size()) + " B) matched lane " + std::to_string(lane) + " (" +
                           std::to_string(p.payload()) + " B)");
                err = "mismatched send/recv";
                return -3;
            }
            uint8_t *d = buf.data() + at[(size_t)k];
            memcpy(d, item.second.data(), (size_t)p.off_bytes());
            memcpy(d + p.o_hit(), item.second.data() + p.off_bytes(), (size_t)p.hits_bytes());
            memcpy(d + p.o_cig(), item.second.data() + p.off_bytes() + p.hits_bytes(), (size_t)p.cig_bytes());
            ++f_.recvs;
        }
        return 0;
    }
    // the RCCL transport makes the batch stream wait on the lane's `sent` event: the batch's next round cannot start
    // before its previous send has been matched.  No deadline here, as on the device: only an abort releases it.
    int batch_resume(int lane, std::string &err) override
    {
        std::unique_lock<std::mutex> lk(f_.mu);
        f_.cv.wait(lk, [&] { return f_.aborted[(size_t)rank_] || f_.matched[{rank_, lane}] >= f_.issued[{rank_, lane}]; });
        if (f_.matched[{rank_, lane}] < f_.issued[{rank_, lane}]) { err = "aborted while waiting for the lane's send"; return -3; }
        return 0;
    }
    int poll(double waited_s, std::string &err) override
    {
        if (waited_s > POLL_DEADLINE_S) { err = "timed out waiting for a local batch"; return -3; }
        return 0;
    }
    void abort() override
    {
        std::lock_guard<std::mutex> lk(f_.mu);
        f_.aborted[(size_t)rank_] = 1;
        f_.cv.notify_all();
    }
    const std::vector<uint8_t> &received(int lane) const { return recv_buf_[(size_t)lane]; }

  private:
    Fabric &f_;
    int rank_;
    int64_t n_ag_ = 0;
    std::vector<uint8_t> staging_;
    std::vector<std::vector<uint8_t>> recv_buf_;
    std::vector<int> n_recv_;   // receives issued per lane (= rounds)
    int fail_lane_, fail_round_;
};

// rank 0's view of lane `i` after round `k`: every other rank's parts, byte for byte
static int check_view(const FakeTransport &t, const Core &c, int W, int i, int k, std::string &why)
{
    const LaneState &ls = c.lane(i);
    const std::vector<uint8_t> &buf = t.received(i);
    for (int r = 1; r < W; ++r) {
        const Gen g = gen(r, i, k);
        const Parts &p = ls.parts[(size_t)r];
        if (p.n_reads != g.n_reads || p.n_hits != g.n_hits || p.n_cigar != g.n_cigar) {
            why = "counts of rank " + std::to_string(r) + " lane " + std::to_string(i) + " round " + std::to_string(k);
            return 1;
        }
        const uint8_t *h = buf.data() + ls.at[(size_t)r];
        if (memcmp(h, g.off.data(), (size_t)p.off_bytes()) || (p.n_hits && memcmp(h + p.o_hit(), g.hits.data(), (size_t)p.hits_bytes())) ||
            (p.n_cigar && memcmp(h + p.o_cig(), g.cig.data(), (size_t)p.cig_bytes()))) {
            why = "bytes of rank " + std::to_string(r) + " lane " + std::to_string(i) + " round " + std::to_string(k);
            return 1;
        }
    }
    return 0;
}

int main(int argc, char **argv)
{
    if (argc < 4) { fprintf(stderr, "usage: xchg_sim world lanes rounds [fail_rank fail_lane fail_round]\n"); return 2; }
    const int W = atoi(argv[1]), L = atoi(argv[2]), R = atoi(argv[3]);
    const int fr = argc > 6 ? atoi(argv[4]) : -1, fl = argc > 6 ? atoi(argv[5]) : -1, fk = argc > 6 ? atoi(argv[6]) : -1;
    const bool recv_mode = argc > 7 && !strcmp(argv[7], "recv");   // rank 0's receive of (fl, fk) fails locally
    Fabric fab(W);
    std::vector<int> rc((size_t)W, 0);
    std::vector<std::string> err((size_t)W);
    std::vector<int> bad_view((size_t)W, 0);
    std::vector<std::string> why((size_t)W);
    std::mutex view_mu;
    auto rank_main = [&](int r) {
        FakeTransport t(fab, r, L, recv_mode && r == 0 ? fl : -1, recv_mode && r == 0 ? fk : -1);
        Core core(t, L, HIT);
        std::vector<Gen> cur((size_t)L);
        auto produce = [&](int i, int k, Records &rec) -> int {
            // shuffle the order in which lanes finish their rounds (and so publish to the exchange thread)
            std::this_thread::sleep_for(std::chrono::microseconds(mix((uint64_t)(r * 131 + i * 17 + k)) % 1500));
            if (r == 0 && k > 0) {   // round k-1 of this lane has been received: check it now
                std::string w;
                if (check_view(t, core, W, i, k - 1, w)) {
                    std::lock_guard<std::mutex> lk(view_mu);
                    if (!bad_view[0]) { bad_view[0] = 1; why[0] = w; }
                }
            }
            if (!recv_mode && r == fr && i == fl && k == fk) return -3;
            cur[(size_t)i] = gen(r, i, k);
            const Gen &g = cur[(size_t)i];
            rec.n_reads = g.n_reads; rec.n_hits = g.n_hits; rec.n_cigar = g.n_cigar;
            rec.off = g.off.data(); rec.hits = g.hits.data(); rec.cig = g.cig.data(); rec.on_device = g.on_device;
            return 0;
        };
        rc[(size_t)r] = core.run(R, produce, err[(size_t)r]);
        if (r == 0 && !rc[0] && !bad_view[0])
            for (int i = 0; i < L && !bad_view[0]; ++i) bad_view[0] = check_view(t, core, W, i, R - 1, why[0]);
        int64_t bytes = 0;
        for (int i = 0; i < L; ++i) bytes += core.lane(i).bytes;
        printf("rank %d rc %d bytes %lld err \"%s\"\n", r, rc[(size_t)r], (long long)bytes, err[(size_t)r].c_str());
    };
    std::vector<std::thread> th;
    for (int r = 0; r < W; ++r) th.emplace_back(rank_main, r);
    for (auto &x : th) x.join();
    for (const std::string &v : fab.violations) printf("VIOLATION %s\n", v.c_str());
    printf("sends %lld recvs %lld staged %lld\n", (long long)fab.sends.load(), (long long)fab.recvs.load(),
           (long long)fab.staged.load());
    if (!fab.violations.empty()) return 1;
    if (bad_view[0]) { printf("BAD VIEW %s\n", why[0].c_str()); return 1; }
    if (fr < 0) {
        for (int r = 0; r < W; ++r) if (rc[(size_t)r]) return 1;
        if (fab.sends.load() != (int64_t)(W - 1) * L * R || fab.recvs.load() != fab.sends.load()) return 1;
        printf("OK\n");
        return 0;
    }
    if (recv_mode) {   // rank 0 names its receive; every other rank stops too (all-gather deadline or poll deadline)
        if (!rc[0] || err[0].find("injected receive failure") == std::string::npos) { printf("rank 0 did not report its receive\n"); return 1; }
        for (int r = 1; r < W; ++r)
            if (!rc[(size_t)r]) { printf("rank %d did not stop\n", r); return 1; }
        printf("OK (receive failure, no hang)\n");
        return 0;
    }
    // failure injected at (fr, fl, fk): every rank fails, naming it; nothing of a later (round, lane) was sent
    const std::string tag = "rank " + std::to_string(fr) + " lane " + std::to_string(fl) + " round " + std::to_string(fk);
    for (int r = 0; r < W; ++r)
        if (!rc[(size_t)r] || err[(size_t)r].find(tag) == std::string::npos) { printf("rank %d did not stop on %s\n", r, tag.c_str()); return 1; }
    if (fab.sends.load() > (int64_t)(W - 1) * ((int64_t)fk * L + fl)) { printf("sent past the failure\n"); return 1; }
    printf("OK (failure propagated)\n");
    return 0;
}
