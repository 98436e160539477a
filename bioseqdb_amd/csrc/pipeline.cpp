// pipeline.cpp -- cursor fetches aligned as a pipeline of batches (include/bsq.h bsq_pipeline_*).
//
// The reference aligns a query cursor one row at a time, each row through the whole of libbwa before the next
// fetch (bioseqdb/extension.cpp:156-195, 362-370).  On the GPU a fetch is one batch, and a lone batch leaves the
// device idle while the backend fetches the next rows, stages them and builds the previous fetch's tuples, and
// leaves the CUs under-filled in the stage tails of its own kernels.  A pipeline owns n_slots batches, each
// with its own HIP stream and host worker thread: submit() stages a fetch (its tuples may be released as soon
// as it returns) and hands it to the next slot's worker, which uploads, aligns, copies the records to pinned
// host memory and, if asked, renders the two nuclseq columns of every row on the GPU.  Results come back in
// submission order (next/release), so up to n_slots fetches are on the device at once while the caller
// produces the next fetch and consumes the last one.  The one-shot bsq_align_batch splits a large call over
// its index's pipeline the same way, and every member of a device group owns one (group.cpp).
//
// Built on the C-ABI of bsq_api.cpp plus its staging halves (bsq_internal.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cstdio>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/bsq.h"
#include "bsq_internal.h"

using namespace bsq;

namespace {

enum class SlotState { FREE, QUEUED, DONE, HELD };   // HELD: taken by the caller (or a failed take, below)

struct Slot {
    SlotState state = SlotState::FREE;
    // job
    bsq_opts opts{};
    uint64_t first_call = 0;
    int32_t n = 0;
    bool cols = false;
    PipeMode mode = PipeMode::COPY;
    const void *const *reads = nullptr;   // PipeMode::DEFER: staged by the worker
    bool stage_pending = false;           // DEFER: the caller's reads are still referenced (bsq_pipeline_wait_staged)
    // batch and staging
    bsq_batch *batch = nullptr;
    int32_t cap_reads = 0;
    int64_t cap_bases = 0;
    NsStage stage;
    bool resident = false;                // the batch holds this staging's reads (a RERUN skips the upload)
    // result
    int rc = BSQ_OK;
    std::string err;
    bool failed_take = false;             // taken with an error: freed once every older taken slot is released
    const bsq_hits *view = nullptr;
    bsq_hits empty{};
    std::vector<int64_t> zeros;
    const uint8_t *col_buf = nullptr;     // the batch's pinned column buffers (borrowed)
    const int64_t *col_off = nullptr;
    std::thread th;
    uint64_t job = 0;                     // submission number (alignment turns go in this order)
    double t[6] = {0, 0, 0, 0, 0, 0};     // BSQ_PIPE_TRACE: submit, start, uploaded, run, columns, taken (ms)
};

double now_ms()
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

bool pipe_trace()
{
    static const bool on = [] { const char *e = getenv("BSQ_PIPE_TRACE"); return e && *e && *e != '0'; }();
    return on;
}

}  // namespace

struct bsq_pipeline {
    bsq_index *idx = nullptr;
    std::vector<std::unique_ptr<Slot>> s;
    uint64_t n_submit = 0, n_take = 0, n_release = 0;   // slot of job j is s[j % S]
    uint64_t run_started = 0;                           // jobs whose alignment turn has begun
    uint64_t stage_turn = 0;                            // the job whose staging may run (submission order)
    int running = 0, run_cap = 6;                       // alignments on the device now, and at most
    int route_via = -1;                                 // record route of the slots' batches (group exchange)
    std::vector<std::array<double, 7>> trace;           // BSQ_PIPE_TRACE: per job, slot then Slot::t
    std::vector<WsSet *> pool;                          // device workspaces between alignment turns (<= run_cap)
    std::mutex mu;
    std::condition_variable cv;
    bool stop = false;
};

namespace {

void drop_cols(Slot &x)
{
    x.col_buf = nullptr;
    x.col_off = nullptr;
}

// Fetch staging (a deferred job) and the upload of its reads: before the slot's turn on the device.
int prep_job(bsq_pipeline *p, Slot &x)
{
    x.t[1] = now_ms();
    // Staging turns go in submission order: a deferred fetch is staged on all of stage_nuclseqs' threads while the
    // fetches behind it wait, so the first fetches reach the device first (16 stagings at once put ~128 threads on
    // the caller's cores and delayed every one of them).  Every job takes its turn, staged or not.
    {
        std::unique_lock<std::mutex> lk(p->mu);
        p->cv.wait(lk, [&] { return x.job == p->stage_turn; });
    }
    struct Turn {   // passes the staging turn on exactly once (early returns included)
        bsq_pipeline *p;
        void pass()
        {
            if (!p) return;
            std::lock_guard<std::mutex> lk(p->mu);
            ++p->stage_turn;
            p->cv.notify_all();
            p = nullptr;
        }
        ~Turn() { pass(); }
    } turn{p};
    if (const char *e = getenv("BSQ_PIPE_FAILPOINT")) {   // tests: job number e fails here (a failed fetch)
        if (*e && strtoull(e, nullptr, 10) == x.job) {
            std::lock_guard<std::mutex> lk(p->mu);
            x.stage_pending = false;
            x.reads = nullptr;
            p->cv.notify_all();
            set_error("injected failure (BSQ_PIPE_FAILPOINT)");
            return BSQ_E_INVALID;
        }
    }
    if (x.mode == PipeMode::DEFER) {
        x.resident = false;
        const int rc = stage_nuclseqs(x.stage, x.reads, x.n);
        {   // the caller's varlenas are no longer read (on success or failure)
            std::lock_guard<std::mutex> lk(p->mu);
            x.stage_pending = false;
            x.reads = nullptr;
            p->cv.notify_all();
        }
        if (rc) return rc;
    } else if (x.mode == PipeMode::COPY) {
        x.resident = false;
    }
    turn.pass();   // the upload below runs beside the next job's staging
    if (x.n == 0 || bsq_index_seq_len(p->idx) <= 0) return BSQ_OK;
    if (!x.batch || x.cap_reads < x.stage.n || x.cap_bases < x.stage.bases) {
        bsq_batch_free(x.batch);
        x.batch = nullptr;
        x.resident = false;
        // grow geometrically so fetches of similar size reuse one workspace
        const int32_t r = std::max<int32_t>(x.stage.n, (int32_t)std::min<int64_t>(2LL * x.cap_reads, 1 << 20));
        const int64_t b = std::max<int64_t>(x.stage.bases, std::min<int64_t>(2 * x.cap_bases, (int64_t)r * 1024));
        const int rc = bsq_batch_create(p->idx, std::max(r, 1), std::max<int64_t>(b, 1), &x.batch);
        if (rc) { x.batch = nullptr; x.cap_reads = 0; x.cap_bases = 0; return rc; }
        x.cap_reads = std::max(r, 1);
        x.cap_bases = std::max<int64_t>(b, 1);
    }
    { const int rc = bsq_batch_set_record_route(x.batch, p->route_via); if (rc) return rc; }   // no-op when unchanged
    if (!x.resident) {
        const int rc = batch_upload_staged(x.batch, x.stage, false);   // workspaces come with the alignment turn
        if (rc) return rc;
        x.resident = true;
    }
    return BSQ_OK;
}

// The alignment itself, in the slot's turn (at most run_cap jobs align at once, started in submission order).
int align_job(bsq_pipeline *p, Slot &x)
{
    x.t[2] = now_ms();
    if (x.n == 0 || bsq_index_seq_len(p->idx) <= 0) {   // bwa.cpp:142-143: no region for any read
        x.zeros.assign((size_t)x.n + 1, 0);
        x.empty = bsq_hits{};
        x.empty.n_reads = x.n;
        x.empty.read_off = x.zeros.data();
        x.view = &x.empty;
        return BSQ_OK;
    }
    // The device workspaces (~8.5 GB per 262,144-read pass) are lent for the turn: at most run_cap alignments run
    // at once, so the pipeline holds run_cap sets however many fetches wait staged and uploaded (16 sets of 16
    // slots did not fit beside a 3 Gbp index).  Sets of the same shape are reused as they are.
    // (A batch that ran outside the pipeline since -- a group's held shares -- may hold its own set: it keeps it.)
    WsSet *ws = nullptr;
    if (!batch_has_workspace(x.batch)) {
        std::lock_guard<std::mutex> lk(p->mu);
        if (!p->pool.empty()) { ws = p->pool.back(); p->pool.pop_back(); }
    }
    batch_attach_workspaces(x.batch, ws);
    int rc = batch_prepare_workspace(x.batch);
    if (!rc) rc = bsq_batch_run(x.batch, &x.opts, x.first_call);
    const std::string err = rc ? std::string(bsq_last_error()) : std::string();
    ws = batch_detach_workspaces(x.batch);
    if (ws) {
        // at most run_cap sets are kept: a batch that brought its own set (a group re-run) would otherwise grow the
        // pool past the alignments that can use it at once (~8.5 GB each)
        std::unique_lock<std::mutex> lk(p->mu);
        if ((int)p->pool.size() < p->run_cap) { p->pool.push_back(ws); ws = nullptr; }
        lk.unlock();
        workspaces_free(ws);
    }
    if (rc) { set_error(err); return rc; }
    x.t[3] = now_ms();
    x.view = bsq_batch_hits(x.batch);
    return BSQ_OK;
}

// build_tuple_bwa's two nuclseq columns, after the slot's turn (the next job aligns meanwhile)
int cols_job(Slot &x)
{
    if (x.cols && x.view != &x.empty && x.view->n_hits > 0) {
        // the staged varlenas carry the reads' hole symbols (the caller's may be gone)
        std::vector<const void *> ptrs((size_t)x.n);
        for (int32_t i = 0; i < x.n; ++i) ptrs[(size_t)i] = x.stage.host + x.stage.meta[(size_t)i];
        const int rc = batch_render_cols(x.batch, ptrs.data(), &x.col_buf, &x.col_off);
        if (rc) return rc;
    }
    x.t[4] = now_ms();
    return BSQ_OK;
}

void worker(bsq_pipeline *p, Slot *x)
{
    std::unique_lock<std::mutex> lk(p->mu);
    for (;;) {
        p->cv.wait(lk, [&] { return p->stop || x->state == SlotState::QUEUED; });
        if (p->stop) return;
        lk.unlock();
        int rc = prep_job(p, *x);
        // Alignment turns go in submission order, at most run_cap at once: a deeper pipeline keeps fetches staged
        // and uploaded ahead, so a new alignment starts the moment one ends instead of the pipeline refilling
        // in lockstep groups when the caller takes the oldest fetch (every job takes its turn, failed or not).
        lk.lock();
        p->cv.wait(lk, [&] { return x->job == p->run_started && p->running < p->run_cap; });
        ++p->run_started;
        ++p->running;
        p->cv.notify_all();
        lk.unlock();
        if (!rc) rc = align_job(p, *x);
        lk.lock();
        --p->running;
        p->cv.notify_all();
        lk.unlock();
        if (!rc) rc = cols_job(*x);
        const std::string err = rc ? std::string(bsq_last_error()) : std::string();
        lk.lock();
        x->rc = rc;
        x->err = err;
        x->state = SlotState::DONE;
        p->cv.notify_all();
    }
}

int fail(int rc, const std::string &m)
{
    set_error(m);
    return rc;
}

// Free the oldest taken slots that were taken with an error (the caller never releases those).  Called with the
// pipeline lock held.  A failed take behind a taken submission the caller still holds stays HELD until that one is
// released, so a new submission can never land on a slot whose view the caller is still reading.
void reap_failed(bsq_pipeline *p)
{
    while (p->n_release < p->n_take) {
        Slot *y = p->s[p->n_release % p->s.size()].get();
        if (!y->failed_take) break;
        y->failed_take = false;
        y->view = nullptr;
        y->state = SlotState::FREE;
        ++p->n_release;
    }
    p->cv.notify_all();
}

}  // namespace

namespace bsq {

int pipeline_submit_ex(bsq_pipeline *p, const bsq_opts *opts, const void *const *reads, int32_t n_reads,
                       uint64_t first_call_seq, int nuclseq_columns, PipeMode mode)
{
    if (!p || !opts || n_reads < 0 || (n_reads && !reads && mode != PipeMode::RERUN)) return fail(BSQ_E_INVALID, "invalid argument");
    if (opts->e_del <= 0 || opts->e_ins <= 0 || opts->max_occ <= 0 || opts->min_seed_len < 0)
        return fail(BSQ_E_INVALID, "gap extension penalties and max_occ must be positive, min_seed_len nonnegative");
    Slot *x;
    {
        std::lock_guard<std::mutex> lk(p->mu);
        x = p->s[p->n_submit % p->s.size()].get();
        if (x->state != SlotState::FREE)
            return fail(BSQ_E_INVALID, "every slot of the pipeline holds a submission (take and release the oldest first)");
    }
    if (mode == PipeMode::RERUN && x->stage.n != n_reads)
        return fail(BSQ_E_INVALID, "re-run of a different read count than the slot's staged reads");
    const double t_submit = now_ms();
    if (mode == PipeMode::COPY) {   // staged on the caller's thread: the caller may release its reads on return
        x->resident = false;
        const int rc = stage_nuclseqs(x->stage, reads, n_reads);
        if (rc) return rc;
    }
    std::lock_guard<std::mutex> lk(p->mu);
    x->opts = *opts;
    x->first_call = first_call_seq;
    x->n = n_reads;
    x->cols = nuclseq_columns != 0;
    x->mode = mode;
    x->reads = mode == PipeMode::DEFER ? reads : nullptr;
    x->stage_pending = mode == PipeMode::DEFER;
    x->view = nullptr;
    drop_cols(*x);
    for (double &t : x->t) t = 0;
    x->t[0] = t_submit;
    x->job = p->n_submit;
    x->state = SlotState::QUEUED;
    ++p->n_submit;
    p->cv.notify_all();
    return BSQ_OK;
}

int pipeline_wait_staged(bsq_pipeline *p, int64_t upto)
{
    if (!p) return fail(BSQ_E_INVALID, "invalid argument");
    std::unique_lock<std::mutex> lk(p->mu);
    p->cv.wait(lk, [&] {
        for (auto &x : p->s)
            if (x->stage_pending && (int64_t)x->job < upto) return false;
        return true;
    });
    return BSQ_OK;
}

int pipeline_set_record_route(bsq_pipeline *p, int via_device)
{
    std::lock_guard<std::mutex> lk(p->mu);
    if (p->n_release != p->n_submit) return fail(BSQ_E_INVALID, "pipeline has outstanding submissions");
    p->route_via = via_device;   // applied by each slot's worker before its next alignment
    return BSQ_OK;
}

int pipeline_rewind(bsq_pipeline *p)
{
    std::lock_guard<std::mutex> lk(p->mu);
    if (p->n_release != p->n_submit) return fail(BSQ_E_INVALID, "pipeline has outstanding submissions");
    p->n_submit = p->n_take = p->n_release = 0;
    p->run_started = 0;
    p->stage_turn = 0;
    return BSQ_OK;
}

int pipeline_next_ex(bsq_pipeline *p, const bsq_hits **view, const uint8_t **cols, const int64_t **col_off,
                     bsq_batch **batch)
{
    if (!p || !view) return fail(BSQ_E_INVALID, "invalid argument");
    std::unique_lock<std::mutex> lk(p->mu);
    if (p->n_take == p->n_submit) return fail(BSQ_E_INVALID, "no submission to take");
    Slot *x = p->s[p->n_take % p->s.size()].get();
    p->cv.wait(lk, [&] { return x->state == SlotState::DONE; });
    if (pipe_trace()) {
        x->t[5] = now_ms();
        std::array<double, 7> r{};
        r[0] = (double)(p->n_take % p->s.size());
        for (int k = 0; k < 6; ++k) r[(size_t)k + 1] = x->t[k];
        p->trace.push_back(r);
    }
    ++p->n_take;
    if (x->rc) {   // consumed: the slot is free again once every older taken submission is released
        const int rc = x->rc;
        const std::string m = x->err;
        x->state = SlotState::HELD;
        x->failed_take = true;
        drop_cols(*x);
        reap_failed(p);
        return fail(rc, m);
    }
    x->state = SlotState::HELD;
    *view = x->view;
    if (cols) *cols = x->col_buf;
    if (col_off) *col_off = x->col_off;
    if (batch) *batch = x->view == &x->empty ? nullptr : x->batch;
    return BSQ_OK;
}

}  // namespace bsq

extern "C" int bsq_pipeline_create(bsq_index *idx, int n_slots, bsq_pipeline **out)
{
    if (!idx || !out || n_slots < 1 || n_slots > 64) return fail(BSQ_E_INVALID, "invalid argument");
    *out = nullptr;
    std::unique_ptr<bsq_pipeline> p(new (std::nothrow) bsq_pipeline());
    if (!p) return fail(BSQ_E_NOMEM, "out of memory");
    p->idx = idx;
    {   // concurrent alignments: 6 measure best on one MI355X with 16 fetches in flight and 8 HIP hardware queues
        // (4 at depth 8 41 M reads/s, 6-7 at depth 16 44-46 M; 16 or 24 queues 25-38 M)
        const char *e = getenv("BSQ_PIPE_RUN");
        const int v = e ? atoi(e) : 6;
        p->run_cap = std::max(1, std::min(v > 0 ? v : 6, 64));
    }
    for (int k = 0; k < n_slots; ++k) p->s.emplace_back(new Slot());
    for (auto &x : p->s) x->th = std::thread(worker, p.get(), x.get());
    *out = p.release();
    return BSQ_OK;
}

extern "C" void bsq_pipeline_free(bsq_pipeline *p)
{
    if (!p) return;
    {
        std::unique_lock<std::mutex> lk(p->mu);
        // submissions still on the device finish first (their workers own the batches)
        p->cv.wait(lk, [&] {
            for (auto &x : p->s)
                if (x->state == SlotState::QUEUED) return false;
            return true;
        });
        p->stop = true;
        p->cv.notify_all();
    }
    if (pipe_trace() && !p->trace.empty()) {   // one line per job, ms relative to the first submission
        const double t0 = p->trace[0][1];
        for (const auto &r : p->trace)
            fprintf(stderr, "bsq_pipe slot %d submit %.2f start %.2f turn %.2f run %.2f cols %.2f taken %.2f\n",
                    (int)r[0], r[1] - t0, r[2] - t0, r[3] - t0, r[4] - t0, r[5] - t0, r[6] - t0);
    }
    for (auto &x : p->s) {
        if (x->th.joinable()) x->th.join();
        drop_cols(*x);
        bsq_batch_free(x->batch);
    }
    for (WsSet *w : p->pool) workspaces_free(w);
    delete p;
}

extern "C" int bsq_pipeline_slots(const bsq_pipeline *p) { return p ? (int)p->s.size() : 0; }

extern "C" int bsq_pipeline_submit(bsq_pipeline *p, const bsq_opts *opts, const void *const *reads, int32_t n_reads,
                                   uint64_t first_call_seq, int nuclseq_columns)
{
    return pipeline_submit_ex(p, opts, reads, n_reads, first_call_seq, nuclseq_columns, PipeMode::COPY);
}

extern "C" int bsq_pipeline_submit_deferred(bsq_pipeline *p, const bsq_opts *opts, const void *const *reads, int32_t n_reads,
                                            uint64_t first_call_seq, int nuclseq_columns, int64_t *job)
{
    uint64_t j = 0;
    if (p) {
        std::lock_guard<std::mutex> lk(p->mu);
        j = p->n_submit;
    }
    const int rc = pipeline_submit_ex(p, opts, reads, n_reads, first_call_seq, nuclseq_columns, PipeMode::DEFER);
    if (!rc && job) *job = (int64_t)j;
    return rc;
}

extern "C" int bsq_pipeline_wait_staged(bsq_pipeline *p, int64_t upto) { return pipeline_wait_staged(p, upto); }

extern "C" int bsq_pipeline_next(bsq_pipeline *p, const bsq_hits **view, const uint8_t **cols, const int64_t **col_off)
{
    return pipeline_next_ex(p, view, cols, col_off, nullptr);
}

extern "C" int bsq_pipeline_release(bsq_pipeline *p)
{
    if (!p) return fail(BSQ_E_INVALID, "invalid argument");
    std::lock_guard<std::mutex> lk(p->mu);
    if (p->n_release == p->n_take) return fail(BSQ_E_INVALID, "no taken submission to release");
    Slot *x = p->s[p->n_release % p->s.size()].get();
    drop_cols(*x);
    x->view = nullptr;
    x->state = SlotState::FREE;
    ++p->n_release;
    reap_failed(p);
    return BSQ_OK;
}
