// bwa_bsq.cpp -- BwaIndex over libbsq (replaces bioseqdb/bwa.cpp; see bwa_bsq.h).
#include "bwa_bsq.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace {

void check(int rc)
{
    if (rc != BSQ_OK) throw BsqFailure(rc, bsq_last_error());
}

// nuclseq varlena fields (sequence.h:18-38): {vl_len[4], holes_num u32, len u32, holes, pac}
uint32_t ns_u32(const void *ns, size_t off)
{
    uint32_t v;
    memcpy(&v, static_cast<const uint8_t *>(ns) + off, 4);
    return v;
}
uint32_t ns_len(const void *ns) { return ns_u32(ns, 8); }
size_t ns_bytes(const void *ns) { return 12 + 16 * (size_t)ns_u32(ns, 4) + (ns_len(ns) + 3) / 4; }

struct CFree { void operator()(void *p) const { bsq_free(p); } };

const bsq_hits kNoHits{};   // n_reads = 0 view for an empty reference (filled per call below)

}  // namespace

uint64_t &bsq_backend_lrand48_calls()
{
    static uint64_t calls = 0;
    return calls;
}

void BwaRows::cigar_text(int64_t k, std::string &out) const
{
    out.clear();
    const bsq_hit &h = view_->hits[k];
    char buf[16];
    for (uint32_t c = 0; c < h.n_cigar; ++c) {
        const uint32_t v = view_->cigar[h.cigar_off + c];
        int n = 0;
        uint32_t len = v >> 4;
        do { buf[n++] = (char)('0' + len % 10); len /= 10; } while (len);
        while (n) out += buf[--n];
        out += "MIDNSHP=XB"[v & 0xf];   // htslib bam_cigar_opchr: libbwa's clip op 3 prints as 'N' (Q8)
    }
}

BwaIndex::BwaIndex(int dev) : BwaIndex(std::vector<int>{dev}) {}

BwaIndex::BwaIndex(const std::vector<int> &devices)
    : options(new BsqMemOpt()), index_(nullptr), devices_(devices.empty() ? std::vector<int>{0} : devices)
{
    const int rc = bsq_index_create(&index_);
    if (rc != BSQ_OK) {
        delete options;
        throw BsqFailure(rc, bsq_last_error());
    }
}

BwaIndex::BwaIndex(BwaIndex &&o) noexcept
    : options(o.options), index_(o.index_), devices_(o.devices_), group_(o.group_), pipe_(o.pipe_)
{
    o.reset_rows();   // a moved-from index keeps no submissions; the pipeline moves empty
    o.options = nullptr;
    o.index_ = nullptr;
    o.group_ = nullptr;
    o.pipe_ = nullptr;
}

BwaIndex::~BwaIndex()
{
    rows_ = BwaRows();
    group_rows_ = BwaRows();
    bsq_pipeline_free(pipe_);   // waits for submissions still on the device
    bsq_group_free(group_);
    bsq_index_free(index_);
    delete options;
}

void BwaIndex::add_ref_sequence(int64_t id, const NucleotideSequence &seq) { check(bsq_index_add_ref(index_, id, &seq)); }

bool BwaIndex::empty() const { return bsq_index_l_pac(index_) <= 0; }

int32_t BwaIndex::n_refs() const { return bsq_index_n_refs(index_); }

bool BwaIndex::same_refs(const BwaIndex &o) const { return bsq_index_same_refs(index_, o.index_) == 1; }

void BwaIndex::build()
{
    if (empty()) return;   // bwa.cpp:108-109
    if (bsq_device_count() > device()) check(bsq_index_build_device(index_, device()));
    else check(bsq_index_build(index_, 0));   // same tables; aligning then reports the missing device
}

int BwaIndex::pipeline_depth() const
{
    if (devices_.size() > 1) return 1;   // a group aligns its fetch at submit (every member pipelines its shard)
    const char *e = getenv("BSQ_PIPE_DEPTH");
    // 16 fetches in flight: up to 6 align at once (bsq_pipeline's run cap) while the next ones are staged and
    // uploaded, so a new alignment starts as soon as one ends (bench.py sql_cursor)
    const int d = e ? atoi(e) : 16;
    return std::max(1, std::min(d, 32));
}

void BwaIndex::ensure_pipe() const
{
    if (pipe_) return;
    check(bsq_index_upload(index_, device()));   // no-op for an index built on the device
    check(bsq_pipeline_create(index_, pipeline_depth(), &pipe_));
}

void BwaIndex::ensure_group() const
{
    if (group_) return;
    check(bsq_index_upload(index_, device()));   // no-op for an index built on the first device
    bsq_group *g = nullptr;
    check(bsq_group_create(devices_.data(), (int)devices_.size(), &g));
    const int rc = bsq_group_replicate(g, index_, nullptr);   // one build, broadcast over xGMI
    if (rc != BSQ_OK) {
        const std::string m = bsq_last_error();
        bsq_group_free(g);
        throw BsqFailure(rc, m);
    }
    group_ = g;
}

int64_t BwaIndex::submit_rows(const NucleotideSequence *const *seqs, int32_t n, bool nuclseq_columns,
                              const BsqMemOpt *opts, bool deferred) const
{
    int64_t ticket = -1;
    if ((int)pending_.size() + held_ >= pipeline_depth())
        throw BsqFailure(BSQ_E_INVALID, "every pipeline slot holds a fetch (take and release the oldest first)");
    Pending pd;
    pd.cols = nuclseq_columns;
    pd.n = std::max(n, 0);
    if (n <= 0 || empty()) {   // bwa.cpp:142-143: no mem_align1 call, no lrand48 value drawn
        pd.empty = true;
        pending_.push_back(pd);
        return ticket;
    }
    const void *const *ptrs = reinterpret_cast<const void *const *>(seqs);
    const bsq_opts o = (opts ? *opts : *options).c_abi();
    uint64_t &calls = bsq_backend_lrand48_calls();
    if (devices_.size() > 1) {   // the fetch spread over the group, member k taking a contiguous share
        ensure_group();
        check(bsq_group_run(group_, &o, ptrs, n, calls));
        group_rows_ = BwaRows();
        group_rows_.view_ = bsq_group_hits(group_);
        if (!group_rows_.view_) throw BsqFailure(BSQ_E_NOMEM, bsq_last_error());
        if (nuclseq_columns && group_rows_.view_->n_hits > 0) {   // rendered now: the reads go away on return
            uint8_t *cols = nullptr;
            int64_t *off = nullptr;
            check(bsq_group_render_nuclseqs(group_, ptrs, &cols, &off));
            group_rows_.own_cols_.reset(cols);
            group_rows_.own_off_.reset(off);
            group_rows_.cols_ = cols;
            group_rows_.col_off_ = off;
        }
    } else {
        ensure_pipe();
        if (deferred) check(bsq_pipeline_submit_deferred(pipe_, &o, ptrs, n, calls, nuclseq_columns ? 1 : 0, &ticket));
        else check(bsq_pipeline_submit(pipe_, &o, ptrs, n, calls, nuclseq_columns ? 1 : 0));
        ++in_pipe_;
    }
    calls += (uint64_t)n;
    pending_.push_back(pd);
    return ticket;
}

void BwaIndex::wait_staged(int64_t ticket) const
{
    if (ticket >= 0 && pipe_) check(bsq_pipeline_wait_staged(pipe_, ticket + 1));
}

const BwaRows &BwaIndex::take_rows() const
{
    if (held_) throw BsqFailure(BSQ_E_INVALID, "release the taken rows first");
    if (pending_.empty()) throw BsqFailure(BSQ_E_INVALID, "no submitted fetch to take");
    const Pending pd = pending_.front();
    pending_.pop_front();
    rows_ = BwaRows();
    if (pd.empty) {
        zeros_.assign((size_t)pd.n + 1, 0);
        none_ = kNoHits;
        none_.n_reads = pd.n;
        none_.read_off = zeros_.data();
        rows_.view_ = &none_;
        held_ = 1;
        held_pipe_ = false;
        return rows_;
    }
    if (devices_.size() > 1) {
        rows_ = std::move(group_rows_);
        group_rows_ = BwaRows();
        held_ = 1;
        held_pipe_ = false;
        return rows_;
    }
    const bsq_hits *v = nullptr;
    const uint8_t *cols = nullptr;
    const int64_t *off = nullptr;
    const int rc = bsq_pipeline_next(pipe_, &v, &cols, &off);
    if (rc != BSQ_OK) {   // a failed submission has freed its slot
        --in_pipe_;
        throw BsqFailure(rc, bsq_last_error());
    }
    rows_.view_ = v;
    rows_.cols_ = pd.cols ? cols : nullptr;
    rows_.col_off_ = pd.cols ? off : nullptr;
    held_ = 1;
    held_pipe_ = true;
    return rows_;
}

void BwaIndex::release_rows() const
{
    if (!held_) return;
    rows_ = BwaRows();
    if (held_pipe_) {
        bsq_pipeline_release(pipe_);
        --in_pipe_;
    }
    held_ = 0;
    held_pipe_ = false;
}

void BwaIndex::reset_rows() const
{
    release_rows();
    while (!pending_.empty()) {
        try {
            take_rows();
        } catch (const BsqFailure &) {   // a failed submission: nothing to release
            continue;
        }
        release_rows();
    }
}

const BwaRows &BwaIndex::align_rows(const NucleotideSequence *const *seqs, int32_t n, bool nuclseq_columns,
                                    const BsqMemOpt *opts) const
{
    std::lock_guard<std::mutex> lk(mu_);
    reset_rows();   // the previous call's rows are released here (they were valid until this call)
    submit_rows(seqs, n, nuclseq_columns, opts);
    return take_rows();
}

std::vector<std::vector<BwaMatch>> BwaIndex::align_sequences(const std::vector<const NucleotideSequence *> &seqs) const
{
    std::vector<std::vector<BwaMatch>> res(seqs.size());
    const BwaRows &rows = align_rows(seqs.data(), (int32_t)seqs.size(), false);
    std::string cig;
    for (size_t i = 0; i < seqs.size(); ++i) {
        const int64_t b = rows.begin((int32_t)i), e = rows.end((int32_t)i);
        if (b == e) continue;
        std::unique_ptr<char, CFree> text(bsq_nuclseq_to_text(seqs[i]));   // to_text_palloc (bwa.cpp:146)
        if (!text) throw BsqFailure(BSQ_E_NOMEM, "out of memory rendering a read");
        for (int64_t k = b; k < e; ++k) {
            const bsq_hit &h = rows.row(k);
            BwaMatch m;
            m.ref_id = h.ref_id;
            m.ref_subseq.resize((size_t)(h.re - h.rb));
            if (bsq_index_ref_subseq(index_, h.rb, h.re, &m.ref_subseq[0]) != h.re - h.rb)
                throw BsqFailure(BSQ_E_INVALID, "row outside the reference");
            m.ref_match_begin = h.ref_match_start;
            m.ref_match_end = h.ref_match_end;
            m.ref_match_len = h.ref_match_len;
            m.query_subseq.assign(text.get() + h.qb, (size_t)(h.qe - h.qb));
            m.query_match_begin = h.qb;
            m.query_match_end = h.qe;
            m.query_match_len = h.qe - h.qb;
            m.is_primary = h.is_primary != 0;
            m.is_secondary = h.is_secondary != 0;
            m.is_reverse = h.is_reverse != 0;
            rows.cigar_text(k, cig);
            m.cigar = cig;
            m.score = h.score;
            res[i].push_back(std::move(m));
        }
    }
    return res;
}

std::vector<BwaMatch> BwaIndex::align_sequence(const NucleotideSequence &seq) const
{
    return std::move(align_sequences({&seq})[0]);
}

// ---- cross-call cache ---------------------------------------------------------------------------

void RefDigest::update(int64_t id, const void *nuclseq)
{
    // Two 64-bit lanes of a multiply-rotate mix over 8-byte words (not cryptographic: a collision between two
    // reference cursors of one backend is what it guards against, at ~2^-128).
    auto mix = [](uint64_t h, uint64_t w, uint64_t k) {
        h ^= w * k;
        h = (h << 31) | (h >> 33);
        return h * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
    };
    const size_t n = ns_bytes(nuclseq);
    h0 = mix(h0, (uint64_t)id, 0xFF51AFD7ED558CCDull);
    h1 = mix(h1, (uint64_t)n, 0xC4CEB9FE1A85EC53ull);
    const uint8_t *p = static_cast<const uint8_t *>(nuclseq) + 4;   // the length word's flag bits excluded
    size_t i = 4;
    for (; i + 16 <= n; i += 16, p += 16) {
        uint64_t a, b;
        memcpy(&a, p, 8);
        memcpy(&b, p + 8, 8);
        h0 = mix(h0, a, 0x87C37B91114253D5ull);
        h1 = mix(h1, b, 0x4CF5AD432745937Full);
    }
    if (i + 8 <= n) {
        uint64_t a;
        memcpy(&a, p, 8);
        h1 = mix(h1, a, 0x4CF5AD432745937Full);
        i += 8;
        p += 8;
    }
    uint64_t t = 0;
    memcpy(&t, p, n - i);
    h0 = mix(h0, t ^ (uint64_t)(n - i), 0x87C37B91114253D5ull);
    h1 ^= h0;
    ++rows;
    bytes += n;
}

BwaIndexCache &BwaIndexCache::backend()
{
    static BwaIndexCache c;
    return c;
}

std::shared_ptr<BwaIndex> BwaIndexCache::get_or_build(const RefDigest &d, std::shared_ptr<BwaIndex> fresh)
{
    const char *e = getenv("BSQ_INDEX_CACHE");
    const size_t cap = e ? (size_t)std::max(0, atoi(e)) : 2;
    std::lock_guard<std::mutex> lk(mu_);
    for (auto it = lru_.begin(); it != lru_.end(); ++it) {
        if (it->d == d && it->devices == fresh->devices() && it->idx->same_refs(*fresh)) {
            lru_.splice(lru_.begin(), lru_, it);
            ++hits_;
            return lru_.front().idx;
        }
    }
    fresh->build();
    ++builds_;
    if (cap) {
        lru_.push_front(Entry{d, fresh->devices(), fresh});
        while (lru_.size() > cap) lru_.pop_back();
    }
    return fresh;
}

void BwaIndexCache::clear()
{
    std::lock_guard<std::mutex> lk(mu_);
    lru_.clear();
    hits_ = builds_ = 0;
}
