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
    : options(o.options), index_(o.index_), devices_(o.devices_), group_(o.group_), batch_(o.batch_),
      batch_reads_(o.batch_reads_), batch_bases_(o.batch_bases_), rows_(std::move(o.rows_))
{
    o.options = nullptr;
    o.index_ = nullptr;
    o.group_ = nullptr;
    o.batch_ = nullptr;
}

BwaIndex::~BwaIndex()
{
    rows_ = BwaRows();
    bsq_batch_free(batch_);
    bsq_group_free(group_);
    bsq_index_free(index_);
    delete options;
}

void BwaIndex::add_ref_sequence(int64_t id, const NucleotideSequence &seq) { check(bsq_index_add_ref(index_, id, &seq)); }

bool BwaIndex::empty() const { return bsq_index_l_pac(index_) <= 0; }

int32_t BwaIndex::n_refs() const { return bsq_index_n_refs(index_); }

void BwaIndex::build()
{
    if (empty()) return;   // bwa.cpp:108-109
    if (bsq_device_count() > device()) check(bsq_index_build_device(index_, device()));
    else check(bsq_index_build(index_, 0));   // same tables; aligning then reports the missing device
}

void BwaIndex::ensure_batch(int32_t n, int64_t bases) const
{
    if (batch_ && batch_reads_ >= n && batch_bases_ >= bases) return;
    check(bsq_index_upload(index_, device()));   // no-op for an index built on the device
    rows_ = BwaRows();
    bsq_batch_free(batch_);
    batch_ = nullptr;
    // grow geometrically so a cursor's fetches of similar size reuse one workspace
    const int32_t r = std::max<int32_t>(n, std::min<int64_t>(2LL * batch_reads_, 1 << 20));
    const int64_t b = std::max<int64_t>(bases, std::min<int64_t>(2 * batch_bases_, (int64_t)r * 1024));
    check(bsq_batch_create(index_, std::max(r, 1), std::max<int64_t>(b, 1), &batch_));
    batch_reads_ = std::max(r, 1);
    batch_bases_ = std::max<int64_t>(b, 1);
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

const BwaRows &BwaIndex::align_rows(const NucleotideSequence *const *seqs, int32_t n, bool nuclseq_columns,
                                    const BsqMemOpt *opts) const
{
    std::lock_guard<std::mutex> lk(mu_);
    rows_ = BwaRows();
    if (n <= 0 || empty()) {   // bwa.cpp:142-143: no mem_align1 call, no lrand48 value drawn
        static thread_local std::vector<int64_t> zeros;
        static thread_local bsq_hits none;
        zeros.assign((size_t)std::max(n, 0) + 1, 0);
        none = kNoHits;
        none.n_reads = std::max(n, 0);
        none.read_off = zeros.data();
        rows_.view_ = &none;
        return rows_;
    }
    int64_t bases = 0;
    for (int32_t i = 0; i < n; ++i) bases += ns_len(seqs[i]);
    const void *const *ptrs = reinterpret_cast<const void *const *>(seqs);
    const bsq_opts o = (opts ? *opts : *options).c_abi();
    uint64_t &calls = bsq_backend_lrand48_calls();
    if (devices_.size() > 1) {   // the fetch spread over the group, member k taking a contiguous share
        ensure_group();
        check(bsq_group_run(group_, &o, ptrs, n, calls));
        rows_.view_ = bsq_group_hits(group_);
    } else {
        ensure_batch(n, bases);
        check(bsq_batch_set_nuclseqs(batch_, ptrs, n));
        check(bsq_batch_run(batch_, &o, calls));
        rows_.view_ = bsq_batch_hits(batch_);
    }
    calls += (uint64_t)n;
    if (nuclseq_columns && rows_.view_->n_hits > 0) {
        uint8_t *cols = nullptr;
        int64_t *off = nullptr;
        check(group_ ? bsq_group_render_nuclseqs(group_, ptrs, &cols, &off)
                     : bsq_batch_render_nuclseqs(batch_, ptrs, &cols, &off));
        rows_.cols_.reset(cols);
        rows_.col_off_.reset(off);
    }
    return rows_;
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
        if (it->d == d && it->devices == fresh->devices()) {
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
