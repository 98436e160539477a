// bwa_bsq.h -- drop-in replacement for bioseqdb/bwa.h (class BwaIndex, struct BwaMatch) over libbsq, the
// MI355X alignment path.  The reference's public interface (bwa.h:15-48) is kept member for member; the
// additions are what a batched, GPU-resident backend needs:
//
//   * BwaIndex::align_rows()      one GPU call for a whole SPI fetch: numeric records, CIGAR ops and the two
//                                 nuclseq columns of every bwa_result row (build_tuple_bwa's two
//                                 nuclseq_from_text calls, extension.cpp:285,290, rendered on the GPU);
//   * submit_rows/take_rows       the same as a pipeline (bsq_pipeline): a fetch is staged and released at
//                                 once, up to pipeline_depth() fetches align on the device while the backend
//                                 fetches the next rows and builds the previous fetch's tuples;
//   * explicit per-call options   a cached index serves calls with different bwa_options;
//   * BwaIndexCache               the index of a reference cursor kept across calls (the reference rebuilds
//                                 it on every call, Q13: extension.cpp:326,359), keyed by a digest of the
//                                 rows' ids and nuclseq bytes;
//   * several devices             BwaIndex({0, 1, ...}) aligns each batch over a bsq_group (one process, one
//                                 RCCL communicator per GPU, the index broadcast once);
//   * failures                    libbwa never fails; libbsq can (no device, HIP error, a read beyond every
//                                 retry capacity).  They surface as BsqFailure, which the fmgr layer turns into
//                                 ereport(ERROR) only after every C++ object is released (extension_bsq.cpp).
#pragma once

#include <cstdint>
#include <list>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "bsq.h"

struct NucleotideSequence;   // sequence.h:18-38; only its varlena bytes are read

struct BwaMatch {            // bwa.h:15-30, field for field (query_subseq owns its text here)
    int64_t ref_id;
    std::string ref_subseq;
    int32_t ref_match_begin;
    int32_t ref_match_end;
    int32_t ref_match_len;
    std::string query_subseq;
    int32_t query_match_begin;
    int32_t query_match_end;
    int32_t query_match_len;
    bool is_primary;
    bool is_secondary;
    bool is_reverse;
    std::string cigar;
    int score;
};

// The mem_opt_t fields extension.cpp:220-231 assigns, with the same member names and mem_opt_init values.
struct BsqMemOpt {
    int max_occ = 500, min_seed_len = 19, a = 1, b = 4, pen_clip3 = 5, pen_clip5 = 5, zdrop = 100, w = 100;
    int o_del = 6, o_ins = 6, e_del = 1, e_ins = 1;
    bsq_opts c_abi() const
    {
        return bsq_opts{min_seed_len, max_occ, a, b, pen_clip3, pen_clip5, zdrop, w, o_del, e_del, o_ins, e_ins};
    }
};

struct BsqFailure : std::runtime_error {
    int code;
    BsqFailure(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

// The rows of one aligned batch, valid until the next align call on the same index.
class BwaRows {
public:
    int32_t n_reads() const { return view_ ? view_->n_reads : 0; }
    int64_t n_rows() const { return view_ ? view_->n_hits : 0; }
    int64_t begin(int32_t read) const { return view_->read_off[read]; }   // rows of read i: [begin(i), end(i))
    int64_t end(int32_t read) const { return view_->read_off[read + 1]; }
    const bsq_hit &row(int64_t k) const { return view_->hits[k]; }
    // cigar_compressed_to_string (bwa.cpp:70-77) with htslib's "MIDNSHP=XB" letters (Q8)
    void cigar_text(int64_t k, std::string &out) const;
    // nuclseq varlenas of ref_subseq / query_subseq (nullptr unless align_rows asked for the columns)
    const void *ref_subseq(int64_t k) const { return cols_ ? cols_ + col_off_[2 * k] : nullptr; }
    const void *query_subseq(int64_t k) const { return cols_ ? cols_ + col_off_[2 * k + 1] : nullptr; }

private:
    friend class BwaIndex;
    struct Free { void operator()(void *p) const { bsq_free(p); } };
    const bsq_hits *view_ = nullptr;
    const uint8_t *cols_ = nullptr;             // borrowed from the pipeline slot, or owned below
    const int64_t *col_off_ = nullptr;
    std::unique_ptr<uint8_t, Free> own_cols_;   // columns rendered over a device group
    std::unique_ptr<int64_t, Free> own_off_;
};

class BwaIndex {
public:
    explicit BwaIndex(int device = 0);
    explicit BwaIndex(const std::vector<int> &devices);   // several: a bsq_group over them
    ~BwaIndex();
    BwaIndex(BwaIndex &&o) noexcept;
    BwaIndex(const BwaIndex &) = delete;
    BwaIndex &operator=(const BwaIndex &) = delete;

    // bwa.h:37-39
    std::vector<BwaMatch> align_sequence(const NucleotideSequence &seq) const;
    void build();   // on the GPU (bsq_index_build_device) when the device is visible, else on the host
    void add_ref_sequence(int64_t id, const NucleotideSequence &seq);

    // Every read of a cursor batch in one GPU call; result[i] are the matches of seqs[i].
    std::vector<std::vector<BwaMatch>> align_sequences(const std::vector<const NucleotideSequence *> &seqs) const;
    // The same as records; with nuclseq_columns the rows' two nuclseq columns are rendered on the GPU too.
    // `opts` overrides `options` (a cached index serves calls with different bwa_options).
    const BwaRows &align_rows(const NucleotideSequence *const *seqs, int32_t n, bool nuclseq_columns,
                              const BsqMemOpt *opts = nullptr) const;

    // Pipelined align_rows for a cursor (bsq_pipeline on one device; a device group runs each fetch at submit):
    // submit_rows copies the fetch, so its tuples may be released on return, and starts it on the device;
    // take_rows waits for the oldest submitted fetch and lends its rows until release_rows.  At most
    // pipeline_depth() fetches may be submitted and not released.  Rows come back in submission order, with
    // lrand48 positions as if aligned one after another.  Not for concurrent use by several threads.
    // deferred = true: the fetch is staged by a pipeline worker instead of on this thread; `seqs` and the values
    // they point to must then stay valid until wait_staged() has passed the returned ticket (group and empty fetches
    // are done at submit and return ticket -1).
    int64_t submit_rows(const NucleotideSequence *const *seqs, int32_t n, bool nuclseq_columns,
                        const BsqMemOpt *opts = nullptr, bool deferred = false) const;
    // every deferred fetch up to and including `ticket` has been staged (its tuples may be freed)
    void wait_staged(int64_t ticket) const;
    const BwaRows &take_rows() const;
    void release_rows() const;
    int pipeline_depth() const;
    // Releases the taken rows and discards submissions nobody took (e.g. left by a call that failed midway).
    void reset_rows() const;

    bool empty() const;          // no reference bases: align_* return no rows and draw no lrand48 value
    int32_t n_refs() const;
    bool same_refs(const BwaIndex &o) const;   // given the same reference rows (the cache's content check)
    int device() const { return devices_[0]; }
    const std::vector<int> &devices() const { return devices_; }

    BsqMemOpt *options;          // bwa.h:41 (mem_opt_t* there)

private:
    void ensure_pipe() const;
    void ensure_group() const;
    bsq_index *index_;
    std::vector<int> devices_;
    mutable bsq_group *group_ = nullptr;
    mutable bsq_pipeline *pipe_ = nullptr;
    struct Pending { bool cols = false, empty = false; int32_t n = 0; };
    mutable std::list<Pending> pending_;   // submitted, not yet taken (group / empty fetches run at submit)
    mutable int held_ = 0;                 // taken, not yet released (0 or 1)
    mutable bool held_pipe_ = false;       // ... and it occupies a slot of pipe_
    mutable BwaRows group_rows_;           // rows of the pending group fetch (aligned and rendered at submit)
    mutable int in_pipe_ = 0;              // submissions inside pipe_ not yet released
    mutable bool group_ready_ = false;     // the group holds the rows of the one pending group fetch
    mutable std::vector<int64_t> zeros_;   // read offsets of an empty fetch
    mutable bsq_hits none_{};
    mutable BwaRows rows_;
    mutable std::mutex mu_;      // align_rows on a shared (cached) index is serialised
};

// Position of this backend in the process-global lrand48 stream (Q10); every aligned read consumes one value,
// as libbwa's mem_align1 does (bwa.cpp:149).
uint64_t &bsq_backend_lrand48_calls();

// Digest of a reference cursor: 128 bits over each row's id and nuclseq varlena bytes, in cursor order.
// On a cache hit the index's own contents are compared too (BwaIndex::same_rows: row count, ids, lengths, bases
// and holes), so a digest collision cannot hand back another reference's index.
struct RefDigest {
    uint64_t h0 = 0x9E3779B97F4A7C15ull, h1 = 0xC2B2AE3D27D4EB4Full, rows = 0, bytes = 0;
    void update(int64_t id, const void *nuclseq);
    bool operator==(const RefDigest &o) const { return h0 == o.h0 && h1 == o.h1 && rows == o.rows && bytes == o.bytes; }
};

// Built indexes of this backend, most recently used first.  Capacity from
// BSQ_INDEX_CACHE (default 2, 0 disables).  Options are per call and not part of the key.
class BwaIndexCache {
public:
    static BwaIndexCache &backend();
    // The cached index for (digest, devices), or `fresh` after building it (and caching it).
    std::shared_ptr<BwaIndex> get_or_build(const RefDigest &d, std::shared_ptr<BwaIndex> fresh);
    void clear();
    size_t hits() const { return hits_; }
    size_t builds() const { return builds_; }

private:
    struct Entry { RefDigest d; std::vector<int> devices; std::shared_ptr<BwaIndex> idx; };
    std::list<Entry> lru_;
    std::mutex mu_;
    size_t hits_ = 0, builds_ = 0;
};
