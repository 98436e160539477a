// bwa_bsq.h -- drop-in replacement for bioseqdb/bwa.h (class BwaIndex, struct BwaMatch) that keeps
// the reference's public interface (bwa.h:15-48) but runs the alignment path in libbsq on MI355X.
// Differences a caller can see: align_sequences() aligns a whole cursor batch in one GPU call, and
// failures (no device, HIP error) are reported by throwing BsqFailure instead of never failing
// (libbwa cannot fail); extension.cpp converts it to ereport(ERROR).
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

#include "bsq.h"

struct NucleotideSequence;   // sequence.h:18-38 (only its varlena bytes are read)

struct BwaMatch {            // bwa.h:15-30, field for field
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

// The mem_opt_t fields extension.cpp:220-231 assigns, with the same member names.
struct BsqMemOpt {
    int max_occ = 500, min_seed_len = 19, a = 1, b = 4, pen_clip3 = 5, pen_clip5 = 5, zdrop = 100, w = 100;
    int o_del = 6, o_ins = 6, e_del = 1, e_ins = 1;
};

struct BsqFailure : std::runtime_error {
    int code;
    BsqFailure(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

class BwaIndex {
public:
    explicit BwaIndex(int device = 0);
    ~BwaIndex();
    BwaIndex(BwaIndex &&o) noexcept;
    BwaIndex(const BwaIndex &) = delete;

    std::vector<BwaMatch> align_sequence(const NucleotideSequence &seq) const;
    // one GPU call for a batch of cursor rows; result[i] are the matches of seqs[i]
    std::vector<std::vector<BwaMatch>> align_sequences(const std::vector<const NucleotideSequence *> &seqs) const;
    void build();
    void add_ref_sequence(int64_t id, const NucleotideSequence &seq);

    BsqMemOpt *options;

private:
    bsq_index *index;
    int device;
    bool uploaded = false;
};

// Position of this backend in the process-global lrand48 stream (Q10); each align consumes one.
uint64_t &bsq_backend_lrand48_calls();
