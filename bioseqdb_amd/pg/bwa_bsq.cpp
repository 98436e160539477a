// bwa_bsq.cpp -- BwaIndex over libbsq (replaces bioseqdb/bwa.cpp; see bwa_bsq.h).
#include "bwa_bsq.h"

#include <cstdlib>
#include <cstring>
#include <sstream>

namespace {
void check(int rc)
{
    if (rc != BSQ_OK) throw BsqFailure(rc, bsq_last_error());
}

std::vector<BwaMatch> parse_rows(const char *tsv, size_t n_rows)
{
    std::vector<BwaMatch> out;
    out.reserve(n_rows);
    std::istringstream in(tsv);
    std::string line;
    while (std::getline(in, line)) {
        std::vector<std::string> f;
        size_t s = 0, e;
        while ((e = line.find('\t', s)) != std::string::npos) { f.push_back(line.substr(s, e - s)); s = e + 1; }
        f.push_back(line.substr(s));
        if (f.size() != 14) throw BsqFailure(BSQ_E_INVALID, "malformed libbsq row");
        out.push_back(BwaMatch{std::stoll(f[0]), f[1], std::stoi(f[2]), std::stoi(f[3]), std::stoi(f[4]), f[5],
                               std::stoi(f[6]), std::stoi(f[7]), std::stoi(f[8]), f[9] == "t", f[10] == "t",
                               f[11] == "t", f[12], std::stoi(f[13])});
    }
    return out;
}
}  // namespace

uint64_t &bsq_backend_lrand48_calls()
{
    static uint64_t calls = 0;
    return calls;
}

BwaIndex::BwaIndex(int dev) : options(new BsqMemOpt()), index(nullptr), device(dev) { check(bsq_index_create(&index)); }

BwaIndex::BwaIndex(BwaIndex &&o) noexcept : options(o.options), index(o.index), device(o.device), uploaded(o.uploaded)
{
    o.options = nullptr;
    o.index = nullptr;
}

BwaIndex::~BwaIndex()
{
    bsq_index_free(index);
    delete options;
}

void BwaIndex::add_ref_sequence(int64_t id, const NucleotideSequence &seq) { check(bsq_index_add_ref(index, id, &seq)); }

void BwaIndex::build() { check(bsq_index_build(index, 0)); }

std::vector<std::vector<BwaMatch>> BwaIndex::align_sequences(const std::vector<const NucleotideSequence *> &seqs) const
{
    std::vector<std::vector<BwaMatch>> res(seqs.size());
    if (bsq_index_l_pac(index) <= 0 || seqs.empty()) return res;   // bwa.cpp:191: empty reference
    if (!uploaded) {
        check(bsq_index_upload(index, device));
        const_cast<BwaIndex *>(this)->uploaded = true;
    }
    const bsq_opts o{options->min_seed_len, options->max_occ, options->a, options->b, options->pen_clip3,
                     options->pen_clip5, options->zdrop, options->w, options->o_del, options->e_del,
                     options->o_ins, options->e_ins};
    std::vector<const void *> ptrs(seqs.begin(), seqs.end());
    uint64_t &calls = bsq_backend_lrand48_calls();
    bsq_hits *h = nullptr;
    check(bsq_align_batch(index, &o, ptrs.data(), (int32_t)ptrs.size(), calls, &h));
    calls += seqs.size();
    char *tsv = bsq_render_tsv(index, h, ptrs.data());
    std::vector<BwaMatch> all = parse_rows(tsv ? tsv : "", (size_t)h->n_hits);
    bsq_free(tsv);
    size_t k = 0;
    for (size_t i = 0; i < seqs.size(); ++i) {
        int64_t n = h->read_off[i + 1] - h->read_off[i];
        for (int64_t j = 0; j < n; ++j) res[i].push_back(std::move(all[k++]));
    }
    bsq_hits_free(h);
    return res;
}

std::vector<BwaMatch> BwaIndex::align_sequence(const NucleotideSequence &seq) const
{
    return align_sequences({&seq})[0];
}
