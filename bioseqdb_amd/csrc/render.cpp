// render.cpp -- bwa_result row rendering (reference: BwaIndex::align_sequence's BwaMatch fields,
// bioseqdb/bwa.cpp:198-226, extract_reference_subseq :104-117, cigar_compressed_to_string :119-126,
// and the htslib bam_cigar_opchr table "MIDNSHP=XB", so libbwa's clip op 3 prints as 'N' -- Q8).
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/bsq.h"
#include "bsq_index.h"

using namespace bsq;


static std::string ref_subseq(const HostIndex &h, int64_t rb, int64_t re)
{
    std::string s((size_t)(re - rb), '?');
    if (rb < h.l_pac) {
        for (int64_t i = 0; i < re - rb; ++i) s[(size_t)i] = "ACGT"[pac_get(h.pac.data(), (uint64_t)(rb + i))];
        for (const Hole &hl : h.holes) {   // Q3: hole offsets are row-relative but compared as concatenated
            int64_t lo = std::max<int64_t>(hl.offset, rb), hi = std::min<int64_t>(hl.offset + hl.len, re);
            for (int64_t i = lo; i < hi; ++i) s[(size_t)(i - rb)] = hl.amb;
        }
    } else {
        // Q7: the reference reads past the forward pac here (undefined behaviour); render the
        // reverse-strand reference text instead.
        for (int64_t i = 0; i < re - rb; ++i)
            s[(size_t)i] = "ACGT"[3 - pac_get(h.pac.data(), (uint64_t)((h.l_pac << 1) - 1 - (rb + i)))];
    }
    return s;
}

extern "C" char *bsq_render_tsv(const bsq_index *idx, const bsq_hits *hits, const void *const *reads)
{
    if (!idx || !hits) return nullptr;
    std::string out;
    for (int32_t r = 0; r < hits->n_reads; ++r) {
        int64_t b = hits->read_off[r], e = hits->read_off[r + 1];
        if (b == e) continue;
        std::string text = ns_to_text(static_cast<const uint8_t *>(reads[r]));
        for (int64_t k = b; k < e; ++k) {
            const bsq_hit &x = hits->hits[k];
            out += std::to_string(x.ref_id); out += '\t';
            out += ref_subseq(idx->h, x.rb, x.re); out += '\t';
            out += std::to_string(x.ref_match_start); out += '\t';
            out += std::to_string(x.ref_match_end); out += '\t';
            out += std::to_string(x.ref_match_len); out += '\t';
            out.append(text, (size_t)x.qb, (size_t)(x.qe - x.qb)); out += '\t';
            out += std::to_string(x.qb); out += '\t';
            out += std::to_string(x.qe); out += '\t';
            out += std::to_string(x.qe - x.qb); out += '\t';
            out += x.is_primary ? 't' : 'f'; out += '\t';
            out += x.is_secondary ? 't' : 'f'; out += '\t';
            out += x.is_reverse ? 't' : 'f'; out += '\t';
            for (uint32_t c = 0; c < x.n_cigar; ++c) {
                uint32_t v = hits->cigar[x.cigar_off + c];
                out += std::to_string(v >> 4);
                out += "MIDNSHP=XB"[v & 0xf];
            }
            out += '\t';
            out += std::to_string(x.score);
            out += '\n';
        }
    }
    char *s = (char *)malloc(out.size() + 1);
    memcpy(s, out.c_str(), out.size() + 1);
    return s;
}
