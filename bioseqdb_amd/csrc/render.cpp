// render.cpp -- bwa_result row rendering (reference: BwaIndex::align_sequence's BwaMatch fields,
// bioseqdb/bwa.cpp:159-175, extract_reference_subseq :55-68, cigar_compressed_to_string :70-77,
// and the htslib bam_cigar_opchr table "MIDNSHP=XB", so libbwa's clip op 3 prints as 'N' -- Q8).
//
// Host materialisation: once alignment runs on the GPU, rendering the rows is the
// host's share of every cursor batch, so it runs on all host cores (reads split by hit count, one text
// buffer per thread, concatenated in read order), looks holes up by offset instead of scanning every
// hole for every row, and formats integers without temporaries.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <queue>
#include <string>
#include <thread>
#include <vector>

#include "../../include/bsq.h"
#include "bsq_index.h"

using namespace bsq;

bsq::HoleIndex::HoleIndex(const std::vector<Hole> &holes)
{
    std::vector<uint32_t> by_beg;
    std::vector<int64_t> cuts;   // every start and end, sorted, distinct
    for (size_t i = 0; i < holes.size(); ++i)
        if (holes[i].len > 0) {
            by_beg.push_back((uint32_t)i);
            cuts.push_back(holes[i].offset);
            cuts.push_back(holes[i].offset + holes[i].len);
        }
    std::sort(by_beg.begin(), by_beg.end(), [&](uint32_t a, uint32_t b) { return holes[a].offset < holes[b].offset; });
    std::sort(cuts.begin(), cuts.end());
    cuts.erase(std::unique(cuts.begin(), cuts.end()), cuts.end());
    std::priority_queue<uint32_t> live;   // hole indices = overwrite order
    size_t si = 0;
    for (size_t c = 0; c + 1 < cuts.size(); ++c) {
        const int64_t a = cuts[c], b = cuts[c + 1];
        while (si < by_beg.size() && holes[by_beg[si]].offset <= a) live.push(by_beg[si++]);
        while (!live.empty() && holes[live.top()].offset + holes[live.top()].len <= a) live.pop();
        if (live.empty()) continue;
        const uint32_t w = live.top();
        if (!segs.empty() && segs.back().end == a && segs.back().amb == holes[w].amb) segs.back().end = b;
        else segs.push_back(HoleRef{a, b, w, holes[w].amb});
    }
}

namespace {

void ref_subseq(const HostIndex &h, const HoleIndex &hx, int64_t rb, int64_t re, std::string &out)
{
    const size_t base = out.size();
    out.resize(base + (size_t)(re - rb));
    char *s = &out[base];
    if (rb < h.l_pac) {
        for (int64_t i = 0; i < re - rb; ++i) s[i] = "ACGT"[pac_get(h.pac.data(), (uint64_t)(rb + i))];
        for (size_t k = hx.first_after(rb); k < hx.segs.size() && hx.segs[k].beg < re; ++k) {
            const int64_t lo = std::max<int64_t>(hx.segs[k].beg, rb), hi = std::min<int64_t>(hx.segs[k].end, re);
            for (int64_t i = lo; i < hi; ++i) s[i - rb] = hx.segs[k].amb;
        }
    } else {
        // Q7: the reference reads past the forward pac here (undefined behaviour); render the
        // reverse-strand reference text instead.
        for (int64_t i = 0; i < re - rb; ++i)
            s[i] = "ACGT"[3 - pac_get(h.pac.data(), (uint64_t)((h.l_pac << 1) - 1 - (rb + i)))];
    }
}

inline void put_int(std::string &out, int64_t v)
{
    char buf[24];
    int n = 0;
    const bool neg = v < 0;
    uint64_t u = neg ? (uint64_t)(-(v + 1)) + 1 : (uint64_t)v;
    do { buf[n++] = (char)('0' + u % 10); u /= 10; } while (u);
    if (neg) buf[n++] = '-';
    while (n) out += buf[--n];
}

void render_reads(const HostIndex &h, const HoleIndex &hx, const bsq_hits *hits, const void *const *reads, int32_t r0,
                  int32_t r1, std::string &out)
{
    std::string text;
    for (int32_t r = r0; r < r1; ++r) {
        const int64_t b = hits->read_off[r], e = hits->read_off[r + 1];
        if (b == e) continue;
        text = ns_to_text(static_cast<const uint8_t *>(reads[r]));
        for (int64_t k = b; k < e; ++k) {
            const bsq_hit &x = hits->hits[k];
            put_int(out, x.ref_id); out += '\t';
            ref_subseq(h, hx, x.rb, x.re, out); out += '\t';
            put_int(out, x.ref_match_start); out += '\t';
            put_int(out, x.ref_match_end); out += '\t';
            put_int(out, x.ref_match_len); out += '\t';
            out.append(text, (size_t)x.qb, (size_t)(x.qe - x.qb)); out += '\t';
            put_int(out, x.qb); out += '\t';
            put_int(out, x.qe); out += '\t';
            put_int(out, x.qe - x.qb); out += '\t';
            out += x.is_primary ? 't' : 'f'; out += '\t';
            out += x.is_secondary ? 't' : 'f'; out += '\t';
            out += x.is_reverse ? 't' : 'f'; out += '\t';
            for (uint32_t c = 0; c < x.n_cigar; ++c) {
                const uint32_t v = hits->cigar[x.cigar_off + c];
                put_int(out, v >> 4);
                out += "MIDNSHP=XB"[v & 0xf];
            }
            out += '\t';
            put_int(out, x.score);
            out += '\n';
        }
    }
}

int render_threads(int64_t n_hits)
{
    const char *e = getenv("BSQ_RENDER_THREADS");
    int t = e ? atoi(e) : (int)std::thread::hardware_concurrency();
    t = std::max(1, std::min(t, 16));
    return (int)std::max<int64_t>(1, std::min<int64_t>(t, n_hits / 2048 + 1));   // small batches: one thread
}

}  // namespace

extern "C" int64_t bsq_index_ref_subseq(const bsq_index *idx, int64_t rb, int64_t re, char *out)
{
    if (!idx || !idx->h.built || rb < 0 || re < rb || re > 2 * idx->h.l_pac) return -1;
    if (!out) return re - rb;
    std::string s;
    ref_subseq(idx->h, const_cast<bsq_index *>(idx)->holes(), rb, re, s);
    memcpy(out, s.data(), s.size());
    return (int64_t)s.size();
}

extern "C" char *bsq_render_tsv(const bsq_index *idx, const bsq_hits *hits, const void *const *reads)
{
    if (!idx || !hits) return nullptr;
    const HoleIndex &hx = const_cast<bsq_index *>(idx)->holes();
    const int32_t n = hits->n_reads;
    const int T = n > 0 ? render_threads(hits->n_hits) : 1;
    std::vector<std::string> part((size_t)T);
    std::vector<int32_t> cut((size_t)T + 1, n);
    cut[0] = 0;
    for (int t = 1; t < T; ++t) {   // equal numbers of rows per thread
        const int64_t target = hits->n_hits * t / T;
        cut[t] = (int32_t)(std::lower_bound(hits->read_off, hits->read_off + n, target) - hits->read_off);
        cut[t] = std::max(cut[t], cut[t - 1]);
    }
    auto work = [&](int t) {
        part[t].reserve((size_t)((hits->n_hits / T + 1) * 400));
        render_reads(idx->h, hx, hits, reads, cut[t], cut[t + 1], part[t]);
    };
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back(work, t);
    work(0);
    for (auto &x : th) x.join();
    size_t total = 0;
    for (auto &p : part) total += p.size();
    char *s = (char *)malloc(total + 1);
    if (!s) return nullptr;
    size_t o = 0;
    for (auto &p : part) { memcpy(s + o, p.data(), p.size()); o += p.size(); }
    s[o] = 0;
    return s;
}
