// index_build.cpp -- host construction of the alignment index (the step before the hot path).
//
// Replaces BwaIndex::add_ref_sequence / BwaIndex::build (bioseqdb/bwa.cpp:82-128): the reference
// rows are concatenated byte-aligned exactly as the reference does (Q3/Q4), the text
// T = pac || revcomp(pac) is suffix-sorted (the BWT of T$ is unique, so any correct suffix sort
// reproduces libbwa's is_bwt + bwt_cal_sa output), and the result is laid out for HBM:
//   * OccBlock[ceil(n/128)]  -- 64-B rank blocks of the $-removed BWT (counts + 2 bit-planes)
//   * full SA (u32 when n < 2^32, else u64) -- one random 4/8-B read per seed instead of an
//     LF-walk over a 1/32-sampled SA (same values, SURVEY.md §5 "Long-context")
// The suffix sort is a parallel MSD bucket sort on 8-base prefixes, then per-bucket sorts on the
// next 32 bases with an exact tie-breaking comparison.
#include <algorithm>
#include <cstdlib>
#include <array>
#include <atomic>
#include <cstring>
#include <thread>

#include "../../include/bsq.h"
#include "bsq_index.h"

namespace bsq {

std::string ns_to_text(const uint8_t *ns)
{
    uint32_t len = ns_len(ns), nh = ns_holes_num(ns);
    const uint8_t *pac = ns_pac(ns);
    std::string t(len, '?');
    for (uint32_t i = 0; i < len; ++i) t[i] = "ACGT"[pac_get(pac, i)];
    for (uint32_t i = 0; i < nh; ++i) {
        Hole h = ns_hole(ns, i);
        for (int64_t j = h.offset; j < h.offset + h.len && j < (int64_t)len; ++j) t[(size_t)j] = h.amb;
    }
    return t;
}

void ns_to_nt4(const uint8_t *ns, std::vector<uint8_t> &out)
{
    uint32_t len = ns_len(ns), nh = ns_holes_num(ns);
    const uint8_t *pac = ns_pac(ns);
    size_t base = out.size();
    out.resize(base + len);
    uint8_t *o = out.data() + base;
    for (uint32_t i = 0; i < len; ++i) o[i] = (uint8_t)pac_get(pac, i);
    for (uint32_t i = 0; i < nh; ++i) {   // every hole symbol (N and IUPAC) is nt4 code 4
        Hole h = ns_hole(ns, i);
        int code = nt4((unsigned char)h.amb);
        for (int64_t j = h.offset; j < h.offset + h.len && j < (int64_t)len; ++j) o[j] = (uint8_t)(code < 4 ? code : 4);
    }
}

// nuclseq_from_text (sequence.cpp:209-245): holes are runs of one non-ACGT symbol; their bases and
// the padding bases up to the byte boundary are std::minstd_rand(holes_num ^ len)() & 3.
static std::vector<uint8_t> ns_from_text(const char *str, size_t len)
{
    uint32_t holes_num = 0;
    char prev = 0;
    for (size_t i = 0; i < len; ++i) {
        if (prev != str[i] && nt4((unsigned char)str[i]) >= 4) ++holes_num;
        prev = str[i];
    }
    const size_t size = 12 + 16 * (size_t)holes_num + pac_byte_size(len);
    std::vector<uint8_t> ns(size, 0);
    uint32_t vl = (uint32_t)(size << 2), l32 = (uint32_t)len;
    memcpy(&ns[0], &vl, 4); memcpy(&ns[4], &holes_num, 4); memcpy(&ns[8], &l32, 4);
    uint8_t *pac = &ns[12 + 16 * (size_t)holes_num];
    uint64_t x = ((uint64_t)holes_num ^ (uint64_t)len) % 2147483647ULL;   // std::minstd_rand seed
    if (x == 0) x = 1;
    auto rng = [&x]() { x = x * 48271ULL % 2147483647ULL; return (uint32_t)x; };
    auto set = [pac](uint64_t i, int v) { pac[i >> 2] |= (uint8_t)(v << ((~i & 3) << 1)); };
    uint8_t *hole = &ns[12] - 16;
    prev = 0;
    for (size_t i = 0; i < len; ++i) {
        char c = str[i];
        int code = nt4((unsigned char)c);
        if (code >= 4) {
            if (prev == c) {
                int32_t hl; memcpy(&hl, hole + 8, 4); ++hl; memcpy(hole + 8, &hl, 4);
            } else {
                hole += 16;
                int64_t off = (int64_t)i; int32_t hl = 1;
                memcpy(hole, &off, 8); memcpy(hole + 8, &hl, 4); hole[12] = (uint8_t)c;
            }
            set(i, rng() & 3);
        } else set(i, code);
        prev = c;
    }
    for (size_t i = len; i < pac_byte_size(len) * 4; ++i) set(i, rng() & 3);
    return ns;
}

void HostIndex::add_ref(int64_t id, const uint8_t *ns)
{
    uint32_t len = ns_len(ns), nh = ns_holes_num(ns);
    anns.push_back(Ann{(int64_t)pac.size() * 4, (int32_t)len, (int32_t)nh, id});
    size_t nb = pac_byte_size(len);
    const uint8_t *p = ns_pac(ns);
    pac.insert(pac.end(), p, p + nb);
    for (uint32_t i = 0; i < nh; ++i) holes.push_back(ns_hole(ns, i));   // Q3: offsets left unshifted
    built = false;
}

template <class F>
static void parallel_for(int threads, F f)
{
    std::vector<std::thread> th;
    for (int t = 1; t < threads; ++t) th.emplace_back(f, t);
    f(0);
    for (auto &x : th) x.join();
}

void HostIndex::occ4(uint64_t k, uint64_t c[4]) const
{
    if (k == (uint64_t)-1) { c[0] = c[1] = c[2] = c[3] = 0; return; }
    k -= (k >= primary);
    const OccBlock &b = occ[k >> 7];
    uint32_t r = (uint32_t)(k & 127) + 1;
    uint64_t m0 = r >= 64 ? ~0ull : ((1ull << r) - 1);
    uint64_t m1 = r >= 128 ? ~0ull : (r > 64 ? ((1ull << (r - 64)) - 1) : 0ull);
    uint32_t n3 = __builtin_popcountll(b.hi[0] & b.lo[0] & m0) + __builtin_popcountll(b.hi[1] & b.lo[1] & m1);
    uint32_t n2 = __builtin_popcountll(b.hi[0] & ~b.lo[0] & m0) + __builtin_popcountll(b.hi[1] & ~b.lo[1] & m1);
    uint32_t n1 = __builtin_popcountll(~b.hi[0] & b.lo[0] & m0) + __builtin_popcountll(~b.hi[1] & b.lo[1] & m1);
    c[0] = b.cnt[0] + (r - n1 - n2 - n3);
    c[1] = b.cnt[1] + n1;
    c[2] = b.cnt[2] + n2;
    c[3] = b.cnt[3] + n3;
}

int HostIndex::build(int threads, std::string &err)
{
    built = false;
    dev_built = false;
    occ.clear(); sa32.clear(); sa64.clear();
    if (pac.empty()) { built = true; l_pac = 0; seq_len = 0; return 0; }   // reference: index stays null
    if (threads < 1) threads = 1;
    l_pac = (int64_t)pac.size() * 4;
    const uint64_t n = (uint64_t)l_pac * 2;
    seq_len = n;
    // ---- T = forward || reverse complement (pac2bwt, bwa.cpp:20-53) ----
    std::vector<uint8_t> T(n);
    for (int c = 0; c < 5; ++c) L2[c] = 0;
    {
        std::vector<std::array<uint64_t, 4>> cnt(threads);
        parallel_for(threads, [&](int t) {
            uint64_t lo = (uint64_t)l_pac * t / threads, hi = (uint64_t)l_pac * (t + 1) / threads;
            std::array<uint64_t, 4> c{0, 0, 0, 0};
            for (uint64_t i = lo; i < hi; ++i) {
                uint8_t b = (uint8_t)pac_get(pac.data(), i);
                T[i] = b;
                T[n - 1 - i] = (uint8_t)(3 - b);
                ++c[b];
            }
            cnt[t] = c;
        });
        uint64_t fc[4] = {0, 0, 0, 0};
        for (auto &c : cnt) for (int b = 0; b < 4; ++b) fc[b] += c[b];
        for (int b = 0; b < 4; ++b) { L2[1 + b] += fc[b]; L2[4 - b] += fc[b]; }
        for (int i = 2; i <= 4; ++i) L2[i] += L2[i - 1];
    }
    auto key_at = [&](uint64_t i, int nb) -> uint64_t {   // nb bases from i, padded with A beyond the end
        uint64_t k = 0;
        if (i + nb <= n) { for (int j = 0; j < nb; ++j) k = k << 2 | T[i + j]; }
        else { for (int j = 0; j < nb; ++j) k = k << 2 | (i + j < n ? T[i + j] : 0); }
        return k;
    };
    // ---- bucket by first 8 bases ----
    const int NB = 1 << 16;
    std::vector<uint64_t> hist((size_t)threads * NB, 0);
    parallel_for(threads, [&](int t) {
        uint64_t lo = n * t / threads, hi = n * (t + 1) / threads;
        uint64_t *h = &hist[(size_t)t * NB];
        for (uint64_t i = lo; i < hi; ++i) ++h[key_at(i, 8)];
    });
    std::vector<uint64_t> bstart(NB + 1, 0);
    {
        uint64_t acc = 0;
        for (int b = 0; b < NB; ++b) {
            bstart[b] = acc;
            for (int t = 0; t < threads; ++t) { uint64_t c = hist[(size_t)t * NB + b]; hist[(size_t)t * NB + b] = acc; acc += c; }
        }
        bstart[NB] = acc;
    }
    // 64-bit rows for texts of >= 2^32 rows; BSQ_FORCE_WIDE=1 selects them for any size (tests of the
    // 3 Gbp code path on small references)
    const char *fw = getenv("BSQ_FORCE_WIDE");
    const bool wide = n >= 0xFFFFFFFFull || (fw && *fw && *fw != '0');
    std::vector<uint64_t> idx64;
    std::vector<uint32_t> idx32;
    if (wide) idx64.resize(n); else idx32.resize(n);
    parallel_for(threads, [&](int t) {
        uint64_t lo = n * t / threads, hi = n * (t + 1) / threads;
        uint64_t *h = &hist[(size_t)t * NB];
        for (uint64_t i = lo; i < hi; ++i) {
            uint64_t b = key_at(i, 8);
            if (wide) idx64[h[b]++] = i; else idx32[h[b]++] = (uint32_t)i;
        }
    });
    hist.clear(); hist.shrink_to_fit();
    // ---- sort each bucket on the next 32 bases, exact comparison on ties ----
    auto suffix_less = [&](uint64_t i, uint64_t j) -> bool {
        uint64_t li = n - i, lj = n - j, m = li < lj ? li : lj;
        if (m > 40) {
            int c = memcmp(&T[i + 40], &T[j + 40], (size_t)(m - 40));
            if (c) return c < 0;
        }
        return li < lj;   // the shorter suffix reaches $ first
    };
    std::atomic<int> next{0};
    parallel_for(threads, [&](int) {
        std::vector<std::pair<uint64_t, uint64_t>> v;
        for (;;) {
            int b = next.fetch_add(1);
            if (b >= NB) break;
            uint64_t s = bstart[b], e = bstart[b + 1];
            if (e - s <= 1) continue;
            v.resize(e - s);
            for (uint64_t j = s; j < e; ++j) {
                uint64_t i = wide ? idx64[j] : idx32[j];
                v[j - s] = {key_at(i + 8 < n ? i + 8 : n, 32), i};
            }
            std::sort(v.begin(), v.end(), [&](const std::pair<uint64_t, uint64_t> &a, const std::pair<uint64_t, uint64_t> &c) {
                if (a.first != c.first) return a.first < c.first;
                return suffix_less(a.second, c.second);
            });
            for (uint64_t j = s; j < e; ++j) {
                if (wide) idx64[j] = v[j - s].second; else idx32[j] = (uint32_t)v[j - s].second;
            }
        }
    });
    // SA rows: row 0 is the $ suffix (position n), then the sorted suffixes
    if (wide) {
        sa64.resize(n + 1);
        sa64[0] = n;
        std::copy(idx64.begin(), idx64.end(), sa64.begin() + 1);
        idx64.clear(); idx64.shrink_to_fit();
    } else {
        sa32.resize(n + 1);
        sa32[0] = (uint32_t)n;
        std::copy(idx32.begin(), idx32.end(), sa32.begin() + 1);
        idx32.clear(); idx32.shrink_to_fit();
    }
    // ---- BWT ($ removed) -> occ blocks ----
    primary = (uint64_t)-1;
    for (uint64_t r = 0; r <= n; ++r) if (sa(r) == 0) { primary = r; break; }
    if (primary == (uint64_t)-1) { err = "suffix array has no row for position 0"; return -1; }
    const uint64_t nblk = (n + 127) / 128 + 1;
    occ.assign(nblk, OccBlock{});
    std::vector<std::array<uint64_t, 4>> bcnt(nblk);
    parallel_for(threads, [&](int t) {
        uint64_t b0 = nblk * t / threads, b1 = nblk * (t + 1) / threads;
        for (uint64_t b = b0; b < b1; ++b) {
            OccBlock &ob = occ[b];
            std::array<uint64_t, 4> c{0, 0, 0, 0};
            for (int j = 0; j < 128; ++j) {
                uint64_t p = b * 128 + (uint64_t)j;
                if (p >= n) break;
                uint64_t row = p + (p >= primary);
                uint8_t ch = T[sa(row) - 1];
                ++c[ch];
                if (ch & 2) ob.hi[j >> 6] |= 1ull << (j & 63);
                if (ch & 1) ob.lo[j >> 6] |= 1ull << (j & 63);
            }
            bcnt[b] = c;
        }
    });
    {
        uint64_t acc[4] = {0, 0, 0, 0};
        for (uint64_t b = 0; b < nblk; ++b) {
            for (int c = 0; c < 4; ++c) { occ[b].cnt[c] = acc[c]; acc[c] += bcnt[b][c]; }
        }
    }
    built = true;
    return 0;
}

}  // namespace bsq

extern "C" void *bsq_nuclseq_from_text(const char *text, size_t len, size_t *out_size)
{
    if (!text && len) return nullptr;
    std::vector<uint8_t> v = bsq::ns_from_text(text, len);
    void *p = malloc(v.size());
    if (!p) return nullptr;
    memcpy(p, v.data(), v.size());
    if (out_size) *out_size = v.size();
    return p;
}

extern "C" char *bsq_nuclseq_to_text(const void *nuclseq)
{
    if (!nuclseq) return nullptr;
    std::string t = bsq::ns_to_text(static_cast<const uint8_t *>(nuclseq));
    char *p = (char *)malloc(t.size() + 1);
    if (!p) return nullptr;
    memcpy(p, t.c_str(), t.size() + 1);
    return p;
}
