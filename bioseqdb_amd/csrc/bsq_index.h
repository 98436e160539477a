// bsq_index.h -- host-side index object behind the C-ABI (replaces bioseqdb's BwaIndex storage,
// bioseqdb/bwa.h:32-48, and libbwa's bwt_t/bntseq_t built in BwaIndex::build, bwa.cpp:107-128).
#pragma once
#include <stdint.h>

#include <algorithm>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "bsq_device.h"

namespace bsq {

struct Hole { int64_t offset; int32_t len; char amb; };           // bntamb1_t
struct Ann { int64_t offset; int32_t len, n_ambs; int64_t id; };    // bntann1_t subset (name = id)

// nuclseq varlena accessors (sequence.h:18-38, 55-61)
inline uint32_t ns_holes_num(const uint8_t *ns) { uint32_t v; __builtin_memcpy(&v, ns + 4, 4); return v; }
inline uint32_t ns_len(const uint8_t *ns) { uint32_t v; __builtin_memcpy(&v, ns + 8, 4); return v; }
inline const uint8_t *ns_pac(const uint8_t *ns) { return ns + 12 + 16 * (size_t)ns_holes_num(ns); }
inline Hole ns_hole(const uint8_t *ns, uint32_t i)
{
    Hole h; const uint8_t *p = ns + 12 + 16 * (size_t)i;
    __builtin_memcpy(&h.offset, p, 8); __builtin_memcpy(&h.len, p + 8, 4); h.amb = (char)p[12];
    return h;
}
inline size_t pac_byte_size(size_t x) { return x / 4 + (x % 4 != 0 ? 1 : 0); }
inline int pac_get(const uint8_t *pac, uint64_t i) { return pac[i >> 2] >> ((~i & 3) << 1) & 3; }
inline int nt4(unsigned char c)
{
    switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    case '-': return 5;
    default: return 4;
    }
}
// to_text rendering (sequence.cpp:71-81) and nt4 coding of a read (bwa.cpp:146 + mem_align1_core)
std::string ns_to_text(const uint8_t *ns);
void ns_to_nt4(const uint8_t *ns, std::vector<uint8_t> &out);

struct DeviceIndex;   // bsq_api.cpp

struct HoleRef { int64_t beg, end; uint32_t order; char amb; };

// The reference's hole overlay as disjoint, offset-ordered segments.  extract_reference_subseq writes the
// holes in their original order (bioseqdb/bwa.cpp:61-66), and holes of different rows share one axis
// (Q3), so they can overlap: the symbol left at p is that of the highest-order hole covering p.  Built
// once per index by a sweep over hole starts/ends with a max-heap on the order (expired holes dropped
// lazily); a window [rb, re) then costs one binary search plus the segments it overlaps, however many
// long holes lie under it.  `order` is the winning hole's index.
struct HoleIndex {
    std::vector<HoleRef> segs;
    explicit HoleIndex(const std::vector<Hole> &holes);
    // first segment with end > rb (segments are disjoint, so ends increase with begs)
    size_t first_after(int64_t rb) const
    {
        return (size_t)(std::upper_bound(segs.begin(), segs.end(), rb,
                                         [](int64_t v, const HoleRef &a) { return v < a.end; }) - segs.begin());
    }
};

struct HostIndex {
    std::vector<uint8_t> pac;    // pac_forward
    std::vector<Hole> holes;     // unshifted offsets (Q3)
    std::vector<Ann> anns;
    bool built = false;
    int64_t l_pac = 0;
    uint64_t seq_len = 0, primary = 0, L2[5] = {0, 0, 0, 0, 0};
    std::vector<OccBlock> occ;
    std::vector<uint32_t> sa32;  // full SA of T$ when seq_len < 2^32
    std::vector<uint64_t> sa64;
    DeviceIndex *dev = nullptr;
    // built on the device (bsq_index_build_device): SA and occ live only in HBM until bsq_index_download
    bool dev_built = false;
    int dev_wide = 0;
    uint64_t dev_nblk = 0;
    int dev_rounds = 0;        // prefix-doubling rounds after the first sort
    uint64_t dev_tied = 0;     // suffixes still tied after the first (21-character) sort

    void add_ref(int64_t id, const uint8_t *ns);
    int build(int threads, std::string &err);
    uint64_t sa(uint64_t row) const { return sa32.empty() ? sa64[row] : sa32[row]; }
    void occ4(uint64_t k, uint64_t c[4]) const;
};

}  // namespace bsq

// opaque C-ABI handles (include/bsq.h)
struct bsq_batch;
struct bsq_pipeline;
// the index plus one reusable pipeline of batches for the one-shot bsq_align_batch (its workspaces survive
// across calls; a concurrent caller that finds it busy uses a pipeline of its own)
struct bsq_index {
    bsq::HostIndex h;
    std::mutex pool_mu;
    bsq_pipeline *pipe = nullptr;
    // the reference holes as render segments in HBM (bsq_api.cpp index_render_holes), uploaded on first use
    std::mutex rh_mu;
    void *d_rh = nullptr;
    int64_t n_rh = -1;
    // offset-ordered holes for host rendering, built on first use after the index is built
    std::once_flag hx_once;
    std::unique_ptr<bsq::HoleIndex> hx;
    const bsq::HoleIndex &holes() { std::call_once(hx_once, [this] { hx.reset(new bsq::HoleIndex(h.holes)); }); return *hx; }
};
