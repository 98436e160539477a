// bsq_device.h -- data layouts shared by the host driver (bsq_api.cpp) and the HIP kernels
// (align_kernels.hip).  Everything here is plain-old-data so the same bytes are valid on both sides.
#pragma once
#include <stdint.h>

namespace bsq {

// One occurrence block of the $-removed BWT: 128 rows, 64 bytes.  cnt[c] = number of base c in
// rows before the block; the 128 bases are stored as two bit-planes (hi, lo) so a rank query is
// three 128-bit popcounts.  Same rank function as libbwa's bwt_occ4 (bwt.c), different bits.
struct alignas(64) OccBlock {
    uint64_t cnt[4];
    uint64_t hi[2];
    uint64_t lo[2];
};
static_assert(sizeof(OccBlock) == 64, "occ block must be one 64-byte sector");

// Half-size rank block for texts with < 2^32 rows: u32 counts before the block + the two bit-planes
// of 64 bases, 32 bytes.  Same 0.5 B/base as OccBlock, but a rank query popcounts one 64-bit word per
// plane instead of two.  Derived from OccBlock at upload (bsq_api.cpp) and used by the seeding kernels.
struct alignas(32) OccBlock32 {
    uint32_t cnt[4];
    uint64_t hi, lo;
};
static_assert(sizeof(OccBlock32) == 32, "occ32 block must be 32 bytes");

// 64-bit rows (texts of >= 2^32 rows, the 3 Gbp configs) use the same 32-B blocks with counts relative to
// their superblock of 2^16 blocks (2^22 rows, so a relative count fits u32).  The superblocks' absolute counts
// follow the blocks in the same table: cnt[c] = rows of base c before the superblock, gt[c] = rows of the bases
// > c before it (the two sums bwt_extend needs per base).  1,431 superblocks (92 KB, cache-resident) at 3 Gbp.
constexpr int SUP_SHIFT = 16;   // log2(64-base blocks per superblock)
struct alignas(64) SupBlock {
    uint64_t cnt[4], gt[4];
};
static_assert(sizeof(SupBlock) == 64, "superblock must be 64 bytes");
inline uint64_t occ32_sup_count(uint64_t nblk32) { return (nblk32 >> SUP_SHIFT) + 1; }

// Per-read interval slots (cap entries each) are laid out by wave of 64 reads: entry k of read li sits at
// [((li / 64) * cap + k) * 64 + li % 64], so the lanes of a wave (one read each, in every kernel that
// touches the slots) access the same entry index at adjacent addresses.  Workspaces hold whole waves.
inline int64_t intv_slot_at(int64_t li, int64_t k, int64_t cap) { return ((li >> 6) * cap + k) * 64 + (li & 63); }
inline int64_t intv_slot_reads(int64_t n) { return (n + 63) / 64 * 64; }

#ifdef __HIP__
// A lane's array interleaved with the other lanes of its wave: element i at p[i * S] (S = 64); S = 1 is the
// contiguous per-thread layout (the retry kernels, which run a handful of reads per launch).
template <typename T, int S = 64> struct SP {
    T *p;
    __host__ __device__ T &operator[](int i) const { return p[(size_t)i * S]; }
    __host__ __device__ SP operator+(int i) const { return SP{p + (size_t)i * S}; }
};
__device__ inline int64_t intv_slot_at_d(int64_t li, int64_t k, int64_t cap) { return ((li >> 6) * cap + k) * 64 + (li & 63); }
#endif

// Device view of the index (passed by value as a kernel argument).
struct DIndex {
    const OccBlock *occ;
    const uint32_t *sa32;     // full suffix array of T$ (rows 0..seq_len) when seq_len < 2^32
    const uint64_t *sa64;     // otherwise
    const uint8_t *pac;       // forward pac, 4 bases per byte, MSB first (sequence.h:55)
    const int64_t *ann_off;   // bntann1_t.offset per reference row
    const int32_t *ann_len;   // bntann1_t.len
    int32_t n_anns;
    int32_t kmer_k;           // k-mer interval table depth (0 = none)
    uint64_t L2[5];
    uint64_t primary, seq_len;
    int64_t l_pac;
    // k-mer interval table: for every string S over ACGT with 1 <= |S| <= kmer_k, the bidirectional
    // interval (x[0], x[1], x[2], 0) that bwt_extend chains produce for S (u32 rows only), at entry
    // (4^|S| - 4)/3 + code(S), code = base-4 value of S with the first base most significant
    const uint32_t *kmer;
    const OccBlock32 *occ32;  // 64-base rank blocks (absolute counts for u32 rows, superblock-relative otherwise)
    const SupBlock *sup;      // 64-bit rows: superblock counts (after the blocks in the occ32 table); else nullptr
    int32_t wide;             // 1: 64-bit rows (seq_len >= 2^32, or forced by BSQ_FORCE_WIDE)
    int32_t pad2;
};

// mem_opt_t fields the path reads (mem_opt_init defaults + bioseqdb overrides).
struct DOpts {
    int32_t a, b, o_del, e_del, o_ins, e_ins, pen_clip5, pen_clip3, w, zdrop;
    int32_t min_seed_len, max_occ, split_width, max_chain_gap, min_chain_weight, max_chain_extend, max_mem_intv;
    float split_factor, mask_level, drop_ratio, mask_level_redun;
    int32_t mat_match, mat_mismatch, mat_amb, mat_max;   // the 5x5 matrix from bwa_fill_scmat (Q2)
};

// Per-batch capacities (the main pass uses small ones; overflowing reads are re-run with large ones).
struct Caps {
    int32_t max_len;     // longest read in the batch
    int32_t intv;        // SMEM intervals per read
    int32_t seeds;       // seeds per read after SA expansion
    int32_t chains;      // chains per read
    int32_t regs;        // alignment regions per read
    int32_t cigar;       // CIGAR ops per region
    int64_t scratch;     // bytes of private scratch per worker thread
    int64_t scr_ext;     // k_extend's stride in that scratch (<= scratch): its own arrays only, so the
                         // extension's lanes sit closer together than the widest stage's stride puts them
};

struct Intv { uint64_t x[3]; uint64_t info; };
struct Seed { int64_t rbeg; int32_t qbeg, len; };
struct ChainDesc { int32_t seed_off, n, rid, w; };

struct Reg {
    int64_t rb, re;
    int32_t qb, qe, rid, score, truesc, sub, csub, sub_n, w, seedcov, secondary, seedlen0, n_comp, pad;
    uint64_t hash;
};

struct Hit {            // one region after mem_reg2aln
    int64_t rb, re;
    int32_t qb, qe, rid, score, flag, is_rev, n_cigar, pad;
};

// status bits per read
enum : uint32_t { ST_OVERFLOW = 1u, ST_UNSUPPORTED = 2u };

enum Stage { STG_SMEM = 0, STG_CHAIN, STG_EXTEND, STG_REG2ALN, STG_PACK, STG_D2H, STG_N };

// device-side algorithmic byte counters, one slot per stage
struct Counters {
    unsigned long long occ_blocks;   // occ block fetches in bwt_extend, in 32-B units (a 64-B OccBlock counts 2)
    unsigned long long sa_values;    // SA values produced
    unsigned long long ref_bases;    // reference bases fetched for extension / CIGAR
    unsigned long long dp_cells;     // DP cells evaluated (secondary figure)
    unsigned long long overflow;     // reads flagged for the retry pass
    unsigned long long kmer_hits;    // 16-B k-mer interval table reads (in place of a bwt_extend)
    unsigned long long sort_guard;   // introsort partition scans stopped by the i < t bound, not the sentinel (must be 0)
    unsigned long long pad;
};

}  // namespace bsq
