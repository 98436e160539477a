// bsq_internal.h -- library-internal C++ interface between bsq_api.cpp (batches) and the host drivers built on
// top of them (pipeline.cpp, group.cpp).  Not part of the C-ABI (include/bsq.h).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/bsq.h"

namespace bsq {

// The host half of bsq_batch_set_nuclseqs: a cursor fetch's nuclseq varlenas validated and packed (8-byte
// aligned, as they are) into pinned host memory, with the offsets the device decode pass needs.  Once staged,
// the caller's varlenas may be released (the SPI tuple table of the fetch); the device half
// (batch_upload_staged) runs later, on any thread.
struct NsStage {
    int32_t n = 0;
    int max_len = 0;
    int64_t bases = 0;
    std::vector<int64_t> meta;    // in_off[n+1] | poff[n+1] | indices of the reads with holes
    std::vector<int64_t> offs;    // base offsets [n+1]
    uint8_t *host = nullptr;      // packed varlenas (pinned)
    int64_t host_cap = 0, host_bytes = 0;
    int64_t meta_at = 0, offs_at = 0;   // pinned copies of meta and offs at host + meta_at / host + offs_at
    NsStage() = default;
    NsStage(const NsStage &) = delete;
    NsStage &operator=(const NsStage &) = delete;
    ~NsStage();
};

// Validates and packs n reads (errors: BSQ_E_INVALID / BSQ_E_NOMEM with the thread's message set).
int stage_nuclseqs(NsStage &s, const void *const *reads, int32_t n);
// H2D of a staged fetch into batch b, nt4 conversion on the device, and (with_workspace) workspace sizing;
// synchronous.
int batch_upload_staged(bsq_batch *b, const NsStage &s, bool with_workspace);
// A batch's device workspaces as a unit (pipeline.cpp lends run_cap sets to the batches whose alignment turn it is):
// detach (after syncing the batch's stream; an empty set when the batch holds none), attach (frees what the batch
// held), free; batch_prepare_workspace sizes the attached set for the uploaded reads.
struct WsSet;
WsSet *batch_detach_workspaces(bsq_batch *b);
void batch_attach_workspaces(bsq_batch *b, WsSet *w);
bool batch_has_workspace(const bsq_batch *b);
void workspaces_free(WsSet *w);
int batch_prepare_workspace(bsq_batch *b);
int32_t batch_max_reads(const bsq_batch *b);
int64_t batch_max_bases(const bsq_batch *b);

void set_error(const std::string &msg);

// Where the last bsq_batch_run's records are (exchange.cpp's send side): on the device when the packed arrays hold
// the whole view (one workspace chunk, no retried read: off = batch-wide read offsets, hits, cig in HBM), else
// the pinned host view.  `stream` is the batch's stream (the next run on it overwrites these arrays).
struct BatchRecords {
    int device = 0;
    void *stream = nullptr;   // hipStream_t
    bool on_device = false;
    const int64_t *off = nullptr;
    const bsq_hit *hits = nullptr;
    const uint32_t *cig = nullptr;
    int32_t n_reads = 0;
    int64_t n_hits = 0, n_cigar = 0;
};
BatchRecords batch_records(const bsq_batch *b);

// The exchange's wire form of one lane-round's records (bsq_xchg, exchange.cpp).  A bsq_hit is 72 B; on the wire a hit
// is 32 B: ref_id and the three ref_match_* fields follow from rid, rb and the length through the index's anns
// (bsq_api k_pack), re = rb + len, read_index from the read's position and cigar_off from the prefix of n_cigar over
// the hits (the batch-wide arrays k_pack fills: read_index = read_base + i, cigar_off = cig_base + that prefix).
// The read offsets travel as one int32 hit count per read after a 16-B header {read_base, cig_base}.  CIGAR words
// travel as they are.  Rank 0 takes the compact form over its PCIe link and expands it on the host.
struct WireHit {
    int64_t rb;
    int32_t len, qb, qe, score, rid;
    uint32_t ncig;   // n_cigar | is_primary << 29 | is_secondary << 30 | is_reverse << 31
};
static_assert(sizeof(WireHit) == 32, "wire hit layout");
constexpr int64_t kWireHead = 16;   // {int64 read_base, int64 cig_base} before the int32 counts
inline int64_t wire_off_bytes(int64_t n_reads) { return kWireHead + 4 * n_reads; }
// device: the wire form of n_reads reads' records (off: n_reads + 1 batch offsets, hits) into off_part (header +
// counts) and wire (n_hits); on stream `st` (hipStream_t)
int launch_wire_pack(void *st, int32_t n_reads, const int64_t *off, const bsq_hit *hits, uint8_t *off_part, WireHit *wire);
// host: the records back, byte for byte as the sender's k_pack wrote them (padding zeroed); ann_off/ann_id of the index
void wire_expand(const uint8_t *off_part, const WireHit *wire, int32_t n_reads, const int64_t *ann_off,
                 const int64_t *ann_id, int64_t n_anns, int64_t *read_off, bsq_hit *hits);
// bsq_batch_render_nuclseqs into the batch's own pinned buffers: *out / *out_off are borrowed until the next
// render or run of the batch (the pipeline hands them out until the slot is released).
int batch_render_cols(bsq_batch *b, const void *const *reads, const uint8_t **out, const int64_t **out_off);

// pipeline.cpp: how a submission's reads reach the slot.  COPY: staged on the caller's thread before submit
// returns (the public bsq_pipeline_submit).  DEFER: staged by the slot's worker (the reads must stay valid
// until the submission is taken; lets a caller that holds all reads stage several slots in parallel).  RERUN:
// the slot's previous staging again (the reads stay on the device: a benchmark's re-run of the same fetch).
enum class PipeMode { COPY, DEFER, RERUN };
int pipeline_submit_ex(bsq_pipeline *p, const bsq_opts *opts, const void *const *reads, int32_t n_reads,
                       uint64_t first_call_seq, int nuclseq_columns, PipeMode mode);
// With nothing outstanding, the next submission goes to slot 0 again (a caller that submits shares j = 0..s-1 per
// round keeps share j on slot j, where a RERUN finds its staging).  BSQ_E_INVALID while submissions are pending.
int pipeline_rewind(bsq_pipeline *p);
// every DEFER submission numbered < upto has stopped reading its caller's varlenas
int pipeline_wait_staged(bsq_pipeline *p, int64_t upto);
// Record route of every batch of the pipeline (bsq_batch_set_record_route; -1: each batch's own device link).
// BSQ_E_INVALID while submissions are pending.
int pipeline_set_record_route(bsq_pipeline *p, int via_device);
// bsq_pipeline_next plus the batch that holds the taken submission's records (NULL for an empty one)
int pipeline_next_ex(bsq_pipeline *p, const bsq_hits **view, const uint8_t **cols, const int64_t **col_off,
                     bsq_batch **batch);

}  // namespace bsq
