/*
 * bsq.h -- C-ABI of libbsq, the MI355X-native BWA-MEM alignment path behind bioseqdb's
 * nuclseq_search_bwa / nuclseq_multi_search_bwa.
 *
 * Every entry point is plain C (pointers, sizes, status codes; no C++ types, exceptions or
 * longjmp cross it).  Each one replaces a piece of the reference's in-process seam
 * (bioseqdb/bwa.h:32-48 `class BwaIndex` over libbwa):
 *
 *   bsq_index_create / bsq_index_free  <- BwaIndex::BwaIndex / ~BwaIndex        (bwa.cpp:80, 131-139)
 *   bsq_index_add_ref                  <- BwaIndex::add_ref_sequence            (bwa.cpp:82-105)
 *   bsq_index_build                    <- BwaIndex::build                       (bwa.cpp:107-128)
 *                                         = pac2bwt + is_bwt + bwt_bwtupdate_core + bwt_cal_sa
 *   bsq_index_upload                   <- (new) copies BWT/occ, SA and pac into HBM once
 *   bsq_align_batch                    <- BwaIndex::align_sequence per read     (bwa.cpp:141-181)
 *                                         = mem_align1 + mem_reg2aln for a whole cursor batch
 *   bsq_render_tsv                     <- the BwaMatch rendering of align_sequence
 *                                         (extract_reference_subseq, cigar_compressed_to_string)
 *   bsq_opts                           <- the mem_opt_t fields set by bwa_index_from_query
 *                                         (extension.cpp:211-236; effective values incl. Q1)
 *
 * Status codes: BSQ_OK (0) or a negative BSQ_E_*; bsq_last_error() gives a thread-local message.
 * Ownership: inputs are borrowed for the duration of the call; outputs are allocated by libbsq and
 * released with the matching *_free.  An index is immutable after bsq_index_upload; concurrent
 * bsq_align_* calls on one index from different host threads are safe (each batch has its own
 * stream and workspace).
 */
#ifndef BSQ_H
#define BSQ_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BSQ_OK 0
#define BSQ_E_INVALID (-1)   /* bad argument / state */
#define BSQ_E_NOMEM (-2)     /* host or device allocation failed */
#define BSQ_E_HIP (-3)       /* HIP runtime error */
#define BSQ_E_NODEV (-4)     /* no usable gfx950 device */
#define BSQ_E_UNSUPPORTED (-5) /* input outside what the path implements (a read beyond even the retry capacities) */

/* Effective BWA-MEM options (mem_opt_t fields bioseqdb writes, extension.cpp:220-231).  The SQL
 * bwa_opts() field-order quirk (Q1) is applied by the caller: defaults are
 * {19, max(500, 2*n_refs), 1, 4, 5, 5, 100, 100, o_del=6, e_del=6, o_ins=1, e_ins=1}. */
typedef struct {
    int32_t min_seed_len, max_occ, a, b, pen_clip3, pen_clip5, zdrop, w, o_del, e_del, o_ins, e_ins;
} bsq_opts;

typedef struct bsq_index bsq_index;
typedef struct bsq_batch bsq_batch;

/* One alignment region = one bwa_result row (bioseqdb--0.0.0.sql:196-212).  Coordinates are the
 * reference's: rb/re in the forward+reverse space [0, 2*l_pac) (Q6). */
typedef struct {
    int64_t ref_id;            /* anns[rid].name reinterpreted as int64 (bwa.cpp:160) */
    int64_t rb, re;            /* mem_alnreg_t rb/re */
    int32_t ref_match_start;   /* (int32)(rb - anns[rid].offset)  */
    int32_t ref_match_end;     /* (int32)(re - anns[rid].offset)  */
    int32_t ref_match_len;     /* (int32)(re - rb)                */
    int32_t qb, qe;            /* query_match_start / _end        */
    int32_t score;             /* mem_aln_t.score = mem_alnreg_t.score (Q9) */
    int32_t rid;
    uint8_t is_primary, is_secondary, is_reverse, pad0;
    int32_t read_index;        /* index of the read within the batch */
    uint32_t cigar_off, n_cigar; /* into bsq_hits.cigar: u32 len<<4 | op, ops 0..4 = M,I,D,S(clip=3),H */
} bsq_hit;

typedef struct {
    int32_t n_reads;
    int64_t n_hits;
    bsq_hit *hits;             /* read order, then libbwa's final region order (Q16) */
    int64_t *read_off;         /* n_reads+1: hits of read i are [read_off[i], read_off[i+1]) */
    int64_t n_cigar;
    uint32_t *cigar;
} bsq_hits;

const char *bsq_last_error(void);
const char *bsq_version(void);
/* Number of HIP devices visible (0 without a GPU; never initialises a device context). */
int bsq_device_count(void);

/* ---- nuclseq codec (the type's text I/O; reference: nuclseq_from_text sequence.cpp:209-245 with
 * std::minstd_rand(holes_num ^ len) fill of hole and padding bases, and to_text_palloc :71-81) ---- */
/* Encodes len characters (nst_nt4 ACGT -> 2-bit, anything else -> run-length hole) into a malloc'd
 * NucleotideSequence varlena; size in *out_size.  No validation of the alphabet (nuclseq_in does it). */
void *bsq_nuclseq_from_text(const char *text, size_t len, size_t *out_size);
/* Renders a NucleotideSequence varlena as text (malloc'd, NUL-terminated). */
char *bsq_nuclseq_to_text(const void *nuclseq);

/* ---- bulk codec and loader ---- */
/* nuclseq_in for a whole batch on `device` (extension.cpp:46-61 + nuclseq_from_text, sequence.cpp:209-245):
 * text i is text[offs[i] - offs[0] .. offs[i+1] - offs[0]).  On success *out holds the n varlenas, varlena i
 * at (*out_off)[i] (8-byte aligned; (*out_off)[n] = total bytes), byte-identical to bsq_nuclseq_from_text.
 * A text longer than INT32_MAX/4 fails with "provided sequence is too long"; with validate != 0 a character
 * outside ACGTNWSMKRYBDHV fails with "invalid nucleotide in nuclseq_in: '<c>'" -- the first failure in
 * text order, as a cursor of nuclseq_in calls would raise it (BSQ_E_INVALID).  Both outputs are malloc'd
 * (bsq_free).  No device: BSQ_E_NODEV (no CPU fallback). */
int bsq_nuclseq_encode_batch(int device, const char *text, const int64_t *offs, int64_t n, int validate,
                             uint8_t **out, int64_t **out_off);
/* nuclseq_out for a whole batch (to_text_palloc, sequence.cpp:71-81,162-166): text i at
 * (*text)[(*text_off)[i] .. (*text_off)[i+1]), *text NUL-terminated; both malloc'd (bsq_free). */
int bsq_nuclseq_decode_batch(int device, const void *const *nuclseqs, int64_t n, char **text, int64_t **text_off);
/* Device time of the last encode/decode call on this thread (kernels only) and the whole call's wall time. */
int bsq_nuclseq_codec_ms(double *kernel_ms, double *call_ms);
/* The FASTA reading of bioseqdb-import (bioseqdb-import/main.cpp:48-71): records split at '>' lines, sequence
 * lines upper-cased and concatenated, empty records dropped.  Record i: sequence (*seq)[(*seq_off)[i] ..
 * (*seq_off)[i+1]), name (*names)[(*name_off)[i] .. (*name_off)[i+1]).  All four outputs malloc'd. */
int bsq_fasta_parse(const char *data, int64_t size, char **seq, int64_t **seq_off, char **names, int64_t **name_off,
                    int64_t *n_records);

/* ---- index ----------------------------------------------------------------------------------- */
int bsq_index_create(bsq_index **out);
void bsq_index_free(bsq_index *idx);
/* `nuclseq` points at a detoasted NucleotideSequence varlena (sequence.h:18-38):
 * {vl_len[4], holes_num u32, len u32, holes_num x bntamb1_t(16 B), ceil(len/4) pac bytes}. */
int bsq_index_add_ref(bsq_index *idx, int64_t id, const void *nuclseq);
/* Host build of T = pac || revcomp(pac), its suffix array, BWT, occ blocks.  `threads` <= 0: all cores. */
int bsq_index_build(bsq_index *idx, int threads);
/* Copies the built index into HBM of `device`.  No-op for an index built on that device. */
int bsq_index_upload(bsq_index *idx, int device);
/* GPU build (replaces BwaIndex::build, bioseqdb/bwa.cpp:107-128, and the
 * host bsq_index_build + bsq_index_upload pair): suffix array of T$ by prefix doubling on rocPRIM radix
 * sorts, BWT and occurrence blocks, all in HBM of `device`; the result is identical to the host build.
 * Leaves the index uploaded; its SA and occ blocks stay on the device until bsq_index_download. */
int bsq_index_build_device(bsq_index *idx, int device);
/* Copies the SA and occ blocks of a device-built index to the host (bsq_index_sa / _occ4 / _sa_data). */
int bsq_index_download(bsq_index *idx);
/* Prefix-doubling rounds of the last device build and the suffixes still tied after its first sort. */
int bsq_index_build_stats(const bsq_index *idx, int *rounds, uint64_t *tied);
/* Certificate of the suffix array in HBM (either build): every value in range, every position once, adjacent
 * suffixes of T$ strictly increasing.  *violations == 0 proves it is the unique SA that libbwa's bwt_cal_sa
 * samples (bioseqdb/bwa.cpp:107-128), so the BWT and occ derived from it are libbwa's.  *suffixes = seq_len+1. */
int bsq_index_certify_sa(const bsq_index *idx, uint64_t *suffixes, uint64_t *violations);
int64_t bsq_index_l_pac(const bsq_index *idx);
int64_t bsq_index_seq_len(const bsq_index *idx);
int64_t bsq_index_primary(const bsq_index *idx);
int32_t bsq_index_n_refs(const bsq_index *idx);
/* 1 when both indexes were given the same reference rows (ids, lengths, packed bases and holes, in order; built
 * or not), else 0 (-1 for a NULL argument).  A backend's index cache confirms a digest hit with it. */
int bsq_index_same_refs(const bsq_index *a, const bsq_index *b);
/* Host copies of the logical FM quantities for tests (valid after build, no GPU needed):
 * sa[row] for row in [0, seq_len] and occ4 per row. */
int64_t bsq_index_sa(const bsq_index *idx, int64_t row);
int bsq_index_occ4(const bsq_index *idx, int64_t k, uint64_t cnt[4]);
/* Export the full suffix array (seq_len+1 entries of `*elem_bytes` = 4 or 8 bytes); borrowed. */
const void *bsq_index_sa_data(const bsq_index *idx, int *elem_bytes);

/* ---- Index replication (one process per GPU, the index built once and broadcast
 * over xGMI).  The device tables are plain byte buffers, so any collective can move them: the root builds,
 * uploads into caller-owned buffers and the caller broadcasts those buffers and the metadata blob; the
 * other ranks import.  Replaces BwaIndex::build per process (bioseqdb/bwa.cpp:107-128). ---- */
#define BSQ_N_TABLES 8   /* occ, occ32, sa, pac, ann_off, ann_id, ann_len, kmer (0 bytes = absent) */
typedef struct { void *ptr; uint64_t bytes; } bsq_table;
/* Bytes of each device table of a built index, and its metadata blob (meta == NULL: size query into
 * *meta_bytes). */
int bsq_index_layout(const bsq_index *idx, uint64_t *bytes, void *meta, uint64_t *meta_bytes);
/* Like bsq_index_upload, into caller-owned device buffers (tables[i].bytes >= layout bytes[i]); the caller
 * keeps them alive while the index is used. */
int bsq_index_upload_into(bsq_index *idx, int device, const bsq_table *tables, int n_tables);
/* A device-only index over caller-owned tables that hold an uploaded index's contents (e.g. received by a
 * broadcast), described by its metadata blob.  Aligns and renders like the original. */
int bsq_index_import(const void *meta, uint64_t meta_bytes, int device, const bsq_table *tables, int n_tables,
                     bsq_index **out);
/* Borrowed device pointers and sizes of an uploaded (or device-built) index's tables and its device: the
 * source buffers of a broadcast. */
int bsq_index_device_tables(const bsq_index *idx, int *device, bsq_table *tables, int n_tables);

/* ---- One process driving several devices (the Postgres backend is a single
 * process, so `bsq_index_upload(idx, devices[], n)` becomes a group).  Replaces the per-read loop of
 * nuclseq_multi_search_bwa (extension.cpp:362-370) spread over n GPUs. ---- */
typedef struct bsq_group bsq_group;
/* One RCCL communicator per device (ncclCommInitAll over xGMI) and one host worker per member.  A device
 * listed twice makes a group of replicas on one GPU: valid (tests use it), replication then copies device to
 * device instead of using RCCL. */
int bsq_group_create(const int *devices, int n_devices, bsq_group **out);
void bsq_group_free(bsq_group *g);
int bsq_group_size(const bsq_group *g);
/* Puts a built index on every member: uploaded to (or built on) the first member's device if it is not there
 * yet, then every device table broadcast from it (ncclBroadcast inside one ncclGroupStart/End) and imported on
 * the others.  The group keeps the replicas until the next replicate or free; `idx` must outlive the group's
 * use of it (member 0 aligns on it).  *broadcast_ms: wall time of the broadcast (NULL: not reported). */
int bsq_group_replicate(bsq_group *g, bsq_index *idx, double *broadcast_ms);
/* Aligns n_reads nuclseq reads over the members: member k takes reads [k*n/G, (k+1)*n/G) with lrand48
 * positions from first_call_seq + its first read (identical rows to one device aligning all reads in
 * order, Q10/Q16).  Every member runs on its own host thread and copies its records to the host over its
 * own PCIe link (pinned memory, one segment per share); the merged view (read order, call-wide read_index and
 * cigar_off) is borrowed until the next run or free.  With reads == NULL the members re-run the reads staged
 * (and still resident on their devices) from the previous call. */
int bsq_group_run(bsq_group *g, const bsq_opts *opts, const void *const *reads, int32_t n_reads,
                  uint64_t first_call_seq);
/* Concurrent shares per member (1..16, default 4): each member splits its shard into up to this many batches
 * of >= 32768 reads that run at once on its device (a bsq_pipeline).  Set before bsq_group_replicate. */
int bsq_group_set_slots(bsq_group *g, int slots);
/* bsq_group_run `rounds` times over the reads staged by the previous bsq_group_run (n_reads as given there), with
 * no barrier between rounds: each member's shares run bsq_batch_run_rounds on the batches that hold them (share j
 * starts its next round as soon as its previous one ends), the schedule of the one-device bench.  Every round
 * aligns every read from first_call_seq; the last round's records are the result (segments / merged view as after
 * bsq_group_run). */
int bsq_group_run_rounds(bsq_group *g, const bsq_opts *opts, int32_t n_reads, uint64_t first_call_seq, int rounds);
/* How the members' records reach host memory (the exchange step of a sharded call):
 * BSQ_XCHG_LINKS     each member's records over its own PCIe link (default; all links at once);
 * BSQ_XCHG_VIA_FIRST each member's records by peer DMA over xGMI into member 0's HBM, then over member 0's link
 *                    (the records gathered on one device first).  Set between runs. */
#define BSQ_XCHG_LINKS 0
#define BSQ_XCHG_VIA_FIRST 1
int bsq_group_set_exchange(bsq_group *g, int mode);
/* The merged view of the last run (built on first call after a run; NULL on allocation failure). */
const bsq_hits *bsq_group_hits(const bsq_group *g);
/* The last run's records without the merge: segment i (one per member share, in read order) covers reads
 * [read_lo[i], read_lo[i] + views[i]->n_reads) with segment-local read_index / cigar_off.  Writes up to `max`
 * entries and returns the number of segments.  Borrowed until the next run or free. */
int bsq_group_segments(const bsq_group *g, const bsq_hits **views, int32_t *read_lo, int max);
/* build_tuple_bwa's two nuclseq columns of the last run's rows, rendered on every member for its shard
 * (layout as bsq_batch_render_nuclseqs, rows in the merged order).  `reads` as given to bsq_group_run. */
int bsq_group_render_nuclseqs(bsq_group *g, const void *const *reads, uint8_t **out, int64_t **out_off);

/* ---- One process per GPU (torchrun): the record exchange to rank 0 ----
 * Every rank's hit records return to the caller (rank 0), the rows nuclseq_multi_search_bwa puts into its
 * tuplestore (extension.cpp:362-370).  Batch i of a rank is lane i.  After each round of each lane, ONE exchange
 * thread per rank -- in the same (round, lane) order on every rank, on one RCCL communicator and one stream, so
 * operations match one-to-one and cannot deadlock -- all-gathers the ranks' record counts and batch status, then
 * every rank r > 0 sends its read offsets, hits and CIGAR words to rank 0 (ncclSend/ncclRecv over xGMI) and rank 0
 * copies them to pinned host memory.  A batch failure on any rank stops every rank at that same (round, lane);
 * a peer silent for BSQ_XCHG_TIMEOUT_S seconds (default 600) aborts the communicator instead of hanging. */
typedef struct bsq_xchg bsq_xchg;
#define BSQ_XCHG_ID_BYTES 128
/* A fresh communicator id (BSQ_XCHG_ID_BYTES bytes) -- rank 0 makes it and the launcher's own channel
 * (torch.distributed) hands it to every rank. */
int bsq_xchg_unique_id(void *id);
/* Joins the communicator `id` (BSQ_XCHG_ID_BYTES, the same on every rank) with `lanes` lanes on `device`; collective. */
int bsq_xchg_create(int world, int rank, int device, const void *id, int lanes, bsq_xchg **out);
void bsq_xchg_free(bsq_xchg *x);
/* bsq_batch_run_rounds with lane i exchanging batch i's records after every round (n == lanes on every rank);
 * x == NULL: bsq_batch_run_rounds.  After a failure (any rank's) the exchange is aborted and later calls fail. */
int bsq_batch_run_rounds_x(bsq_batch *const *batches, int n, const bsq_opts *opts, const uint64_t *first_call,
                           int rounds, bsq_xchg *x);
/* Waits for every lane's last exchange (rank 0: the records are in its host memory).  *bytes_moved: bytes
 * received (rank 0) or sent (others) over all rounds; *wait_ms: host time the batch threads spent exchanging. */
int bsq_xchg_finish(bsq_xchg *x, int64_t *bytes_moved, double *wait_ms);
/* Rank 0: the last round's records of lane `lane` from rank src_rank > 0 (read_index and cigar_off local to that
 * rank's batch), borrowed until the next round or free.  They travel in a compact wire form (32 B per hit and 4 B
 * per read instead of 72 + 8: ref_id, re, ref_match_*, read_index and cigar_off are implied) and are expanded here,
 * byte for byte what the sender's batch holds, with the anns of the index given to bsq_xchg_set_index. */
int bsq_xchg_view(const bsq_xchg *x, int lane, int src_rank, bsq_hits *out);
/* Rank 0: the index (the one every rank aligns against) whose anns expand the received records. */
int bsq_xchg_set_index(bsq_xchg *x, const bsq_index *idx);
/* One GPU: the batch's last records through the exchange's wire form and back (the send path's device pack, the
 * view's host expansion), compared byte for byte with the batch's view (*mismatches: differing read offsets and
 * records).  *wire_bytes / *raw_bytes: the round's bytes on the link in the wire form / as bsq_hit + int64 offsets. */
int bsq_xchg_wire_check(bsq_batch *b, const bsq_index *idx, int64_t *wire_bytes, int64_t *raw_bytes, int64_t *mismatches);

/* ---- Pipelined cursor fetches (replaces the fetch-align-materialise loop of
 * nuclseq_multi_search_bwa, extension.cpp:156-195 + 362-370, which leaves the device idle between fetches).
 * A pipeline owns n_slots batches on the index's device, each with its own HIP stream and host worker.
 * bsq_pipeline_submit copies the fetch's nuclseq varlenas (they may be released when it returns) and starts
 * upload, alignment, the record D2H and, with nuclseq_columns != 0, build_tuple_bwa's two nuclseq columns
 * per row (as bsq_batch_render_nuclseqs) on the next slot; read i draws lrand48 value first_call_seq + i.
 * bsq_pipeline_next waits for the oldest submission not yet taken and lends its rows (and columns, NULL when
 * not asked for or no rows) until bsq_pipeline_release, which frees the oldest taken slot.  At most n_slots
 * submissions may be submitted and not released: a further submit fails with BSQ_E_INVALID.  A failed
 * submission reports its error from bsq_pipeline_next and frees its slot. */
typedef struct bsq_pipeline bsq_pipeline;
int bsq_pipeline_create(bsq_index *idx, int n_slots, bsq_pipeline **out);
void bsq_pipeline_free(bsq_pipeline *p);
int bsq_pipeline_slots(const bsq_pipeline *p);
int bsq_pipeline_submit(bsq_pipeline *p, const bsq_opts *opts, const void *const *reads, int32_t n_reads,
                        uint64_t first_call_seq, int nuclseq_columns);
/* As bsq_pipeline_submit, but the fetch is staged by the slot's worker thread instead of the caller's: `reads` and
 * the varlenas they point to must stay valid until bsq_pipeline_wait_staged(p, k) returns for some k > *job (the
 * submission's number, counted from the pipeline's creation).  A backend frees fetch k's tuples after fetching k+1
 * and waiting for k's staging, so the staging overlaps its own SPI work (extension.cpp:156-195's fetch loop). */
int bsq_pipeline_submit_deferred(bsq_pipeline *p, const bsq_opts *opts, const void *const *reads, int32_t n_reads,
                                 uint64_t first_call_seq, int nuclseq_columns, int64_t *job);
/* Returns once no deferred submission numbered < upto still reads its caller's varlenas. */
int bsq_pipeline_wait_staged(bsq_pipeline *p, int64_t upto);
int bsq_pipeline_next(bsq_pipeline *p, const bsq_hits **view, const uint8_t **cols, const int64_t **col_off);
int bsq_pipeline_release(bsq_pipeline *p);

/* ---- alignment --------------------------------------------------------------------------------- */
/* Value of the (pos+1)-th lrand48() call of an unseeded glibc/musl process (Q10). */
int64_t bsq_lrand48_at(uint64_t pos);

/* Align n_reads nuclseq reads (each a NucleotideSequence varlena pointer).  Read i uses the
 * lrand48 value of call number first_call_seq + i (mem_align1's mem_mark_primary_se id).
 * On success *out holds every region of every read. */
int bsq_align_batch(bsq_index *idx, const bsq_opts *opts, const void *const *reads, int32_t n_reads,
                    uint64_t first_call_seq, bsq_hits **out);
void bsq_hits_free(bsq_hits *hits);
/* Frees the batches and workspaces bsq_align_batch keeps with the index between calls (a backend done with a
 * large cursor gives the device memory back; the next call re-creates them).  BSQ_E_INVALID while in use. */
int bsq_index_release_pool(bsq_index *idx);

/* Renders hits as bwa_result rows (TSV, one line per hit, columns as bioseqdb--0.0.0.sql:196-212
 * without query_id): ref_id ref_subseq ref_match_start ref_match_end ref_match_len query_subseq
 * query_match_start query_match_end query_match_len is_primary is_secondary is_reverse cigar score.
 * ref_subseq on reverse-strand rows, where the reference reads out of bounds (Q7), is rendered
 * as the reverse-strand reference text.  Returns a malloc'd string (free with bsq_free). */
char *bsq_render_tsv(const bsq_index *idx, const bsq_hits *hits, const void *const *reads);
/* ref_subseq of one row (extract_reference_subseq, bioseqdb/bwa.cpp:55-68, Q3 hole overlay; reverse-strand
 * text where the reference reads out of bounds, Q7): writes re - rb characters (no NUL) to out and returns
 * that count; out == NULL: returns the count only.  -1 for an unbuilt index or a range outside [0, 2*l_pac). */
int64_t bsq_index_ref_subseq(const bsq_index *idx, int64_t rb, int64_t re, char *out);
void bsq_free(void *p);

/* ---- device-resident batches (bench / multi-GPU drivers) --------------------------------------- */
/* A batch owns a HIP stream and a device workspace for up to max_reads reads / max_bases bases. */
int bsq_batch_create(bsq_index *idx, int32_t max_reads, int64_t max_bases, bsq_batch **out);
void bsq_batch_free(bsq_batch *b);
/* Stage reads given as nt4 codes (0..3 = ACGT, 4 = other), offsets[n+1] (host arrays) into HBM. */
int bsq_batch_set_reads(bsq_batch *b, const uint8_t *codes, const int64_t *offsets, int32_t n_reads);
/* Stage reads given as nuclseq varlenas (the cursor's detoasted values): uploaded as they are and turned
 * into nt4 codes on the device.  bsq_align_batch uses this path. */
int bsq_batch_set_nuclseqs(bsq_batch *b, const void *const *reads, int32_t n_reads);
/* Run the whole alignment pipeline on the staged reads and copy the packed hits to the host. */
int bsq_batch_run(bsq_batch *b, const bsq_opts *opts, uint64_t first_call_seq);
/* Seeding only (BASELINE.json configs[1]; libbwa mem_collect_intv as called by mem_align1_core,
 * bwamem.c, for every read): SMEM passes 1 and 2 plus bwt_seed_strategy1, kept if end-start >=
 * min_seed_len, sorted by info.  The intervals stay on the device until bsq_batch_intervals. */
int bsq_batch_seed(bsq_batch *b, const bsq_opts *opts);
/* Intervals of the last bsq_batch_seed in read order: read i owns intervals [read_off[i],
 * read_off[i+1]); interval k is intv[4k..4k+3] = (x[0], x[1], x[2], info = qbeg<<32 | qend).  x[1]
 * (the reverse-strand interval start) is not part of the contract (the main-pass kernel does not keep
 * it for SMEMs; nothing on the alignment path reads it).  Borrowed arrays, valid until the next call
 * on the batch. */
int bsq_batch_intervals(bsq_batch *b, const int64_t **read_off, const uint64_t **intv, int64_t *n_intv);
/* The last run's rows rendered on the GPU as bwa_result text: the same bytes as bsq_render_tsv
 * (SURVEY.md 8(f) row 2).  `reads` are the batch's reads as nuclseq varlenas, for the symbols of their
 * holes (NULL: ambiguous bases print as N).  *text is borrowed (NUL-terminated, *len bytes), valid until
 * the next run, render or free of the batch. */
int bsq_batch_render(bsq_batch *b, const void *const *reads, const char **text, int64_t *len);
/* build_tuple_bwa's nuclseq columns of the last run's rows on the GPU (extension.cpp:282-305; per row it calls
 * nuclseq_from_text on ref_subseq and query_subseq, :285,290): varlena 2k = ref_subseq of row k, 2k+1 = its
 * query_subseq, the same bytes nuclseq_from_text gives for the texts bsq_render_tsv prints.  Layout as
 * bsq_nuclseq_encode_batch; both outputs malloc'd (bsq_free). */
int bsq_batch_render_nuclseqs(bsq_batch *b, const void *const *reads, uint8_t **out, int64_t **out_off);
/* Runs n batches concurrently (one host thread and HIP stream each); batch i draws lrand48 values from
 * first_call[i].  Each batch keeps its own result view.  Returns the first error, prefixed by the batch
 * index. */
int bsq_batch_run_many(bsq_batch *const *batches, int n, const bsq_opts *opts, const uint64_t *first_call);
/* bsq_batch_run_many `rounds` times with no barrier between rounds: each batch's thread runs its batch again as
 * soon as its previous run ends (a steady stream of cursor batches, extension.cpp:362-370 looped: one batch's
 * next seeding overlaps the others' dynamic-programming tails).  Every round re-aligns the batch's reads from
 * first_call[i], so the results equal one bsq_batch_run_many call's.  Stage times and bytes are the last
 * round's. */
int bsq_batch_run_rounds(bsq_batch *const *batches, int n, const bsq_opts *opts, const uint64_t *first_call,
                         int rounds);
/* Where bsq_batch_run copies the packed records: via_device = -1 (default) over this device's PCIe link into the
 * pinned view; via_device >= 0: by peer DMA (xGMI) into that device's HBM and from there into the same pinned view
 * over its link (the gather-to-one-device exchange of a device group).  The view and stage times are unchanged. */
int bsq_batch_set_record_route(bsq_batch *b, int via_device);
/* Borrowed view of the last run's hits (valid until the next run or free). */
const bsq_hits *bsq_batch_hits(const bsq_batch *b);
/* The last run's records as bytes in device memory on the batch's device: the bsq_hit array, then the CIGAR
   words (the exchange step's send buffer of a read-sharded multi-GPU job; the caller-side receive of
   extension.cpp:362-370's rows).  dst == NULL returns the size in *bytes.  BSQ_E_INVALID when cap is short. */
int bsq_batch_copy_records(const bsq_batch *b, void *dst, int64_t cap, int64_t *bytes);
/* Per-stage device time of the last run in ms, measured with HIP events on the batch stream.
 * Writes up to `max` values; returns the number of stages; names via bsq_stage_name(). */
int bsq_batch_stage_ms(const bsq_batch *b, float *ms, int max);
const char *bsq_stage_name(int stage);
/* Algorithmic bytes of the last run (SURVEY.md §8(d) counting), per stage: occ-block fetches x64,
 * SA values x8, reference windows ceil(bases/4), reads and hit records.  Returns stages written. */
int bsq_batch_stage_bytes(const bsq_batch *b, double *bytes, int max);
/* Work counters of the last run, per stage: DP cells evaluated (extend, reg2aln) and, for the
 * seeding stage, bwt_extend-equivalent steps (occ-block pairs + k-mer table reads).  Diagnostics. */
int bsq_batch_stage_work(const bsq_batch *b, double *work, int max);
/* Number of reads of the last run that needed the large-capacity retry pass. */
int64_t bsq_batch_retried(const bsq_batch *b);
/* Partition scans of klib's introsort (mem_chain_flt, mem_sort_dedup_patch, mem_mark_primary_se) that the kernels'
 * `i < t` bound stopped where klib's sentinel would not have -- summed over every run of this batch.  Always 0
 * for a correct sort (the sentinel is never swapped); the tests and bench.py assert it.  -1 for NULL. */
int64_t bsq_batch_sort_guard(const bsq_batch *b);
/* The same count over every batch run in this process (pipelines, one-shot calls and groups included). */
int64_t bsq_sort_guard_total(void);

#ifdef __cplusplus
}
#endif
#endif
