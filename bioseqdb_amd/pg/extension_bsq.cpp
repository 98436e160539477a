// extension_bsq.cpp -- bioseqdb's BWA alignment functions over libbsq: the fmgr/SPI layer of
// bioseqdb/extension.cpp:154-378 (iterate_nuclseq_table, get_opt_or, bwa_index_from_query, the SRF checks,
// create_tuplestore, build_tuple_bwa, nuclseq_search_bwa, nuclseq_multi_search_bwa) rewritten for a batched
// GPU backend.  The SQL surface (bioseqdb--0.0.0.sql:160-222), the symbols, the argument meaning, the row
// layout and order, and every error message and SQLSTATE are the reference's.  What differs:
//
//  * the query cursor is fetched BSQ_FETCH_ROWS rows at a time (default 262144; the reference fetches one,
//    Q14) and every fetch is aligned by one libbsq call while its tuples are still valid;
//  * the two nuclseq columns of each row (build_tuple_bwa's nuclseq_from_text calls) come from the GPU
//    renderer, the CIGAR text is formatted from the records, and rows go to the tuplestore with
//    tuplestore_putvalues (no heap_form_tuple / palloc per row);
//  * the built index is cached across calls (BwaIndexCache, keyed by a digest of the reference rows), where
//    the reference rebuilds it on every call (Q13);
//  * Postgres errors raised inside SPI/tuplestore calls are caught (PG_TRY) and re-raised only after the C++
//    objects of the call are destroyed; libbsq failures become ereport(ERROR) at the same point, so nothing
//    longjmps over a destructor;
//  * CHECK_FOR_INTERRUPTS() between fetches and an elog(DEBUG1) summary per call.
//
// Deliberate divergence: max_occ, e_del and e_ins of 0 are rejected ("bwa_opt %s must be positive"); the
// reference divides by them (libbwa mem_chain, cal_max_gap, ksw_extend2), i.e. crashes or computes with inf.
// The rest of bioseqdb's extension.cpp (nuclseq I/O and operators, PG_MODULE_MAGIC) is unchanged.
extern "C" {
#include <postgres.h>
#include <fmgr.h>
#include <funcapi.h>
#include <miscadmin.h>
#include <executor/spi.h>
#include <catalog/pg_type.h>
}

#include <algorithm>
#include <chrono>
#include <list>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "bwa_bsq.h"

namespace {

// ---- errors ------------------------------------------------------------------------------------------

struct PgError { ErrorData *edata; };                  // a Postgres error caught by pg_call
struct SqlError { int sqlstate; std::string message; };  // an error of ours, raised after cleanup

// Runs Postgres calls that may ereport/elog.  f must not throw C++ exceptions (it runs inside PG_TRY).
template <class F>
void pg_call(F &&f)
{
    MemoryContext mcx = CurrentMemoryContext;
    ErrorData *volatile edata = nullptr;
    PG_TRY();
    {
        f();
    }
    PG_CATCH();
    {
        MemoryContextSwitchTo(mcx);
        edata = CopyErrorData();
        FlushErrorState();
    }
    PG_END_TRY();
    if (edata) throw PgError{edata};
}

struct Failure {
    ErrorData *pg = nullptr;
    int sqlstate = 0;
};

thread_local char g_message[1024];   // our error text, kept outside the unwound frames

// Runs the body of an SQL function; every C++ object it creates is destroyed before this returns.
template <class F>
Failure run_body(F &&body) noexcept
{
    Failure f;
    auto keep = [&](int code, const char *what) {
        f.sqlstate = code;
        snprintf(g_message, sizeof g_message, "%s", what);
    };
    try {
        body();
    } catch (const PgError &e) {
        f.pg = e.edata;
    } catch (const SqlError &e) {
        keep(e.sqlstate, e.message.c_str());
    } catch (const BsqFailure &e) {
        const int code = e.code == BSQ_E_NOMEM ? ERRCODE_OUT_OF_MEMORY
                         : e.code == BSQ_E_INVALID ? ERRCODE_INVALID_PARAMETER_VALUE
                         : ERRCODE_EXTERNAL_ROUTINE_EXCEPTION;
        keep(code, (std::string("libbsq: ") + e.what()).c_str());
    } catch (const std::bad_alloc &) {
        keep(ERRCODE_OUT_OF_MEMORY, "out of memory");
    } catch (const std::exception &e) {
        keep(ERRCODE_INTERNAL_ERROR, e.what());
    }
    return f;
}

void raise_after_cleanup(const Failure &f)
{
    if (f.pg) ReThrowError(f.pg);
    if (f.sqlstate) ereport(ERROR, (errcode(f.sqlstate), errmsg("%s", g_message)));
}

// ---- configuration ---------------------------------------------------------------------------------

long env_long(const char *name, long dflt, long lo)
{
    const char *e = getenv(name);
    return e && *e ? std::max(lo, atol(e)) : dflt;
}
// BSQ_DEVICES="0,1,2,3": the backend aligns over a group of GPUs (bsq_group); else the one BSQ_DEVICE
std::vector<int> backend_devices()
{
    std::vector<int> d;
    if (const char *e = getenv("BSQ_DEVICES")) {
        for (const char *p = e; *p;) {
            char *end = nullptr;
            const long v = strtol(p, &end, 10);
            if (end == p) { ++p; continue; }
            if (v >= 0) d.push_back((int)v);
            p = end;
        }
    }
    if (d.empty()) d.push_back((int)env_long("BSQ_DEVICE", 0, 0));
    return d;
}
long query_fetch_rows() { return env_long("BSQ_FETCH_ROWS", 1L << 18, 1); }
constexpr long kRefFetchRows = 64;   // reference rows are long; their bytes are copied by add_ref_sequence

// ---- SPI cursor ----------------------------------------------------------------------------------------

// iterate_nuclseq_table (extension.cpp:156-195): (int2/4/8 id, nuclseq) rows of `sql`, NULL rows skipped,
// the column types checked on every fetch with the reference's messages.  Each fetch of up to `fetch` rows is
// handed to on_rows(ids, seqs, submitted) while its tuples are valid, then released.
// If on_rows stores a ticket >= 0 in `submitted` (a deferred pipeline submission that still reads the tuples; it
// must store it right after the submission, before anything that can throw), the tuples of that fetch are freed
// only after the NEXT fetch has been fetched and handed over and wait(ticket) has returned, so the staging of fetch
// k runs on a pipeline worker while this backend fetches k+1.  Unwinding with a ticket outstanding -- held, or just
// submitted when on_rows or the release of the previous fetch threw -- waits for the newest one first (fetches are
// staged in submission order): no worker reads tuple memory after control leaves this function.
template <class F, class W>
void for_each_fetch_held(const char *sql, Oid nuclseq_oid, long fetch, F &&on_rows, W &&wait)
{
    Portal portal = nullptr;
    pg_call([&] { portal = SPI_cursor_open_with_args(nullptr, sql, 0, nullptr, nullptr, nullptr, true, 0); });
    std::vector<int64_t> ids[2];
    std::vector<const NucleotideSequence *> seqs[2];   // alternate: the held fetch's pointers stay valid
    SPITupleTable *held_tt = nullptr;
    int64_t held_ticket = -1, pending = -1;
    struct Guard {
        W &wait;
        int64_t &held, &pending;
        ~Guard()
        {
            const int64_t t = std::max(held, pending);
            if (t >= 0) {
                try { wait(t); } catch (...) {}
            }
        }
    } guard{wait, held_ticket, pending};
    auto release_held = [&] {
        if (held_ticket >= 0) { const int64_t t = held_ticket; held_ticket = -1; wait(t); }
        if (held_tt) { SPITupleTable *t = held_tt; held_tt = nullptr; pg_call([&] { SPI_freetuptable(t); }); }
    };
    for (int cur = 0;; cur ^= 1) {
        uint64 n = 0;
        SPITupleTable *tt = nullptr;
        pg_call([&] {
            CHECK_FOR_INTERRUPTS();
            SPI_cursor_fetch(portal, true, fetch);
            n = SPI_processed;
            tt = SPI_tuptable;
        });
        if (n == 0 || tt == nullptr) break;
        Oid id_type = InvalidOid, seq_type = InvalidOid;
        pg_call([&] {
            id_type = SPI_gettypeid(tt->tupdesc, 1);
            seq_type = SPI_gettypeid(tt->tupdesc, 2);
        });
        if (id_type != INT2OID && id_type != INT4OID && id_type != INT8OID)
            throw SqlError{ERRCODE_DATATYPE_MISMATCH, "expected column of integers"};
        if (seq_type != nuclseq_oid) throw SqlError{ERRCODE_DATATYPE_MISMATCH, "expected column of nuclseqs"};
        std::vector<int64_t> &id_v = ids[cur];
        std::vector<const NucleotideSequence *> &seq_v = seqs[cur];
        id_v.resize((size_t)n);
        seq_v.resize((size_t)n);
        size_t kept = 0;
        pg_call([&] {
            for (uint64 i = 0; i < n; ++i) {
                bool null_id = false, null_seq = false;
                const Datum id = SPI_getbinval(tt->vals[i], tt->tupdesc, 1, &null_id);
                const Datum seq = SPI_getbinval(tt->vals[i], tt->tupdesc, 2, &null_seq);
                if (null_id || null_seq) continue;
                id_v[kept] = id_type == INT2OID ? (int64_t)DatumGetInt16(id)
                             : id_type == INT4OID ? (int64_t)DatumGetInt32(id) : (int64_t)DatumGetInt64(id);
                seq_v[kept] = reinterpret_cast<const NucleotideSequence *>(PG_DETOAST_DATUM(seq));
                ++kept;
            }
        });
        id_v.resize(kept);
        seq_v.resize(kept);
        pending = -1;
        on_rows(id_v, seq_v, pending);
        release_held();   // the previous fetch: staged by now or waited for
        if (pending >= 0) { held_tt = tt; held_ticket = pending; pending = -1; }
        else pg_call([&] { SPI_freetuptable(tt); });
    }
    release_held();
    pg_call([&] { SPI_cursor_close(portal); });
}

template <class F>
void for_each_fetch(const char *sql, Oid nuclseq_oid, long fetch, F &&on_rows)
{
    for_each_fetch_held(sql, nuclseq_oid, fetch,
                        [&](const std::vector<int64_t> &ids, const std::vector<const NucleotideSequence *> &seqs,
                            int64_t &) { on_rows(ids, seqs); },
                        [](int64_t) {});
}

// ---- options and index ---------------------------------------------------------------------------------

// get_opt_or (extension.cpp:197-209)
int32_t opt_or(HeapTupleHeader opts, const char *name, int32_t dflt)
{
    bool isnull = false;
    Datum v = 0;
    pg_call([&] { v = GetAttributeByName(opts, name, &isnull); });
    if (isnull) return dflt;
    const int32_t x = DatumGetInt32(v);
    if (x < 0) throw SqlError{ERRCODE_INVALID_PARAMETER_VALUE, std::string("bwa_opt ") + name + " must be nonnegative"};
    return x;
}

struct CallIndex {
    std::shared_ptr<BwaIndex> index;
    BsqMemOpt opt;
    size_t n_refs = 0;
    bool cached = false;
    double ms = 0;
};

// bwa_index_from_query (extension.cpp:211-236): reference rows, then the options in the reference's order
// (mem_opt_t names; the Q1 swap happened in bwa_opts()), then the index, built or found in the backend cache.
CallIndex index_from_query(const char *sql, HeapTupleHeader opts, Oid nuclseq_oid)
{
    const auto t0 = std::chrono::steady_clock::now();
    auto fresh = std::make_shared<BwaIndex>(backend_devices());
    RefDigest digest;
    for_each_fetch(sql, nuclseq_oid, kRefFetchRows, [&](const std::vector<int64_t> &ids,
                                                       const std::vector<const NucleotideSequence *> &seqs) {
        for (size_t i = 0; i < ids.size(); ++i) {
            digest.update(ids[i], seqs[i]);
            fresh->add_ref_sequence(ids[i], *seqs[i]);
        }
    });
    CallIndex c;
    c.n_refs = (size_t)digest.rows;
    BsqMemOpt &o = c.opt;
    o.max_occ = opt_or(opts, "max_occ", std::max<int>(500, (int)(c.n_refs * 2)));
    o.min_seed_len = opt_or(opts, "min_seed_len", 19);
    o.a = opt_or(opts, "match_score", 1);
    o.b = opt_or(opts, "mismatch_penalty", 4);
    o.pen_clip3 = opt_or(opts, "pen_clip3", 5);
    o.pen_clip5 = opt_or(opts, "pen_clip5", 5);
    o.zdrop = opt_or(opts, "zdrop", 100);
    o.w = opt_or(opts, "bandwidth", 100);
    o.o_del = opt_or(opts, "o_del", 6);
    o.o_ins = opt_or(opts, "o_ins", 6);
    o.e_del = opt_or(opts, "e_del", 1);
    o.e_ins = opt_or(opts, "e_ins", 1);
    const std::pair<const char *, int> divisors[] = {{"max_occ", o.max_occ}, {"e_del", o.e_del}, {"e_ins", o.e_ins}};
    for (const auto &d : divisors)
        if (d.second == 0)
            throw SqlError{ERRCODE_INVALID_PARAMETER_VALUE, std::string("bwa_opt ") + d.first + " must be positive"};
    const size_t builds = BwaIndexCache::backend().builds();
    c.index = BwaIndexCache::backend().get_or_build(digest, std::move(fresh));
    c.cached = BwaIndexCache::backend().builds() == builds;
    c.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return c;
}

// ---- result set ------------------------------------------------------------------------------------

// assert_can_return_set (extension.cpp:238-247)
void check_can_return_set(ReturnSetInfo *rsi)
{
    bool is_rsi = false;
    int modes = 0;
    pg_call([&] {
        is_rsi = rsi != nullptr && IsA(rsi, ReturnSetInfo);
        if (is_rsi) modes = rsi->allowedModes;
    });
    if (!is_rsi)
        throw SqlError{ERRCODE_FEATURE_NOT_SUPPORTED, "set-valued function called in context that cannot accept a set"};
    if (!(modes & SFRM_Materialize))
        throw SqlError{ERRCODE_FEATURE_NOT_SUPPORTED, "materialize mode required, but it is not allowed in this context"};
}

// get_retval_tupledesc (extension.cpp:249-266)
TupleDesc call_result_desc(FunctionCallInfo fcinfo)
{
    TupleDesc desc = nullptr;
    TypeFuncClass cls = TYPEFUNC_OTHER;
    pg_call([&] { cls = get_call_result_type(fcinfo, nullptr, &desc); });
    if (cls == TYPEFUNC_RECORD)
        throw SqlError{ERRCODE_FEATURE_NOT_SUPPORTED,
                       "function returning record called in context that cannot accept type record"};
    if (cls != TYPEFUNC_COMPOSITE) throw SqlError{ERRCODE_FEATURE_NOT_SUPPORTED, "return type must be a row type"};
    return desc;
}

// create_tuplestore (extension.cpp:268-280)
Tuplestorestate *create_store(ReturnSetInfo *rsi, TupleDesc &desc)
{
    Tuplestorestate *store = nullptr;
    pg_call([&] {
        MemoryContext old = MemoryContextSwitchTo(rsi->econtext->ecxt_per_query_memory);
        desc = BlessTupleDesc(CreateTupleDescCopy(desc));
        store = tuplestore_begin_heap((rsi->allowedModes & SFRM_Materialize_Random) != 0, false, work_mem);
        MemoryContextSwitchTo(old);
    });
    return store;
}

// build_tuple_bwa (extension.cpp:282-305) for every row of an aligned batch, straight into the tuplestore.
// query_ids == nullptr: the single-query function (query_id NULL).
void put_rows(Tuplestorestate *store, TupleDesc desc, const BwaRows &rows, const int64_t *query_ids)
{
    const int64_t n_rows = rows.n_rows();
    if (n_rows == 0) return;
    // CIGAR text datums (4-byte varlena headers, 8-byte aligned), formatted before entering Postgres calls
    std::vector<int64_t> cig_off((size_t)n_rows + 1, 0);
    std::string arena, cig;
    for (int64_t k = 0; k < n_rows; ++k) {
        rows.cigar_text(k, cig);
        const size_t at = arena.size(), size = VARHDRSZ + cig.size();
        arena.resize((at + size + 7) & ~(size_t)7);
        SET_VARSIZE(&arena[at], size);
        memcpy(VARDATA(&arena[at]), cig.data(), cig.size());
        cig_off[(size_t)k + 1] = (int64_t)arena.size();
    }
    pg_call([&] {
        Datum values[15];
        bool nulls[15] = {false};
        nulls[5] = query_ids == nullptr;
        for (int32_t i = 0; i < rows.n_reads(); ++i) {
            for (int64_t k = rows.begin(i); k < rows.end(i); ++k) {
                const bsq_hit &h = rows.row(k);
                values[0] = Int64GetDatum(h.ref_id);
                values[1] = PointerGetDatum(rows.ref_subseq(k));
                values[2] = Int32GetDatum(h.ref_match_start);
                values[3] = Int32GetDatum(h.ref_match_end);
                values[4] = Int32GetDatum(h.ref_match_len);
                values[5] = Int64GetDatum(query_ids ? query_ids[i] : 0);
                values[6] = PointerGetDatum(rows.query_subseq(k));
                values[7] = Int32GetDatum(h.qb);
                values[8] = Int32GetDatum(h.qe);
                values[9] = Int32GetDatum(h.qe - h.qb);
                values[10] = BoolGetDatum(h.is_primary != 0);
                values[11] = BoolGetDatum(h.is_secondary != 0);
                values[12] = BoolGetDatum(h.is_reverse != 0);
                values[13] = PointerGetDatum(&arena[(size_t)cig_off[(size_t)k]]);
                values[14] = Int32GetDatum(h.score);
                tuplestore_putvalues(store, desc, values, nulls);
            }
        }
    });
}

struct CallStats {
    long long reads = 0, rows = 0;
    double align_ms = 0;
};

void finish(ReturnSetInfo *rsi, Tuplestorestate *store, TupleDesc desc, const char *fn, const CallIndex &ci,
            const CallStats &st)
{
    pg_call([&] {
        SPI_finish();
        elog(DEBUG1, "%s: %zu reference rows, index %s in %.1f ms on device %d; %lld reads, %lld rows, %.1f ms aligning",
             fn, ci.n_refs, ci.cached ? "cached" : "built", ci.ms, ci.index->device(), st.reads, st.rows, st.align_ms);
        rsi->returnMode = SFRM_Materialize;
        rsi->setResult = store;
        rsi->setDesc = desc;
    });
}

void connect_spi()
{
    int ret = 0;
    pg_call([&] { ret = SPI_connect(); });
    if (ret < 0) throw SqlError{ERRCODE_INTERNAL_ERROR, "connectby: SPI_connect returned " + std::to_string(ret)};
}

// nuclseq_multi_search_bwa (extension.cpp:345-378)
void multi_search(FunctionCallInfo fcinfo)
{
    ReturnSetInfo *rsi = nullptr;
    pg_call([&] { rsi = reinterpret_cast<ReturnSetInfo *>(fcinfo->resultinfo); });
    check_can_return_set(rsi);
    const char *query_sql = nullptr, *reference_sql = nullptr;
    HeapTupleHeader opts = nullptr;
    pg_call([&] {
        query_sql = PG_GETARG_CSTRING(0);
        reference_sql = PG_GETARG_CSTRING(1);
        opts = PG_GETARG_HEAPTUPLEHEADER(2);
    });
    connect_spi();
    TupleDesc desc = call_result_desc(fcinfo);
    Oid nuclseq_oid = InvalidOid;
    pg_call([&] { nuclseq_oid = TupleDescAttr(desc, 1)->atttypid; });
    const CallIndex ci = index_from_query(reference_sql, opts, nuclseq_oid);
    Tuplestorestate *store = create_store(rsi, desc);
    CallStats st;
    // The cursor loop as a pipeline (bsq_pipeline): each fetch is staged and submitted, its tuples released at
    // once, and the oldest fetch's rows go into the tuplestore only when the pipeline is full -- so the GPU
    // aligns fetches k-depth+1..k while the backend fetches k+1 and builds the tuples of k-depth.  Rows still
    // come out in cursor order (extension.cpp:362-370 aligns and stores one row at a time).
    const BwaIndex &index = *ci.index;
    index.reset_rows();   // a cached index may hold submissions of a call that failed midway
    const int depth = index.pipeline_depth();
    std::list<std::vector<int64_t>> ids_q;   // query ids of the submitted fetches, oldest first
    const auto t0 = std::chrono::steady_clock::now();
    auto drain_one = [&] {
        const BwaRows &rows = index.take_rows();
        put_rows(store, desc, rows, ids_q.front().data());
        st.rows += rows.n_rows();
        index.release_rows();
        ids_q.pop_front();
    };
    // Each fetch is staged by a pipeline worker (deferred submission) while this backend fetches the next one; its
    // tuples are freed once that staging is done (for_each_fetch_held).
    for_each_fetch_held(query_sql, nuclseq_oid, query_fetch_rows(),
                        [&](const std::vector<int64_t> &ids, const std::vector<const NucleotideSequence *> &seqs,
                            int64_t &submitted) {
                            if ((int)ids_q.size() >= depth) drain_one();
                            submitted = index.submit_rows(seqs.data(), (int32_t)seqs.size(), true, &ci.opt, true);
                            ids_q.push_back(ids);
                            st.reads += (long long)seqs.size();
                        },
                        [&](int64_t ticket) { index.wait_staged(ticket); });
    while (!ids_q.empty()) drain_one();
    st.align_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    finish(rsi, store, desc, "nuclseq_multi_search_bwa", ci, st);
}

// nuclseq_search_bwa (extension.cpp:311-343)
void single_search(FunctionCallInfo fcinfo)
{
    ReturnSetInfo *rsi = nullptr;
    pg_call([&] { rsi = reinterpret_cast<ReturnSetInfo *>(fcinfo->resultinfo); });
    check_can_return_set(rsi);
    const NucleotideSequence *query = nullptr;
    const char *reference_sql = nullptr;
    HeapTupleHeader opts = nullptr;
    pg_call([&] {
        query = reinterpret_cast<const NucleotideSequence *>(PG_DETOAST_DATUM(PG_GETARG_DATUM(0)));
        reference_sql = PG_GETARG_CSTRING(1);
        opts = PG_GETARG_HEAPTUPLEHEADER(2);
    });
    connect_spi();
    TupleDesc desc = call_result_desc(fcinfo);
    Oid nuclseq_oid = InvalidOid;
    pg_call([&] { nuclseq_oid = TupleDescAttr(desc, 1)->atttypid; });
    const CallIndex ci = index_from_query(reference_sql, opts, nuclseq_oid);
    Tuplestorestate *store = create_store(rsi, desc);
    CallStats st;
    const auto t0 = std::chrono::steady_clock::now();
    const BwaRows &rows = ci.index->align_rows(&query, 1, true, &ci.opt);
    put_rows(store, desc, rows, nullptr);
    st.align_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    st.reads = 1;
    st.rows = rows.n_rows();
    finish(rsi, store, desc, "nuclseq_search_bwa", ci, st);
}

}  // namespace

extern "C" {

PG_FUNCTION_INFO_V1(nuclseq_search_bwa);
Datum nuclseq_search_bwa(PG_FUNCTION_ARGS)
{
    raise_after_cleanup(run_body([&] { single_search(fcinfo); }));
    return (Datum)0;
}

PG_FUNCTION_INFO_V1(nuclseq_multi_search_bwa);
Datum nuclseq_multi_search_bwa(PG_FUNCTION_ARGS)
{
    raise_after_cleanup(run_body([&] { multi_search(fcinfo); }));
    return (Datum)0;
}

}  // extern "C"
