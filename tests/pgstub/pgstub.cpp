// pgstub.cpp -- TEST STUB: the runtime behind tests/pgstub/include/postgres.h and a fake executor that calls
// the extension's fmgr functions the way Postgres does (fcinfo with a ReturnSetInfo, SPI over registered
// "tables", a top-level error handler that longjmp'd ereports land in).  Built with
// bioseqdb_amd/pg/extension_bsq.cpp + bwa_bsq.cpp into a library that tests/test_pg_extension.py loads; the
// harness API (pgstub_*) registers tables, runs a call and returns its rows as text or its error.
//
// Checks built into the fake: SPI tuples are poisoned when SPI_freetuptable releases them (a batch that
// kept pointers past its fetch would read garbage), palloc'd memory is counted, and errors longjmp exactly
// like ereport(ERROR) so C++ frames between the error and the handler would be skipped.
#include "postgres.h"

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "bsq.h"
#include "bwa_bsq.h"

struct MemoryContextData { int id; };
struct HeapTupleHeaderData {
    int n;
    char names[16][32];
    int32 values[16];
    bool nulls[16];
};
struct PortalData { void *table; size_t pos; };
struct Tuplestorestate { std::vector<std::string> rows; };

extern "C" {
MemoryContext CurrentMemoryContext;
sigjmp_buf *PG_exception_stack;
uint64 SPI_processed;
SPITupleTable *SPI_tuptable;
int work_mem = 4096;
Datum nuclseq_search_bwa(FunctionCallInfo fcinfo);
Datum nuclseq_multi_search_bwa(FunctionCallInfo fcinfo);
}

namespace {

MemoryContextData g_top{1}, g_per_query{2};

// ---- memory ---------------------------------------------------------------------------------------
std::map<void *, size_t> g_allocs;
std::vector<std::unique_ptr<Tuplestorestate>> g_stores;   // released at the end of each call

// ---- errors -----------------------------------------------------------------------------------------
struct Err { int elevel = 0, code = 0; std::string msg; } g_err;
std::string g_debug;   // last DEBUG1..WARNING message
int g_cancel_after = -1, g_interrupts = 0;

// ---- SPI -----------------------------------------------------------------------------------------
struct Row { int64 id; bool id_null; std::vector<uint8_t> seq; bool seq_null; };
struct Table { Oid id_type, seq_type; std::vector<Row> rows; };
std::map<std::string, Table> g_tables;
bool g_spi_connected = false;
Oid g_nuclseq_oid = 16500;
int g_result_class = TYPEFUNC_COMPOSITE, g_allowed_modes = SFRM_Materialize | SFRM_ValuePerCall;
bool g_rsi_null = false;

TupleDesc new_desc(int natts, const Oid *types)
{
    TupleDesc d = (TupleDesc)palloc(sizeof(TupleDescData));
    memset(d, 0, sizeof *d);
    d->natts = natts;
    for (int i = 0; i < natts; ++i) d->attrs[i].atttypid = types[i];
    return d;
}

uint64_t fnv(const uint8_t *p, size_t n)
{
    uint64_t h = 0xcbf29ce484222325ull;
    for (size_t i = 0; i < n; ++i) { h ^= p[i]; h *= 0x100000001b3ull; }
    return h;
}

}  // namespace

extern "C" {

// ---- Postgres API (stub) -----------------------------------------------------------------------------
MemoryContext MemoryContextSwitchTo(MemoryContext c)
{
    MemoryContext old = CurrentMemoryContext;
    CurrentMemoryContext = c;
    return old;
}
void *palloc(size_t size)
{
    void *p = malloc(size ? size : 1);
    if (!p) ereport(ERROR, (errcode(ERRCODE_OUT_OF_MEMORY), errmsg("out of memory")));
    g_allocs[p] = size;
    return p;
}
void pfree(void *p)
{
    g_allocs.erase(p);
    free(p);
}
char *pstrdup(const char *s)
{
    char *p = (char *)palloc(strlen(s) + 1);
    strcpy(p, s);
    return p;
}

bool pgstub_errstart(int elevel)
{
    g_err = Err();
    g_err.elevel = elevel;
    g_err.code = elevel >= ERROR ? ERRCODE_INTERNAL_ERROR : 0;
    return true;
}
void pgstub_errfinish(void)
{
    if (g_err.elevel < ERROR) {
        g_debug = g_err.msg;
        return;
    }
    if (!PG_exception_stack) abort();   // an ereport outside any handler
    siglongjmp(*PG_exception_stack, 1);
}
int errcode(int sqlerrcode)
{
    g_err.code = sqlerrcode;
    return 0;
}
int errmsg(const char *fmt, ...)
{
    char buf[2048];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err.msg = buf;
    return 0;
}
ErrorData *CopyErrorData(void)
{
    ErrorData *e = (ErrorData *)palloc(sizeof(ErrorData));
    e->elevel = g_err.elevel;
    e->sqlerrcode = g_err.code;
    e->message = pstrdup(g_err.msg.c_str());
    return e;
}
void FlushErrorState(void) { g_err = Err(); }
void ReThrowError(ErrorData *edata)
{
    g_err.elevel = edata->elevel;
    g_err.code = edata->sqlerrcode;
    g_err.msg = edata->message;
    if (!PG_exception_stack) abort();
    siglongjmp(*PG_exception_stack, 1);
}
void pgstub_check_for_interrupts(void)
{
    if (g_cancel_after >= 0 && g_interrupts++ >= g_cancel_after)
        ereport(ERROR, (errcode(ERRCODE_QUERY_CANCELED), errmsg("canceling statement due to user request")));
}

TupleDesc CreateTupleDescCopy(TupleDesc t)
{
    TupleDesc d = (TupleDesc)palloc(sizeof(TupleDescData));
    memcpy(d, t, sizeof *d);
    return d;
}
TupleDesc BlessTupleDesc(TupleDesc t) { return t; }

Datum GetAttributeByName(HeapTupleHeader t, const char *name, bool *isnull)
{
    for (int i = 0; i < t->n; ++i) {
        if (!strcmp(t->names[i], name)) {
            *isnull = t->nulls[i];
            return Int32GetDatum(t->values[i]);
        }
    }
    ereport(ERROR, (errcode(ERRCODE_SYNTAX_ERROR), errmsg("attribute \"%s\" does not exist", name)));
    return 0;
}

Tuplestorestate *tuplestore_begin_heap(bool, bool, int)
{
    g_stores.emplace_back(new Tuplestorestate());
    return g_stores.back().get();
}

// Rows are kept as text, one column per field: nuclseq values are decoded (and fingerprinted) on the spot, so
// the datums handed in must be valid varlenas at the moment of the call (the tuplestore copies them).
void tuplestore_putvalues(Tuplestorestate *s, TupleDesc d, Datum *values, bool *isnull)
{
    std::string row;
    char buf[64];
    std::string fps;
    for (int i = 0; i < d->natts; ++i) {
        if (i) row += '\t';
        if (isnull[i]) { row += "\\N"; continue; }
        const Oid t = d->attrs[i].atttypid;
        if (t == INT8OID) { snprintf(buf, sizeof buf, "%lld", (long long)DatumGetInt64(values[i])); row += buf; }
        else if (t == INT4OID) { snprintf(buf, sizeof buf, "%d", DatumGetInt32(values[i])); row += buf; }
        else if (t == BOOLOID) row += DatumGetBool(values[i]) ? 't' : 'f';
        else if (t == TEXTOID) row.append(VARDATA(DatumGetPointer(values[i])), VARSIZE(DatumGetPointer(values[i])) - VARHDRSZ);
        else if (t == g_nuclseq_oid) {
            const uint8_t *ns = (const uint8_t *)DatumGetPointer(values[i]);
            if (!ns) { row += "<null pointer>"; continue; }
            char *txt = bsq_nuclseq_to_text(ns);
            row += txt;
            bsq_free(txt);
            snprintf(buf, sizeof buf, "\t%016llx", (unsigned long long)fnv(ns, VARSIZE(ns)));
            fps += buf;
        } else row += "?";
    }
    s->rows.push_back(row + fps);
}
void tuplestore_puttuple(Tuplestorestate *s, HeapTuple t)
{
    (void)s;
    (void)t;
    abort();   // the extension uses tuplestore_putvalues
}
HeapTuple heap_form_tuple(TupleDesc, Datum *, bool *)
{
    abort();
    return nullptr;
}
void heap_freetuple(HeapTuple) { abort(); }

TypeFuncClass get_call_result_type(FunctionCallInfo, Oid *, TupleDesc *desc)
{
    // bwa_result (bioseqdb--0.0.0.sql:196-212)
    const Oid types[15] = {INT8OID, g_nuclseq_oid, INT4OID, INT4OID, INT4OID, INT8OID, g_nuclseq_oid, INT4OID,
                           INT4OID, INT4OID, BOOLOID, BOOLOID, BOOLOID, TEXTOID, INT4OID};
    if (desc) *desc = new_desc(15, types);
    return (TypeFuncClass)g_result_class;
}

int SPI_connect(void)
{
    if (g_spi_connected) return -1;
    g_spi_connected = true;
    return 1;
}
int SPI_finish(void)
{
    g_spi_connected = false;
    return 2;
}
Portal SPI_cursor_open_with_args(const char *, const char *src, int, Oid *, Datum *, const char *, bool, int)
{
    if (!g_spi_connected) ereport(ERROR, (errmsg("SPI cursor opened while not connected")));
    auto it = g_tables.find(src);
    if (it == g_tables.end())
        ereport(ERROR, (errcode(ERRCODE_SYNTAX_ERROR), errmsg("stub executor: no table for query \"%s\"", src)));
    Portal p = (Portal)palloc(sizeof(PortalData));
    p->table = &it->second;
    p->pos = 0;
    return p;
}
void SPI_cursor_fetch(Portal portal, bool, long count)
{
    Table &t = *(Table *)portal->table;
    const size_t n = std::min<size_t>((size_t)count, t.rows.size() - portal->pos);
    SPI_processed = n;
    if (n == 0) { SPI_tuptable = nullptr; return; }
    SPITupleTable *tt = (SPITupleTable *)palloc(sizeof(SPITupleTable));
    const Oid types[2] = {t.id_type, t.seq_type};
    tt->tupdesc = new_desc(2, types);
    tt->numvals = n;
    tt->vals = (HeapTuple *)palloc(sizeof(HeapTuple) * n);
    for (size_t i = 0; i < n; ++i) {
        const Row &r = t.rows[portal->pos + i];
        HeapTuple h = (HeapTuple)palloc(sizeof(HeapTupleData));
        memset(h, 0, sizeof *h);
        h->natts = 2;
        h->values[0] = t.id_type == INT2OID ? Int32GetDatum((int16)r.id)
                       : t.id_type == INT4OID ? Int32GetDatum((int32)r.id) : Int64GetDatum(r.id);
        h->nulls[0] = r.id_null;
        if (!r.seq_null) {   // the tuple's own copy of the value, poisoned by SPI_freetuptable
            void *v = palloc(r.seq.size());
            memcpy(v, r.seq.data(), r.seq.size());
            h->values[1] = PointerGetDatum(v);
        }
        h->nulls[1] = r.seq_null;
        tt->vals[i] = h;
    }
    portal->pos += n;
    SPI_tuptable = tt;
}
void SPI_cursor_close(Portal portal) { pfree(portal); }
Oid SPI_gettypeid(TupleDesc d, int f) { return d->attrs[f - 1].atttypid; }
Datum SPI_getbinval(HeapTuple t, TupleDesc, int f, bool *isnull)
{
    *isnull = t->nulls[f - 1];
    return t->values[f - 1];
}
void SPI_freetuptable(SPITupleTable *tt)
{
    if (!tt) return;
    for (uint64 i = 0; i < tt->numvals; ++i) {
        HeapTuple h = tt->vals[i];
        if (!h->nulls[1]) {
            void *v = DatumGetPointer(h->values[1]);
            memset(v, 0xDB, g_allocs[v]);
            pfree(v);
        }
        pfree(h);
    }
    pfree(tt->vals);
    pfree(tt->tupdesc);
    pfree(tt);
    if (SPI_tuptable == tt) SPI_tuptable = nullptr;
}

// ---- harness API ---------------------------------------------------------------------------------------
void pgstub_reset(void)
{
    g_tables.clear();
    g_cancel_after = -1;
    g_interrupts = 0;
    g_result_class = TYPEFUNC_COMPOSITE;
    g_allowed_modes = SFRM_Materialize | SFRM_ValuePerCall;
    g_rsi_null = false;
    g_debug.clear();
}
void pgstub_clear_index_cache(void) { BwaIndexCache::backend().clear(); }
long pgstub_index_cache_hits(void) { return (long)BwaIndexCache::backend().hits(); }
long pgstub_index_cache_builds(void) { return (long)BwaIndexCache::backend().builds(); }
void pgstub_set_lrand48_calls(uint64_t calls) { bsq_backend_lrand48_calls() = calls; }
uint64_t pgstub_lrand48_calls(void) { return bsq_backend_lrand48_calls(); }
void pgstub_add_table(const char *sql, Oid id_type, Oid seq_type) { g_tables[sql] = Table{id_type, seq_type, {}}; }
void pgstub_add_row(const char *sql, int64 id, int id_null, const void *seq, int64 seq_bytes, int seq_null)
{
    Row r{id, id_null != 0, {}, seq_null != 0};
    if (seq && !seq_null) r.seq.assign((const uint8_t *)seq, (const uint8_t *)seq + seq_bytes);
    g_tables.at(sql).rows.push_back(std::move(r));
}
Oid pgstub_nuclseq_oid(void) { return g_nuclseq_oid; }
void pgstub_set_result_class(int cls) { g_result_class = cls; }
void pgstub_set_allowed_modes(int modes) { g_allowed_modes = modes; }
void pgstub_set_rsi_null(int on) { g_rsi_null = on != 0; }
void pgstub_cancel_after(int n)
{
    g_cancel_after = n;
    g_interrupts = 0;
}
const char *pgstub_last_debug(void) { return g_debug.c_str(); }
long pgstub_live_allocs(void) { return (long)g_allocs.size(); }

// bwa_options composite in the type's field order (bioseqdb--0.0.0.sql:160-173); nulls[i] != 0 is SQL NULL.
typedef struct { int32 values[12]; uint8_t nulls[12]; } pgstub_opts;

// Runs one call like the executor: on success *rows is the result set as text (one line per row, the 15
// columns then the fingerprints of the two nuclseq values) and 0 is returned; on an error *sqlstate (5 chars)
// and *message are set and 1 is returned.  Everything palloc'd by the call is released afterwards, as the
// end of the transaction would.
int pgstub_call(int multi, const char *query_sql, const void *query_nuclseq, const char *ref_sql, const pgstub_opts *o,
                char **rows, char *sqlstate, char **message)
{
    static const char *names[12] = {"min_seed_len", "max_occ", "match_score", "mismatch_penalty", "pen_clip3",
                                    "pen_clip5", "zdrop", "bandwidth", "o_del", "e_del", "o_ins", "e_ins"};
    HeapTupleHeaderData opts{};
    opts.n = 12;
    for (int i = 0; i < 12; ++i) {
        snprintf(opts.names[i], sizeof opts.names[i], "%s", names[i]);
        opts.values[i] = o->values[i];
        opts.nulls[i] = o->nulls[i] != 0;
    }
    ExprContext econtext{&g_per_query};
    ReturnSetInfo rsi{};
    rsi.type = T_ReturnSetInfo;
    rsi.econtext = &econtext;
    rsi.allowedModes = g_allowed_modes;
    FunctionCallInfoBaseData fc{};
    fc.resultinfo = g_rsi_null ? nullptr : (Node *)&rsi;
    fc.nargs = 3;
    fc.args[0].value = multi ? PointerGetDatum(query_sql) : PointerGetDatum(query_nuclseq);
    fc.args[1].value = PointerGetDatum(ref_sql);
    fc.args[2].value = PointerGetDatum(&opts);
    CurrentMemoryContext = &g_top;
    g_spi_connected = false;
    sigjmp_buf top;
    PG_exception_stack = &top;
    volatile int rc = 0;
    *rows = nullptr;
    *message = nullptr;
    sqlstate[0] = 0;
    if (sigsetjmp(top, 0) == 0) {
        if (multi) nuclseq_multi_search_bwa(&fc);
        else nuclseq_search_bwa(&fc);
        std::string out;
        if (rsi.setResult)
            for (const std::string &r : rsi.setResult->rows) { out += r; out += '\n'; }
        *rows = strdup(out.c_str());
    } else {
        rc = 1;
        for (int i = 0; i < 5; ++i) sqlstate[i] = (char)(((g_err.code >> (6 * i)) & 0x3F) + '0');
        sqlstate[5] = 0;
        *message = strdup(g_err.msg.c_str());
    }
    PG_exception_stack = nullptr;
    g_spi_connected = false;   // AtEOXact_SPI
    for (auto &a : g_allocs) free(a.first);
    g_allocs.clear();
    g_stores.clear();
    return rc;
}

}  // extern "C"
