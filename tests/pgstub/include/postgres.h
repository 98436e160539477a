/*
 * postgres.h -- TEST STUB of the slice of the Postgres server API that bioseqdb_amd/pg/extension_bsq.cpp uses
 * (fmgr V1 calls, SPI cursors, set-returning functions via a tuplestore, ereport/elog with PG_TRY/PG_CATCH,
 * GetAttributeByName on the bwa_options composite).  Postgres server headers are not in this image; this
 * stand-in lets tests/test_pg_extension.py compile the extension layer and drive it from a fake executor
 * (tests/pgstub/pgstub.cpp).  Semantics follow the Postgres API: errors at ERROR level longjmp to the
 * innermost PG_TRY (or the fake executor), Datums are pointer-sized, varlenas carry 4-byte headers.
 * It is not Postgres and is only ever linked into the test harness library.
 */
#ifndef PGSTUB_POSTGRES_H
#define PGSTUB_POSTGRES_H

#include <setjmp.h>
#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef uintptr_t Datum;
typedef unsigned int Oid;
typedef int16_t int16;
typedef int32_t int32;
typedef int64_t int64;
typedef uint32_t uint32;
typedef uint64_t uint64;

#define InvalidOid ((Oid)0)
#define BOOLOID 16
#define INT8OID 20
#define INT2OID 21
#define INT4OID 23
#define TEXTOID 25

/* ---- varlena -------------------------------------------------------------------------------------- */
struct varlena { char vl_len_[4]; char vl_dat[1]; };
typedef struct varlena text;
#define VARHDRSZ ((int32)sizeof(int32))
#define SET_VARSIZE(p, len) (*(uint32 *)(p) = ((uint32)(len)) << 2)
#define VARSIZE(p) ((*(const uint32 *)(p)) >> 2)
#define VARDATA(p) (((char *)(p)) + VARHDRSZ)

static inline Datum PointerGetDatum(const void *p) { return (Datum)p; }
#define DatumGetPointer(d) ((char *)(d))
static inline Datum Int64GetDatum(int64 x) { return (Datum)x; }
static inline Datum Int32GetDatum(int32 x) { return (Datum)(intptr_t)x; }
static inline Datum BoolGetDatum(bool x) { return (Datum)(x ? 1 : 0); }
static inline int64 DatumGetInt64(Datum d) { return (int64)d; }
static inline int32 DatumGetInt32(Datum d) { return (int32)d; }
static inline int16 DatumGetInt16(Datum d) { return (int16)d; }
static inline bool DatumGetBool(Datum d) { return d != 0; }

/* ---- memory ---------------------------------------------------------------------------------------- */
typedef struct MemoryContextData *MemoryContext;
extern MemoryContext CurrentMemoryContext;
MemoryContext MemoryContextSwitchTo(MemoryContext context);
void *palloc(size_t size);
void pfree(void *p);
char *pstrdup(const char *s);
extern int work_mem;

/* ---- errors ---------------------------------------------------------------------------------------- */
#define DEBUG1 14
#define LOG 15
#define NOTICE 18
#define WARNING 19
#define ERROR 21

#define PGSIXBIT(ch) (((ch) - '0') & 0x3F)
#define MAKE_SQLSTATE(c1, c2, c3, c4, c5) \
    (PGSIXBIT(c1) + (PGSIXBIT(c2) << 6) + (PGSIXBIT(c3) << 12) + (PGSIXBIT(c4) << 18) + (PGSIXBIT(c5) << 24))
#define ERRCODE_FEATURE_NOT_SUPPORTED MAKE_SQLSTATE('0', 'A', '0', '0', '0')
#define ERRCODE_INVALID_PARAMETER_VALUE MAKE_SQLSTATE('2', '2', '0', '2', '3')
#define ERRCODE_INVALID_TEXT_REPRESENTATION MAKE_SQLSTATE('2', '2', 'P', '0', '2')
#define ERRCODE_EXTERNAL_ROUTINE_EXCEPTION MAKE_SQLSTATE('3', '8', '0', '0', '0')
#define ERRCODE_DATATYPE_MISMATCH MAKE_SQLSTATE('4', '2', '8', '0', '4')
#define ERRCODE_SYNTAX_ERROR MAKE_SQLSTATE('4', '2', '6', '0', '1')
#define ERRCODE_OUT_OF_MEMORY MAKE_SQLSTATE('5', '3', '2', '0', '0')
#define ERRCODE_QUERY_CANCELED MAKE_SQLSTATE('5', '7', '0', '1', '4')
#define ERRCODE_INTERNAL_ERROR MAKE_SQLSTATE('X', 'X', '0', '0', '0')

typedef struct ErrorData {
    int elevel;
    int sqlerrcode;
    char *message;
} ErrorData;

extern sigjmp_buf *PG_exception_stack;
bool pgstub_errstart(int elevel);
void pgstub_errfinish(void);
int errcode(int sqlerrcode);
int errmsg(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
ErrorData *CopyErrorData(void);
void FlushErrorState(void);
void ReThrowError(ErrorData *edata) __attribute__((noreturn));

#define ereport(elevel, ...)                      \
    do {                                          \
        if (pgstub_errstart(elevel)) {            \
            __VA_ARGS__;                          \
            pgstub_errfinish();                   \
        }                                         \
    } while (0)
#define elog(elevel, ...)                         \
    do {                                          \
        if (pgstub_errstart(elevel)) {            \
            errmsg(__VA_ARGS__);                  \
            pgstub_errfinish();                   \
        }                                         \
    } while (0)

#define PG_TRY()                                                  \
    do {                                                          \
        sigjmp_buf *_save_exception_stack = PG_exception_stack;   \
        sigjmp_buf _local_sigjmp_buf;                             \
        if (sigsetjmp(_local_sigjmp_buf, 0) == 0) {               \
            PG_exception_stack = &_local_sigjmp_buf;
#define PG_CATCH()                                                \
        } else {                                                  \
            PG_exception_stack = _save_exception_stack;
#define PG_END_TRY()                                              \
        }                                                         \
        PG_exception_stack = _save_exception_stack;               \
    } while (0)

void pgstub_check_for_interrupts(void);
#define CHECK_FOR_INTERRUPTS() pgstub_check_for_interrupts()

/* ---- tuples ----------------------------------------------------------------------------------------- */
#define PGSTUB_MAX_ATTS 16
typedef struct FormData_pg_attribute { Oid atttypid; char attname[64]; } FormData_pg_attribute;
typedef FormData_pg_attribute *Form_pg_attribute;
typedef struct TupleDescData { int natts; FormData_pg_attribute attrs[PGSTUB_MAX_ATTS]; } TupleDescData;
typedef TupleDescData *TupleDesc;
#define TupleDescAttr(tupdesc, i) (&(tupdesc)->attrs[(i)])
TupleDesc CreateTupleDescCopy(TupleDesc tupdesc);
TupleDesc BlessTupleDesc(TupleDesc tupdesc);

typedef struct HeapTupleData { int natts; Datum values[PGSTUB_MAX_ATTS]; bool nulls[PGSTUB_MAX_ATTS]; } HeapTupleData;
typedef HeapTupleData *HeapTuple;
typedef struct HeapTupleHeaderData HeapTupleHeaderData;   /* a composite value (bwa_options) */
typedef HeapTupleHeaderData *HeapTupleHeader;
Datum GetAttributeByName(HeapTupleHeader tuple, const char *attname, bool *isNull);

typedef struct Tuplestorestate Tuplestorestate;
Tuplestorestate *tuplestore_begin_heap(bool randomAccess, bool interXact, int maxKBytes);
void tuplestore_putvalues(Tuplestorestate *state, TupleDesc tdesc, Datum *values, bool *isnull);
void tuplestore_puttuple(Tuplestorestate *state, HeapTuple tuple);
HeapTuple heap_form_tuple(TupleDesc tupleDescriptor, Datum *values, bool *isnull);
void heap_freetuple(HeapTuple htup);

/* ---- fmgr ------------------------------------------------------------------------------------------- */
typedef struct Node { int type; } Node;
typedef struct NullableDatum { Datum value; bool isnull; } NullableDatum;
typedef struct FunctionCallInfoBaseData {
    void *flinfo;
    Node *context;
    Node *resultinfo;
    Oid fncollation;
    bool isnull;
    short nargs;
    NullableDatum args[8];
} FunctionCallInfoBaseData;
typedef FunctionCallInfoBaseData *FunctionCallInfo;
#define PG_FUNCTION_ARGS FunctionCallInfo fcinfo
#define PG_GETARG_DATUM(n) (fcinfo->args[(n)].value)
#define PG_GETARG_POINTER(n) DatumGetPointer(PG_GETARG_DATUM(n))
#define PG_GETARG_CSTRING(n) ((char *)DatumGetPointer(PG_GETARG_DATUM(n)))
#define PG_DETOAST_DATUM(datum) ((struct varlena *)DatumGetPointer(datum))
#define PG_GETARG_HEAPTUPLEHEADER(n) ((HeapTupleHeader)DatumGetPointer(PG_GETARG_DATUM(n)))
#define PG_FUNCTION_INFO_V1(funcname) extern Datum funcname(PG_FUNCTION_ARGS)
#define PG_MODULE_MAGIC extern int pgstub_module_magic

/* ---- set-returning functions (funcapi.h, nodes/execnodes.h) ----------------------------------------- */
typedef enum TypeFuncClass {
    TYPEFUNC_SCALAR,
    TYPEFUNC_COMPOSITE,
    TYPEFUNC_COMPOSITE_DOMAIN,
    TYPEFUNC_RECORD,
    TYPEFUNC_OTHER
} TypeFuncClass;
TypeFuncClass get_call_result_type(FunctionCallInfo fcinfo, Oid *resultTypeId, TupleDesc *resultTupleDesc);
typedef enum SetFunctionReturnMode {
    SFRM_ValuePerCall = 0x01,
    SFRM_Materialize = 0x02,
    SFRM_Materialize_Random = 0x04,
    SFRM_Materialize_Preferred = 0x08
} SetFunctionReturnMode;
typedef struct ExprContext { MemoryContext ecxt_per_query_memory; } ExprContext;
#define T_ReturnSetInfo 418
typedef struct ReturnSetInfo {
    int type;
    ExprContext *econtext;
    TupleDesc expectedDesc;
    int allowedModes;
    SetFunctionReturnMode returnMode;
    int isDone;
    Tuplestorestate *setResult;
    TupleDesc setDesc;
} ReturnSetInfo;
#define IsA(nodeptr, _type_) (((const Node *)(nodeptr))->type == T_##_type_)

/* ---- SPI ------------------------------------------------------------------------------------------- */
typedef struct PortalData *Portal;
typedef struct SPITupleTable { TupleDesc tupdesc; HeapTuple *vals; uint64 numvals; } SPITupleTable;
extern uint64 SPI_processed;
extern SPITupleTable *SPI_tuptable;
int SPI_connect(void);
int SPI_finish(void);
Portal SPI_cursor_open_with_args(const char *name, const char *src, int nargs, Oid *argtypes, Datum *Values,
                                 const char *Nulls, bool read_only, int cursorOptions);
void SPI_cursor_fetch(Portal portal, bool forward, long count);
void SPI_cursor_close(Portal portal);
Oid SPI_gettypeid(TupleDesc tupdesc, int fnumber);
Datum SPI_getbinval(HeapTuple tuple, TupleDesc tupdesc, int fnumber, bool *isnull);
void SPI_freetuptable(SPITupleTable *tuptable);

#ifdef __cplusplus
}
#endif
#endif
