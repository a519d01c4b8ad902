/*
 * packos_oracle.h — CPU ORACLE (test infrastructure only).
 *
 * A from-scratch plain-C restatement of the reference PackOS algorithms
 * (quickwritereader/PackOS, pure Go) used ONLY as the checker for the HIP
 * path: by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
 * The product (packos_amd / libpackos.so) never links or calls it.
 *
 * Parity pinning: every encoder/decoder here is checked against the byte-exact
 * golden vectors transcribed from the reference's own tests
 * (tests/golden/vectors.json, made by tests/golden/make_golden.py from
 * access/put_test.go, packable/pack_test.go, access/get_test.go,
 * access/seqget_test.go and README.md).  The reference is Go and no Go
 * toolchain exists here, so the reference itself cannot be executed.
 */
#ifndef PACKOS_ORACLE_H
#define PACKOS_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#include "../include/packos.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- typetags (typetags/types.go:44-63) ---- */
uint16_t or_encode_header(int64_t offset, int tag);
uint16_t or_encode_end(int64_t offset);

/* ---- PutAccess restatement (access/put.go) ---- */
typedef struct or_put {
    uint8_t* buf;  size_t len,  cap;    /* payload */
    uint8_t* offs; size_t olen, ocap;   /* header entries */
    int64_t position;
    int overflow;                       /* any EncodeHeader offset >= 8192 */
} or_put;

void   or_put_init(or_put* p);
void   or_put_free(or_put* p);
void   or_put_reset(or_put* p);
/* AppendTagAndValue / Add*: header EncodeHeader(position, tag), then bytes */
void   or_put_add(or_put* p, int tag, const uint8_t* bytes, size_t n);
/* AddNullable*(nil): header only */
void   or_put_add_nil(or_put* p, int tag);
/* BeginTuple/BeginMap: header in parent; child must be or_put_init'ed */
void   or_put_begin(or_put* parent, int tag);
/* EndNested: parent.buf = child.PackAppend(parent.buf) */
void   or_put_end(or_put* parent, or_put* child);
size_t or_put_pack_size(const or_put* p);            /* PackSize (put.go:655) */
/* Pack(): appends End, rewrites h0 (mutates p, Q4), writes out; returns size */
size_t or_put_pack(or_put* p, uint8_t* out);

/* ---- oracle schema nodes (pre-order, 4 int32 per node) ----
 * kind codes below; for containers b = number of children that follow.     */
enum {
    ORN_INT = 1,    /* a = width, b = nullable                    SInt8..64 */
    ORN_UINT = 2,   /* a = width, b = nullable                    (PutAccess AddUint*) */
    ORN_FLOAT = 3,  /* a = width, b = nullable                    SFloat32/64 */
    ORN_BOOL = 4,   /* a = 1,     b = nullable                    SBool */
    ORN_STRING = 5, /* a = SchemaString.Width (0 nullable, >0 exact, -1 optional) */
    ORN_BYTES = 6,  /* a = SchemaBytes.Width */
    ORN_MATCH = 7,  /* a = literal index, b = SchemaString Width (SString.Match / map key) */
    ORN_TUPLE = 8,  /* a = nullable, b = nchild, c = ORT_* flags */
    ORN_MAP = 9     /* a = sorted,   b = nchild (key,value,...) */
};
/* ORN_TUPLE c flags */
enum {
    ORT_VARIABLE = 1,      /* VariableLength: no arg-count check                */
    ORT_NAMED = 2,         /* TupleSchemaNamed: the check has no argCount > 0 guard */
    ORT_NAMES_BAD = 4      /* TupleSchemaNamed with len(FieldNames) != len(Schemas) */
};

typedef struct or_schema {
    const int32_t* nodes;     /* 4 ints per node, pre-order */
    int            n_nodes;
    int            n_top;     /* number of top-level nodes (chain length) */
    const uint8_t* lit;       /* literal pool */
    const int32_t* lit_off;   /* n_lit+1 offsets */
    /* derived by or_schema_prepare: */
    int            n_cols;    /* columns = every non-MATCH node, pre-order */
    int32_t        col_of_node[512];
    int32_t        next_sibling[512];
    int32_t        top_nodes[256];
    /* optional value checks, 4 int64 per node (NULL = none):
     *   [0] flags: 1 min, 2 max, 4 date (ErrDateOutOfRange), 8 prefix,
     *       16 suffix, 32 decodeDefault       (same bits as CHK_* in the product)
     *   [1] min  [2] max
     *   [3] (prefix/suffix literal index + 1) | (default literal index + 1) << 32 */
    const int64_t* ext;
    /* SchemaNamedChain (schema.go:943-946) whose len(FieldNames) differs from
     * len(Schemas): that FieldNames length, else 0.  EncodeValueNamed walks
     * FieldNames (schema.go:968-995): with fewer names only the first
     * chain_names schemas are encoded; with more, the walk indexes past
     * Schemas once the present fields are written (a Go panic).
     * DecodeBufferNamed fails every blob NewSeqGetAccess accepts
     * (schema.go:953-956).  ValidateBuffer takes the plain SchemaChain: no
     * change.                                                                */
    int            chain_names;
} or_schema;

int or_schema_prepare(or_schema* s);   /* 0 ok */

/* Encode blob i into out (cap bytes).  mode = PACKOS_MODE_PUTACCESS /
 * PACKOS_MODE_PACKABLE, optionally | PACKOS_MODE_EXTENDED (ADR-001 extended
 * containers: this build's format extension, include/packos.h).  Returns size or
 * -1 if cap too small.  *overflow set when a 13-bit truncation happened.     */
int64_t or_encode_one(const or_schema* s, const packos_column* cols, size_t i, int mode,
                      uint8_t* out, size_t cap, int* overflow);
/* Whole batch, host buffers; out_offsets n+1.  nthreads >= 1. Returns total
 * bytes or -1.                                                               */
int64_t or_encode_batch(const or_schema* s, const packos_column* cols, size_t n, int mode,
                        uint8_t* out, size_t cap, uint64_t* out_offsets, uint32_t* status,
                        int nthreads);
int64_t or_encoded_size_one(const or_schema* s, const packos_column* cols, size_t i, int mode);
/* total bytes of the batch; offs_scratch (n+1) receives per-blob sizes at [1..n] */
int64_t or_encoded_total(const or_schema* s, const packos_column* cols, size_t n, int mode, uint64_t* offs_scratch,
                         int nthreads);

/* schema.DecodeBuffer over a batch (host buffers).  offsets n+1 or NULL with
 * stride.  Returns 0.                                                        */
int or_decode_batch(const or_schema* s, const uint8_t* arena, const uint64_t* offsets,
                    uint64_t stride, size_t n, packos_column* out_cols, uint32_t* status,
                    int nthreads);
/* same, mode = PACKOS_MODE_EXTENDED reads ADR-001 extended containers */
int or_decode_batch_mode(const or_schema* s, const uint8_t* arena, const uint64_t* offsets,
                         uint64_t stride, size_t n, packos_column* out_cols, uint32_t* status,
                         int nthreads, int mode);
/* ValidateBuffer (schema/schema.go:880-891): status only, Validate rules */
int or_validate_batch(const or_schema* s, const uint8_t* arena, const uint64_t* offsets,
                      uint64_t stride, size_t n, uint32_t* status, int nthreads, int mode);

/* ---- SeqGetAccess restatement (access/seqget.go) ---- */
typedef struct or_seq {
    const uint8_t* buf; int64_t len;
    int64_t count, base, pos;
    int64_t next_off; int next_type;
    int64_t cur_off;  int cur_type;
    int xw;                            /* 1: ADR-001 extended container (u32 entries) */
} or_seq;
int or_seq_init(or_seq* s, const uint8_t* buf, int64_t len);          /* 0 ok */
/* extended container of kind xkind (4 tuple / 7 map), PACKOS_MODE_EXTENDED:
 * 02 00 | kind | u32 entries (include/packos.h); 0 ok                      */
int or_seq_init_ext(or_seq* s, const uint8_t* buf, int64_t len, int xkind);
int or_seq_peek(const or_seq* s, int* typ, int64_t* width);            /* 0 ok */
int or_seq_advance(or_seq* s);                                         /* 0 ok */
int or_seq_next(or_seq* s, int64_t* start, int64_t* width, int* typ);  /* 0 ok */
int or_seq_peek_nested(const or_seq* s, or_seq* nested);               /* 0 ok */

/* ---- GetAccess restatement (access/get.go) ---- */
typedef struct or_get {
    const uint8_t* buf; int64_t len; int64_t arg_count, base;
    int xw;      /* 1: an ADR-001 extended container (u32 entries after a 4-byte lead) */
    int xmode;   /* PACKOS_GET_EXTENDED: tag-2 fields open extended accessors */
} or_get;
int  or_get_init(or_get* g, const uint8_t* buf, int64_t len);          /* 0 = nil accessor */
void or_get_range(const or_get* g, int64_t pos, int* tp, int64_t* start, int64_t* end);
/* Get{Int,Uint,Float,Bool}XX semantics: tag and exact width; 0 ok, 1 error */
int  or_get_fixed(const or_get* g, int64_t pos, int tag, int width, int64_t* start);
/* GetNullable*: 0 ok, 1 error, 2 nil */
int  or_get_nullable(const or_get* g, int64_t pos, int tag, int width, int64_t* start);
/* GetBytes / GetString: 0 ok, 1 error */
int  or_get_span(const or_get* g, int64_t pos, int64_t* start, int64_t* end);
/* GetNestedGetAccess: 0 ok, 1 error, 2 nil */
int  or_get_nested(const or_get* g, int64_t pos, or_get* nested, int* tp);

/* ---- batch GetAccess gather, same contract as packos_get_field_batch ---- */
int or_get_field_batch(const uint8_t* arena, const uint64_t* offsets, uint64_t stride, size_t n,
                       const int32_t* path, int depth, int want_tag, int want_width,
                       uint64_t* out_start, uint32_t* out_len, uint8_t* out_tag, uint8_t* status);

/* ---- batch GetAccess getters, same contract as packos_get_batch ---- */
int or_get_batch(const uint8_t* arena, const uint64_t* offsets, uint64_t stride, size_t n,
                 const int32_t* path, int depth, int getter, int want_tag, int want_width,
                 uint8_t* out_values, uint32_t value_width, uint64_t* out_start, uint32_t* out_len,
                 uint8_t* out_tag, uint8_t* status);
int or_get_map_batch(const uint8_t* arena, const uint64_t* offsets, uint64_t stride, size_t n,
                     const int32_t* path, int depth, int flags, uint32_t max_pairs, uint32_t* out_pairs,
                     uint64_t* key_start, uint32_t* key_len, uint64_t* val_start, uint32_t* val_len,
                     uint8_t* val_tag, uint8_t* status);

/* splitmix64 stream (synthetic data generator shared with the Python side) */
uint64_t or_splitmix64(uint64_t* state);

#ifdef __cplusplus
}
#endif
#endif
