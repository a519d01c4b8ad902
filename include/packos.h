/*
 * packos.h — C ABI of the MI355X-native bulk PackOS encoder/decoder.
 *
 * One call encodes (or decodes) a whole batch of independent PackOS blobs that
 * share one fixed schema.  Everything is plain pointers and sizes: no HIP or
 * torch types cross this boundary, so a Go cgo shim, a C++
 * program or Python ctypes can bind it directly.
 *
 * Reference interfaces each entry point replaces (quickwritereader/PackOS):
 *   packos_schema_compile  <- schema.BuildSchema(*SchemaJSON)          schema/schemabuilder_json.go:124
 *                             + utils.SortKeys resolved once             utils/utils.go:7
 *   packos_encode_batch    <- access.PutAccess Add..., Pack()  (MODE_PUTACCESS)   access/put.go:69-308,619
 *                             schema.EncodeValue / EncodeValueNamed (MODE_PUTACCESS) schema/schema.go:912,968
 *                             packable.Pack(args...)        (MODE_PACKABLE)    packable/pack.go:59
 *   packos_encoded_size_batch <- PutAccess.PackSize / Tuple.ValueSize      access/put.go:655, packable/pack.go:17
 *   packos_decode_batch    <- schema.DecodeBuffer / DecodeBufferNamed
 *                             over access.SeqGetAccess                  schema/schema.go:893,948; access/seqget.go
 *   packos_validate_batch  <- schema.ValidateBuffer (the Validate methods'  schema/schema.go:880
 *                             rules, which differ from Decode's: see below)
 *   packos_get_field_batch <- access.GetAccess Get*(pos) / GetNestedGetAccess  access/get.go:19-375,492
 *   packos_get_batch          + GetInt / GetFloating / GetTypeAndValue      access/get.go:120-170,504-536
 *   packos_get_map_batch   <- GetMapStr / GetMapAny / GetMapOrderedAny       access/get.go:412-490
 *   packos_strerror        <- Go error strings (errors.New / SchemaError.Error)
 *
 * Conventions
 *   - All data pointers passed to the batch calls are DEVICE pointers (hipMalloc
 *     or torch CUDA tensors) unless stated otherwise; the caller owns every
 *     buffer.  Calls are asynchronous on the given stream (a hipStream_t passed
 *     as void*, NULL = default stream).
 *   - Return value: 0 on success, a negative PACKOS_E* code otherwise.  Per-blob
 *     outcomes go to the `status` array (see PACKOS_STATUS_ macros).
 *   - A compiled schema handle is immutable and may be shared across threads and
 *     devices.
 */
#ifndef PACKOS_H
#define PACKOS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PACKOS_ABI_VERSION 4   /* 4: packos_validate_* */

/* ---- return codes (library-level errors) -------------------------------- */
#define PACKOS_OK              0
#define PACKOS_E_INVALID      -1   /* bad argument */
#define PACKOS_E_SCHEMA       -2   /* schema JSON rejected (message via packos_last_error) */
#define PACKOS_E_UNSUPPORTED  -3   /* schema feature outside the compiled subset */
#define PACKOS_E_ALIGN        -4   /* a fixed-width column is not 16-byte aligned */
#define PACKOS_E_WORKSPACE    -5   /* workspace too small */
#define PACKOS_E_CAPACITY     -6   /* output arena smaller than the encoded batch */
#define PACKOS_E_HIP          -7   /* HIP runtime error (message via packos_last_error) */
#define PACKOS_E_NODEVICE     -8   /* no GPU visible */

/* ---- encode modes --------------------------------------------------------- */
/* PutAccess.Pack() / schema.EncodeValue bytes: no slack, empty nested
 * container written by BeginTuple/EndNested is the 2-byte blob 10 00.         */
#define PACKOS_MODE_PUTACCESS  0
/* packable.Pack(args...) bytes: buffer sized by ValueSize(), so every nil
 * nullable leaves its full width as zero slack after the End-marked payload
 * (access/direct_write_nullables.go:10-12, packable/packable_nullables.go:23);
 * PackTuple() with no args writes nothing (packable/pack.go:31).             */
#define PACKOS_MODE_PACKABLE   1
/* ADR-001 extended containers, OR-ed into either mode above at
 * packos_schema_compile.  A FORMAT EXTENSION beyond the reference: PackOS
 * reserves tag 2 (typetags.TypeExtendedTagContainer, typetags/types.go:11)
 * and names the ADR (README.md:34) but ships no code, test or wire format for
 * it, so this build defines one.  Every container whose payload fits 13 bits
 * (<= 8191 bytes) is written exactly as the reference writes it, so blobs
 * without a large container are byte-identical to the plain modes.  A
 * container whose payload exceeds 8191 bytes (the reference would truncate
 * its End offset, Q1) is written extended instead:
 *     u16  0x0002            EncodeHeader(0, TypeExtendedTagContainer)
 *     u16  tag               the container's own tag: 4 tuple (also the
 *                            top-level chain) / 7 map
 *     u32  e[0..n]           e[j] = off_j << 3 | tag_j — the 16-bit header
 *                            rules widened: e[0] off = header bytes
 *                            4 + 4(n+1), e[j] = field j's start relative to
 *                            the payload, e[n] = End = payload length
 *     payload
 * and the parent entry of a field holding an extended container carries
 * tag 2.  Offsets reach 2^29 - 1 (512 MiB).  The decoders of a schema
 * compiled with this bit read such blobs (a top-level blob starting 02 00 is
 * extended; a tag-2 field must be an extended container of the schema's
 * kind, else ErrInvalidFormat).  Encode status never carries
 * PACKOS_STATUS_OVERFLOW13 in this mode.  Packable slack (Q2) still follows
 * the top-level payload.                                                     */
#define PACKOS_MODE_EXTENDED   0x100

/* ---- PackOS type tags (typetags/types.go:6-20) ---------------------------- */
#define PACKOS_TAG_END      0
#define PACKOS_TAG_INTEGER  1
#define PACKOS_TAG_EXTENDED 2
#define PACKOS_TAG_FLOATING 3
#define PACKOS_TAG_TUPLE    4
#define PACKOS_TAG_BOOL     5
#define PACKOS_TAG_STRING   6
#define PACKOS_TAG_MAP      7

/* ---- leaf (column) kinds -------------------------------------------------- */
#define PACKOS_KIND_INT     1   /* int8/16/32/64  (tag Integer)  */
#define PACKOS_KIND_UINT    2   /* uint8/16/32/64 (tag Integer)  */
#define PACKOS_KIND_FLOAT   3   /* float32/64 raw bits (tag Floating) */
#define PACKOS_KIND_BOOL    4   /* one byte, any non-zero input encodes as 1 */
#define PACKOS_KIND_STRING  5   /* tag String */
#define PACKOS_KIND_BYTES   6   /* tag String (ByteArray) */
#define PACKOS_KIND_TUPLE   7   /* nested tuple: column carries only `valid` */
#define PACKOS_KIND_MAP     8   /* nested map:   column carries only `valid` */

/* ---- per-blob status word -------------------------------------------------
 * bits 0..7   schema ErrorCode of the error DecodeBuffer (packos_decode_batch)
 *             or ValidateBuffer (packos_validate_batch) would return
 *             (schema/schema.go:24-41); 0 = ok
 * bits 8..23  top-level field position of that error + 1 (0 = position -1)
 * bits 24..29 encode only: the ErrorCode of the leaf error that EncodeValue
 *             wraps in ErrEncode (schema.go:919-936), e.g. ErrOutOfRange for
 *             a Range violation; bits 0..7 then hold PACKOS_ERR_ENCODE and
 *             bits 8..23 are 0 (position -1, as the wrapping SchemaError)
 * bit 30      the reference would panic (Go runtime index out of range) on
 *             this blob, e.g. a nullable int16 field of width 1
 * bit 31      encode: an offset >= 8192 was truncated to 13 bits exactly as
 *             typetags.EncodeHeader does (Q1); the bytes still match the
 *             reference, the flag only reports it
 */
#define PACKOS_STATUS_CODE(s)      ((int)((s) & 0xFFu))
#define PACKOS_STATUS_POS(s)       ((int)(((s) >> 8) & 0xFFFFu) - 1)
#define PACKOS_STATUS_INNER(s)     ((int)(((s) >> 24) & 0x3Fu))
#define PACKOS_STATUS_PANIC        0x40000000u
#define PACKOS_STATUS_OVERFLOW13   0x80000000u

/* schema.ErrorCode values (schema/schema.go:24-41) */
#define PACKOS_ERR_INVALID_FORMAT        1
#define PACKOS_ERR_UNEXPECTED_EOF        2
#define PACKOS_ERR_CONSTRAINT_VIOLATED   3
#define PACKOS_ERR_ENCODE                4
#define PACKOS_ERR_STRING_PREFIX         6
#define PACKOS_ERR_STRING_SUFFIX         7
#define PACKOS_ERR_STRING_MATCH          9
#define PACKOS_ERR_OUT_OF_RANGE         13
#define PACKOS_ERR_DATE_OUT_OF_RANGE    14

/* decode view of a string leaf with a decodeDefault whose payload was empty:
 * start = PACKOS_VIEW_DEFAULT, length = the default's length; the bytes are
 * the schema's literal (packos_schema_column_default), as the reference
 * returns DefaultDecodeVal instead of "" (schema/schema.go:279-286)          */
#define PACKOS_VIEW_DEFAULT  0x8000000000000000ull

/* ---- columns ---------------------------------------------------------------
 * One packos_column per schema node in depth-first (pre-order) schema order:
 * every leaf and every nested tuple/map has a column; map-key literals
 * ("exact" strings) are compile-time constants and have none.  A tuple/map
 * column only uses `valid` (nil container = header with zero width, the
 * AddAnyTuple(nil)/AddMapAny(nil) form, access/put.go:343-352,547-553).
 *
 *   fixed-width leaf : data = n*width bytes, row i at data + i*width
 *                      (16-byte aligned base; little-endian scalars)
 *   var-width leaf   : encode input: data = byte arena, offsets = n+1 uint32
 *                      (row i = data[offsets[i] .. offsets[i+1])); or
 *                      offsets64 = n+1 uint64 for arenas past 4 GiB (when
 *                      offsets64 is set it is used and offsets is ignored;
 *                      one value must stay below 4 GiB)
 *                      decode output: start[i] = absolute arena offset of the
 *                      payload, length[i] = its width (the payload aliases the
 *                      input arena, like GetBytes/GetStringUnsafe,
 *                      access/get.go:335-375)
 *   nullable leaf    : valid = n bytes, 1 = value present, 0 = nil
 *                      (encode input; decode output).  NULL on encode = all
 *                      present.
 */
typedef struct packos_column {
    void*           data;
    const uint32_t* offsets;
    uint8_t*        valid;
    uint64_t*       start;
    uint32_t*       length;
    const uint64_t* offsets64;   /* ABI 2: 64-bit var offsets (encode input), NULL = use offsets */
} packos_column;

typedef struct packos_column_info {
    int32_t kind;       /* PACKOS_KIND_* */
    int32_t width;      /* fixed byte width, 0 = variable */
    int32_t nullable;   /* 1 = has a validity column */
    int32_t tag;        /* PACKOS_TAG_* written in its header */
    int32_t top_index;  /* index of the top-level field this leaf belongs to */
    int32_t depth;      /* 0 = top-level field */
    char    name[96];   /* dotted path of fieldNames ("" when unnamed) */
} packos_column_info;

typedef struct packos_schema packos_schema;

/* ---- schema compiler (host only, no GPU needed) -------------------------- */

/* Compile a schema given in the SchemaJSON vocabulary
 * (schema/schemabuilder_json.go:8-30).  Accepted top level: a JSON array
 * (SChain) or {"type":"chain","schema":[...],"fieldNames":[...]}
 * (SchemaNamedChain).  Supported node types: bool, int8..int64,
 * uint8..uint64, float32, float64, string (width / nullable / exact),
 * bytes (width), tuple (schema, fieldNames, nullable, variableLength),
 * map (schema = key,value,... ; keys with "exact" become constants; an
 * odd schema count compiles: a present value then fails encode and decode
 * with ErrConstraintViolated (schema.go:369-377, 422-429), as SMap does;
 * "sorted": true sorts the pairs by key bytes at compile time, which is
 * PackMapSorted / AddMapSortedKey order).
 * Value checks, as BuildSchema builds them:
 *   int16/32/64 "min"/"max"   -> SInt*.Range: never nullable, ErrOutOfRange
 *                                (schema.go:1172-1364); int8 ignores them
 *   "date" (dateFrom/dateTo   -> SDateRange: int64 payload, nullable per
 *   RFC3339, both or neither)    "nullable", ErrDateOutOfRange (:2188-2250)
 *   string "decodeDefault"    -> an empty payload decodes as the literal
 *   string "prefix"/"suffix"  -> HasPrefix / HasSuffix, ErrStringPrefix /
 *                                ErrStringSuffix on decode, ErrEncode on
 *                                encode (:1070-1158; exact > prefix > suffix)
 * Encode reports a failing check in the blob's status (bits 24..29 =
 * the leaf's ErrorCode); the blob's bytes are then not a reference output.
 * Tuples are always nullable (every STuple* constructor; a "nullable" key is
 * ignored, schemabuilder_json.go:244-260).
 * Extensions beyond SchemaJSON (documented, not in the reference's
 * vocabulary): uint8..uint64 (PutAccess AddUint*) and "sorted" maps.       */
int  packos_schema_compile(const char* schema_json, int mode, packos_schema** out);
void packos_schema_free(packos_schema* s);
int  packos_schema_num_columns(const packos_schema* s);
int  packos_schema_num_top_fields(const packos_schema* s);
int  packos_schema_column_info(const packos_schema* s, int col, packos_column_info* out);
/* Blob size in bytes when the schema has no variable-width leaf and a call
 * passes no validity columns (every nullable present), else -1 (also -1 in
 * extended mode when that size exceeds 8191: blobs may be extended).       */
int64_t packos_schema_fixed_blob_size(const packos_schema* s);
/* Extended mode: the most bytes extended header blocks can add to one blob
 * (sum over containers with fields of 4 + 2(n+1)); 0 for the plain modes.
 * Host arenas sized n * (static size + this) + all var bytes always fit.    */
int64_t packos_schema_ext_overhead(const packos_schema* s);
/* 1 when packos_decode_batch can use the tiled fixed-layout decoder for this
 * schema (fixed size B, B % 4 == 0, B <= 1024, and the all-present blob
 * decodes cleanly), else 0.  Decided at compile time, without a GPU; results
 * never depend on it (non-canonical blobs fall back to the exact decoder).  */
int  packos_schema_decode_fast(const packos_schema* s);
/* 1 when the schema has encode-time value checks (int "min"/"max", "date",
 * string "prefix"/"suffix"): packos_encode_batch / packos_encode_host_batch
 * then require a status array, since a failing value makes EncodeValue return
 * ErrEncode (schema/schema.go:919-936), which only the status can report.  */
int  packos_schema_has_checks(const packos_schema* s);
/* decodeDefault literal of column `col` (a string leaf): copies at most cap
 * bytes into buf and returns the literal's length (0 = no default, -1 = bad
 * column).                                                                  */
int64_t packos_schema_column_default(const packos_schema* s, int col, char* buf, size_t cap);
/* Host-side dump of the compiled layout program (debug/testing). Returns the
 * number of bytes needed (including NUL); writes at most cap bytes.          */
size_t packos_schema_describe(const packos_schema* s, char* buf, size_t cap);
/* Host-side encoded size of one blob given its var widths / valid flags,
 * without a GPU (used by shard planning).  widths[c] is read for var
 * columns, valid[c] for nullable columns (may be NULL).                      */
int64_t packos_schema_blob_size_host(const packos_schema* s, const uint32_t* widths,
                                     const uint8_t* valid);

/* ---- batch encode ---------------------------------------------------------- */

/* Device scratch a variable-size batch of n blobs may need: the look-back
 * words of the size pass when blob sizes depend on nil values.  Batches whose
 * presence is data-independent (no nil container / nullable value in the
 * call) need none: their out_offsets have a closed form.  Fixed-size batches
 * need none. */
size_t packos_encode_workspace_size(const packos_schema* s, size_t n_blobs);

/* Size pass + exclusive scan: out_offsets[0..n] (device, uint64).  Fixed-size
 * schemas write i*B without reading columns.                                 */
int packos_encoded_size_batch(const packos_schema* s, const packos_column* cols, size_t n_blobs,
                              uint64_t* out_offsets, void* workspace, size_t workspace_bytes,
                              void* stream);

/* Encode n blobs into out_arena.  For a variable-size schema out_offsets
 * (n+1, device) receives each blob's start (computed in the encode kernel
 * itself when no presence depends on the data, else by a size pass first);
 * pass flags PACKOS_ENC_OFFSETS_READY when out_offsets already holds the
 * layout to encode into (e.g. from packos_encoded_size_batch).  For a fixed-size schema out_offsets may be NULL (blob i
 * is at i*B).  status (n, device) may be NULL unless the schema has value
 * checks (packos_schema_has_checks; PACKOS_E_INVALID then).  out_capacity is checked only
 * when offsets are known on the host side (fixed schemas); for variable
 * schemas blobs that would end past out_capacity are not written and get
 * PACKOS_ERR_ENCODE in their status.  Var-width column offsets must be
 * non-decreasing over all n+1 entries (also for rows inside nil containers).
 * Offsets that do not match the schema's sizes (a caller-made layout with
 * gaps) are honoured: such blobs take a per-blob path and gap bytes are
 * never written.                                                             */
#define PACKOS_ENC_OFFSETS_READY 1u
/* testing/benchmark knob: fixed-size batches use the general 4-blob-period
 * kernel even when the lane-invariant one applies; variable-size batches use
 * the generic one-wavefront-per-blob kernel instead of the tiled one         */
#define PACKOS_ENC_FORCE_GENERIC 2u
/* out_capacity is the batch's exact encoded size (e.g. out_offsets[n] of
 * packos_encoded_size_batch): the library takes out_capacity / n as the mean
 * blob size when it picks the kernel for a flat chain of leaves with every
 * value present.  Without it, a batch whose capacity admits >= 256 bytes per
 * blob launches both candidate kernels and each decides on the device from
 * the var columns' first and last offsets (no host read-back: every call
 * stays asynchronous on `stream` and can be captured in a HIP graph).
 * Results never depend on the choice.                                        */
#define PACKOS_ENC_CAP_EXACT 4u
/* out_offsets (n+1, device) already hold packos_encoded_size_batch's result
 * for these same columns: the library does not run the size pass again.  A
 * closed-form layout (no presence depending on the data) is recomputed by the
 * encoder itself (the same offsets, rewritten), so its fast kernels stay
 * eligible; other layouts are encoded into the given offsets as with
 * PACKOS_ENC_OFFSETS_READY.                                                  */
#define PACKOS_ENC_SIZED 8u
/* testing/benchmark knob: pick the fixed-layout kernel variant (0 = auto):
 * 13 one tile per workgroup, LDS-DMA staging, single-source dwords (auto
 *    when B % 4 == 0, 16 <= B <= 1024, <= 16 fixed columns);
 * 2  lane-invariant dword kernel (auto otherwise when B % 4 == 0; also the
 *    partial last tile of variant 13);
 * 8  general 4-blob-period kernel (any B)                                    */
#define PACKOS_ENC_FIXED_VARIANT(v) (((uint32_t)(v) & 0xFu) << 4)
int packos_encode_batch(const packos_schema* s, const packos_column* cols, size_t n_blobs,
                        uint8_t* out_arena, uint64_t out_capacity, uint64_t* out_offsets,
                        uint32_t* status, void* workspace, size_t workspace_bytes,
                        uint32_t flags, void* stream);

/* ---- host-resident batches ------------------------------------------------ */

/* A host pipeline: the device buffers, three HIP streams (H2D, kernels, D2H)
 * and events of a chunked host <-> device loop, bound to the device current
 * at creation and kept across calls (buffers grow on demand, never shrink),
 * so a steady stream of host batches pays no allocation.  Chunk k's H2D runs
 * while chunk k-1's kernels and chunk k-2's D2H run: both PCIe directions
 * busy at once.  `slots` (>= 2; 0 = 3) chunks are in flight; chunk_blobs 0 =
 * 131072.  One call at a time per pipeline (calls serialise on its lock);
 * the schema must outlive it.  packos_encode_host_batch /
 * packos_decode_host_batch use a pipeline cached on the schema handle.     */
typedef struct packos_pipeline packos_pipeline;
int  packos_pipeline_create(const packos_schema* s, size_t chunk_blobs, int slots, packos_pipeline** out);
void packos_pipeline_free(packos_pipeline* p);
/* packos_encode_host_batch / packos_decode_host_batch /
 * packos_validate_host_batch on an explicit pipeline (same arguments and
 * results; chunking from the pipeline)                                      */
int  packos_pipeline_encode(packos_pipeline* p, const packos_column* host_cols, size_t n_blobs, uint8_t* host_out,
                            uint64_t out_capacity, uint64_t* host_offsets, uint32_t* host_status);
int  packos_pipeline_decode(packos_pipeline* p, const uint8_t* host_arena, const uint64_t* host_offsets,
                            uint64_t stride, size_t n_blobs, packos_column* host_cols, uint32_t* host_status);
int  packos_pipeline_validate(packos_pipeline* p, const uint8_t* host_arena, const uint64_t* host_offsets,
                              uint64_t stride, size_t n_blobs, uint32_t* host_status);

/* Encode n blobs whose columns live in HOST memory into a host arena — the
 * entry point a cgo / JNI shim calls for RPC payloads or BadgerDB values
 * (PackAppend / Pack per blob, access/put.go:619-681, for a whole batch).
 * Chunks of `chunk_blobs` blobs (0 = 131072) move through the schema's
 * cached pipeline on the current device (packos_pipeline_create): H2D of
 * chunk k, the encode kernel(s) of chunk k-1 and D2H of chunk k-2 run at
 * once.  Var columns go over as they are (data bytes + offsets of either
 * width, no host rebasing).  Pinned host buffers (hipHostMalloc / hipHostRegister)
 * make the copies asynchronous; pageable ones work too.  host_cols use the
 * same layout as packos_encode_batch's device columns.  host_offsets (n+1)
 * receives the blob starts (required for variable-size batches); host_status
 * (n) may be NULL.  Blocks until done.  Returns PACKOS_E_CAPACITY when the
 * output exceeds out_capacity (n * static size + all var bytes always fits). */
int packos_encode_host_batch(const packos_schema* s, const packos_column* host_cols, size_t n_blobs,
                             uint8_t* host_out, uint64_t out_capacity, uint64_t* host_offsets,
                             uint32_t* host_status, size_t chunk_blobs);

/* Decode n blobs of a HOST arena into HOST columns — the read side of the
 * cgo shim (BadgerDB values, RPC payloads: DecodeBuffer per blob,
 * schema/schema.go:893).  Blob i = host_arena[host_offsets[i] ..
 * host_offsets[i+1]) or, with host_offsets NULL, the `stride`-byte slot i.
 * Chunks of `chunk_blobs` blobs (0 = 131072) go H2D (their offsets and the
 * arena bytes between the chunk's smallest and largest offset), through
 * packos_decode_batch, and D2H, pipelined like the encode side.  Offsets need
 * not be monotone (a blob whose end precedes its start fails to decode).
 * host_cols use packos_decode_batch's layout in host memory; var views are
 * absolute host_arena offsets (or PACKOS_VIEW_DEFAULT); validity is written
 * for nullable leaves and containers; rows the decoder does not write (nil
 * values, leaves inside nil containers) read as zero data and views and 0xFF
 * validity.  host_status (n) is required.  Pinned
 * buffers make the copies asynchronous.  Blocks until done.                  */
int packos_decode_host_batch(const packos_schema* s, const uint8_t* host_arena, const uint64_t* host_offsets,
                             uint64_t stride, size_t n_blobs, packos_column* host_cols, uint32_t* host_status,
                             size_t chunk_blobs);

/* ValidateBuffer over a HOST arena (schema/schema.go:880-891): chunks go H2D
 * like packos_decode_host_batch, through packos_validate_batch, and only the
 * status comes back.  host_status (n) is required.  Blocks until done.     */
int packos_validate_host_batch(const packos_schema* s, const uint8_t* host_arena, const uint64_t* host_offsets,
                               uint64_t stride, size_t n_blobs, uint32_t* host_status, size_t chunk_blobs);

/* ---- batch decode (schema.DecodeBuffer semantics) ------------------------- */

/* blob i = arena[offsets[i] .. offsets[i+1]); offsets == NULL means fixed
 * stride `stride` bytes.  Every blob is validated with SeqGetAccess/precheck
 * rules; status[i] gets the error DecodeBuffer would return.  Columns of a
 * failing blob are left unspecified.                                         */
int packos_decode_batch(const packos_schema* s, const uint8_t* arena, const uint64_t* offsets,
                        uint64_t stride, size_t n_blobs, packos_column* out_cols,
                        uint32_t* status, void* stream);

/* ---- batch validate (schema.ValidateBuffer semantics) --------------------- */

/* status[i] = the error ValidateBuffer(blob i, chain) would return, in the
 * status-word layout above (a ValidateBuffer panic sets bit 30).  No columns.
 * ValidateBuffer runs each schema's Validate method, whose rules differ from
 * Decode's (packos_decode_batch) in three places of the compiled subset:
 *   - a nullable bool / int / uint / float leaf never reads its payload
 *     (validatePrimitive, schema.go:596-715): a payload shorter than the type
 *     passes, where Decode panics; Range / date leaves read it either way
 *     (:1177-1188, :2198-2212)
 *   - a prefix / suffix / exact string check of a nullable string (width <= 0)
 *     passes an empty value (after the decodeDefault substitution) without
 *     testing it (CheckFunc ValidateFunc, :1085-1087); Decode tests it
 *   - a map with an odd schema count validates its schemas in sequence
 *     (SchemaMap.Validate, :336-359); Decode fails ErrConstraintViolated
 * A blob DecodeBuffer accepts is always accepted here.  blob i =
 * arena[offsets[i] .. offsets[i+1]) or the `stride`-byte slot i.           */
int packos_validate_batch(const packos_schema* s, const uint8_t* arena, const uint64_t* offsets,
                          uint64_t stride, size_t n_blobs, uint32_t* status, void* stream);

/* ---- random-access gather (GetAccess semantics) --------------------------- */

/* For each blob walk `depth` (<= 16) positions (GetNestedGetAccess for all
 * but the last) and read the field at the last position.  `path` is HOST
 * memory (copied into the launch); the outputs are device arrays:
 *   out_start[i]/out_len[i] = absolute [start,end) of the field payload,
 *   out_tag[i]  = its tag,
 *   status[i]   = 0 ok, 1 decode error (the Get* call would return an error
 *                 for `want_tag`/`want_width`), 2 nil nested access (empty
 *                 container), 3 nil accessor (NewGetAccess returned nil: the
 *                 reference would dereference nil and panic).
 * want_width < 0 accepts any width >= 0 (GetBytes/GetString);
 * want_width == 0 is not used.                                               */
int packos_get_field_batch(const uint8_t* arena, const uint64_t* offsets, uint64_t stride,
                           size_t n_blobs, const int32_t* path, int depth, int want_tag,
                           int want_width, uint64_t* out_start, uint32_t* out_len,
                           uint8_t* out_tag, uint8_t* status, void* stream);

/* General GetAccess getter over every blob (walk `depth` positions like
 * packos_get_field_batch, then apply one Get* family to the last position):
 *   PACKOS_GET_FIXED     Get{Bool,Int8..64,Uint8..64,Float32/64}: tag ==
 *                        want_tag and width == want_width (access/get.go:60-66,
 *                        :80-94, :173-226, :287-305)
 *   PACKOS_GET_NULLABLE  GetNullable*: width 0 -> status 4 (nil, no error),
 *                        checked BEFORE the tag; otherwise as FIXED
 *                        (access/get.go:68-78, :96-118, :214-284, :307-333)
 *   PACKOS_GET_SPAN      GetBytes / GetString(Unsafe): tag == want_tag and
 *                        end >= start (access/get.go:335-375)
 *   PACKOS_GET_INT       GetInt: tag Integer (checked first), width 0 -> nil,
 *                        1/2/4/8 -> int8..int64 (access/get.go:120-146)
 *   PACKOS_GET_FLOAT     GetFloating: tag Floating, width 0 -> nil, 4/8
 *                        (access/get.go:148-170)
 *   PACKOS_GET_ANY       GetTypeAndValue / GetAsPackable: any tag, end >=
 *                        start, else status 1 (the reference returns
 *                        TypeInvalid and a nil value); a position past the
 *                        field count is status 3 (rangeAt's (-2, -1) slices
 *                        buf[-2:-1]: a Go panic) (access/get.go:38-45,
 *                        504-536); out_tag is the header's tag either way
 * Typed gather: when out_values is not NULL, row i of out_values
 * (value_width bytes) receives the value of a successful FIXED / NULLABLE
 * getter (its LE bytes; a Bool as 0/1), or for INT the integer sign-extended
 * to int64, for FLOAT the raw bits (a float32 in the low 4 bytes); zero
 * otherwise.  value_width: want_width for FIXED / NULLABLE, 8 for INT / FLOAT.
 * With a typed gather, out_start / out_len / out_tag may each be NULL (not
 * written): Get<T> / GetInt / GetFloating return only (value, error); SPAN
 * and ANY need all three.
 * status: 0 ok, 1 decode error, 2 nil nested accessor (empty container on
 * the path), 3 the reference panics (NewGetAccess returned nil and is
 * dereferenced, or GET_ANY past the field count), 4 nil value.              */
#define PACKOS_GET_FIXED     0
#define PACKOS_GET_NULLABLE  1
#define PACKOS_GET_SPAN      2
#define PACKOS_GET_INT       3
#define PACKOS_GET_FLOAT     4
#define PACKOS_GET_ANY       5
/* OR-ed into `getter`: read ADR-001 extended containers (PACKOS_MODE_EXTENDED
 * blobs): a blob starting 02 00 is an extended top-level chain, a tag-2 field
 * on the path an extended tuple / map (malformed -> status 1); the final
 * field's tag is reported as written (2 for an extended container)        */
#define PACKOS_GET_EXTENDED  0x100
int packos_get_batch(const uint8_t* arena, const uint64_t* offsets, uint64_t stride, size_t n_blobs,
                     const int32_t* path, int depth, int getter, int want_tag, int want_width,
                     uint8_t* out_values, uint32_t value_width, uint64_t* out_start, uint32_t* out_len,
                     uint8_t* out_tag, uint8_t* status, void* stream);

/* Map walk over every blob: walk `depth` - 1 positions like packos_get_batch,
 * then read the map at the last position as the reference's
 *   PACKOS_MAP_STR  GetMapStr        (access/get.go:464-490): every key and
 *                   every value must pass GetString (tag String, end >= start)
 *   PACKOS_MAP_ANY  GetMapAny / GetMapOrderedAny (get.go:412-462): keys pass
 *                   GetString; values pass GetAny (get.go:377-410): Integer ->
 *                   GetInt (width 0 = nil, 1/2/4/8), Floating -> GetFloating
 *                   (0 = nil, 4/8), String -> GetString, Map -> GetMapAny
 *                   recursively (validated to any depth up to 32 levels),
 *                   every other tag (End, Tuple, Bool, ...) an error
 * (OR PACKOS_GET_EXTENDED in to read ADR-001 extended containers).  Pair j of
 * blob i (in wire order) lands in row i * max_pairs + j of key_start/key_len
 * (absolute arena offsets of the key bytes) and val_start/val_len/val_tag
 * (the value's payload span and tag; a nested map value's span is its whole
 * container, to be read with a longer path); out_pairs[i] = the map's pair
 * count.  Wire order is what GetMapOrderedAny keeps; building a Go map from
 * the pairs in order reproduces GetMapStr / GetMapAny (a later duplicate key
 * overwrites an earlier one).
 * status: 0 ok, 1 decode error (the call returns an error), 2 nil nested
 * accessor on the path, 3 nil accessor (the reference dereferences nil:
 * panic), 4 nil map (empty payload: the call returns nil, nil), 5 ok but
 * more than max_pairs pairs (the first max_pairs are written), 6 nested maps
 * deeper than 32 levels (a limit of this implementation).                   */
#define PACKOS_MAP_STR 0
#define PACKOS_MAP_ANY 1
int packos_get_map_batch(const uint8_t* arena, const uint64_t* offsets, uint64_t stride, size_t n_blobs,
                         const int32_t* path, int depth, int flags, uint32_t max_pairs, uint32_t* out_pairs,
                         uint64_t* key_start, uint32_t* key_len, uint64_t* val_start, uint32_t* val_len,
                         uint8_t* val_tag, uint8_t* status, void* stream);

/* ---- misc ------------------------------------------------------------------ */
const char* packos_strerror(int code);
const char* packos_last_error(void);   /* thread-local detail of the last failure */
int         packos_abi_version(void);
/* Diagnostics: the encode kernel the last packos_encode_batch call of this
 * thread launched ("fixed_tile", "fixed_dw", "fixed", "var", "ext", "flat",
 * "tiles", "tiles6" = the tile encoder at six workgroups per CU; "" before
 * any call and after a call that launched none).  No reference counterpart; tests use it to
 * assert which encoder a batch exercised.                                      */
const char* packos_last_encoder(void);

#ifdef __cplusplus
}
#endif
#endif /* PACKOS_H */
