// program.h — compiled schema programs shared by the host compiler
// (compile.cpp) and the HIP kernels (kernels.hip).  Plain POD structs.
#pragma once
#include <stdint.h>

namespace packos {

constexpr int kMaxCols = 64;      // columns per schema (kernel-argument tables)
constexpr int kMaxDepth = 16;     // nesting depth supported by the decoders
constexpr int kMaxConts = 64;     // containers per schema (bitmask in the encoder)

enum NodeKind : int32_t {
    K_INT = 1, K_UINT = 2, K_FLOAT = 3, K_BOOL = 4, K_STRING = 5, K_BYTES = 6,
    K_MATCH = 7, K_TUPLE = 8, K_MAP = 9, K_ROOT = 10
};

// Value checks of a leaf (schema-level constraints on top of the wire format).
enum : uint32_t {
    CHK_MIN = 1u,        // int value >= rmin        (SInt*.Range / SDateRange)
    CHK_MAX = 2u,        // int value <= rmax
    CHK_DATE = 4u,       // range error is ErrDateOutOfRange, not ErrOutOfRange
    CHK_PREFIX = 8u,     // strings.HasPrefix(value, lit)   -> ErrStringPrefix
    CHK_SUFFIX = 16u,    // strings.HasSuffix(value, lit)   -> ErrStringSuffix
    CHK_DEFAULT = 32u,   // empty payload decodes as the default literal
    CHK_FAIL = 64u,      // encode check only: fails whenever its container is present
                         // (TupleSchemaNamed names / schemas length mismatch, schema.go:1808-1810)
    CHK_PANIC = 128u,    // encode check only, last in emission order: every blob that passed the
                         // checks before it panics (EncodeValueNamed indexing past Schemas once
                         // it has written them all, schema.go:976-987)
    CHK_RANGE = CHK_MIN | CHK_MAX,
    CHK_STR = CHK_PREFIX | CHK_SUFFIX,
};

// One encode-time value check (EncodeFunc of Range / SDateRange / CheckFunc),
// evaluated per blob by k_encode_checks after the encode kernel.
struct EncCheck {
    int32_t col;         // leaf column
    int32_t cont;        // container whose presence gates the value
    int32_t top;         // top-level field index (status position)
    uint32_t flags;      // CHK_*
    uint32_t width;      // int width (range) / fixed string width (0 = var)
    uint32_t lit, lit_len;
    uint32_t inner;      // schema ErrorCode of the leaf's own error
    int64_t rmin, rmax;
};

// ---------------------------------------------------------------- encode ----
// Items are the byte runs of one blob in wire order.  Positions are the
// exclusive prefix sum of item sizes; header words are differences of
// positions (the h0 / End / relative-offset rules of access/put.go:619-652
// and packable/pack.go:30-57).
enum : uint8_t { IT_HDR = 0, IT_FIXED = 1, IT_VAR = 2, IT_CONST = 3 };

struct EncItem {
    uint8_t type;      // IT_*
    uint8_t nullable;  // fixed leaf with a validity column
    uint8_t is_bool;   // normalise any non-zero input byte to 1
    uint8_t vslot;     // IT_VAR: index among the var items
    int16_t cont;      // container whose presence gates this item
    int16_t col;       // leaf column (IT_FIXED / IT_VAR), -1 otherwise
    uint32_t size;     // fixed width / literal length / header-block bytes
    uint32_t lit;      // literal offset (IT_CONST)
    uint32_t magic;    // ceil(2^32 / size) when size > 1 (division by size)
    uint8_t reg;       // IT_FIXED: index among the fixed items (staging region), 255 otherwise
    uint8_t pad[3];
};

struct EncHdr {            // one uint16 header word
    uint16_t hdr_item;     // the container's IT_HDR item
    uint16_t target;       // item whose position the offset points to
    uint16_t cont;         // container id (gates the write)
    uint8_t tag;
    uint8_t relative;      // 0 = constant `value`, 1 = pos(target) - payload start
    uint16_t j;            // index within the header block
    uint16_t value;        // constant word (h0, or 0x0010 for an empty nested block)
    uint16_t ovf;          // constant word overflowed 13 bits
    uint16_t child;        // container id + 1 of the field this entry starts (0: a leaf / End);
                           // extended mode: its tag becomes 2 when that container is extended
};

struct EncCont {
    int16_t parent;        // -1 for the root (the chain itself)
    int16_t valid_col;     // column holding the nil flag, -1 if never nil
    uint16_t hdr_item;
    uint16_t n_kids;
    uint16_t end_item;     // items of the container's payload: (hdr_item, end_item)
    uint8_t tag;           // its own tag: Tuple 4 (also the root chain) / Map 7
    uint8_t pad;
};

// ADR-001 extended containers (PACKOS_MODE_EXTENDED, include/packos.h): a
// container whose payload exceeds 8191 bytes (its End offset would be cut to
// 13 bits by EncodeHeader, typetags/types.go:44-46) is written as
//   u16 EncodeHeader(0, TypeExtendedTagContainer) = 0x0002 | u16 own tag |
//   u32 entries e[0..n] (off << 3 | tag, the 16-bit rules widened; e[0] off =
//   header bytes 4 + 4(n+1), e[n] = End) | payload
// and the parent entry of such a field carries tag 2.
constexpr uint32_t kExtMaxPayload = 8191;
constexpr uint32_t kExtMarker = 0x0002;
constexpr uint32_t ext_hdr_bytes(uint32_t n_kids) { return 4u + 4u * (n_kids + 1u); }

struct EncProgram {
    const EncItem* items;
    const EncHdr* hdrs;
    const EncCont* conts;
    const uint8_t* lits;
    int32_t n_items, n_hdrs, n_conts, mode;
    int32_t n_lits;
    int32_t ext;           // PACKOS_MODE_EXTENDED
    const uint32_t* ipk;   // per item: bits 0-15 static size, 16-23 var slot (255 = not var)
    const uint32_t* ihr;   // per item: IT_HDR -> first header entry | count << 16
};

// Fixed-size layout (no var-width leaves, no nils in the call): every blob is
// B bytes and byte q of a blob is either a constant or byte `off` of a fixed
// column row.  The kernel works on tiles of T blobs; for each dword r of a
// 4-blob period (4B bytes = B dwords) a short list of segments says where its
// bytes come from in the LDS-staged input tile.
struct FixSeg {
    int32_t a;          // LDS byte address of dword byte 0 for the period's blob 0
    uint32_t stride4;   // LDS bytes between periods (4 * column width); 0 = constant
    uint32_t mask;      // byte-lane mask of this segment within the dword
    uint32_t cval;      // constant bytes (stride4 == 0) or flags (bit0: bool normalise)
};

struct FixCol {
    int32_t col;         // column index
    uint32_t width;      // row width in bytes
    uint32_t lds_off;    // LDS offset of this column's tile region
    uint32_t chunk_begin;// first 16-byte chunk of this column within the tile
    uint32_t flags;      // bit0: bool column (any non-zero byte encodes as 1)
};

// Lane-invariant form (B % 4 == 0): thread t always builds output dword
// q = t % (B/4) of successive blobs, so its (at most 4) byte sources live in
// registers for the whole tile.
struct DwSeg {
    int32_t a;        // LDS byte address of dword byte 0 for tile blob 0
    uint32_t w;       // LDS bytes between consecutive blobs (column width)
    uint32_t mask;    // byte-lane mask
    uint32_t flags;   // bit0: bool normalise
};
struct DwDesc {
    DwSeg seg[4];
    uint32_t nseg;
    uint32_t cval;    // constant bytes (header words, key literals)
    uint32_t pad[2];
};

struct FixProgram {
    const FixSeg* segs;
    const uint32_t* seg_index;   // B+1 entries: segments of period-dword r
    const FixCol* fcols;
    const DwDesc* dw;            // B/4 entries when B % 4 == 0
    int32_t B, T, n_fcols, lds_bytes, total_chunks, overflow;
    int32_t fc_lds;              // LDS offset of the per-launch copy of fcols (set at launch)
    // k_encode_fixed_tile: output dwords fed by >1 column run or by a bool
    // byte ("X dwords") are assembled once per blob into an LDS X region
    // (T rows x nx dwords at x_lds); tdw then gives every dword ONE aligned-
    // or-shifted source (its column run, or its X slot)
    const DwDesc* tdw;           // B/4 single-source descriptors
    const DwDesc* xdw;           // nx full descriptors of the X dwords
    const uint32_t* xq;          // nx: output dword index of each X dword (unused by kernels)
    int32_t nx, x_lds;
};

// Staging plan of the pipelined fixed-layout kernel, passed BY VALUE as a
// kernel argument so a workgroup can issue its first tile's loads straight
// from kernarg (no dependent global table read in front of them).
constexpr int kStageCols = 16;
struct FixStageCol {
    const uint8_t* base;   // column data pointer (row 0)
    uint32_t width;        // row bytes
    uint32_t lds_off;      // LDS offset of the column's tile region
    uint32_t chunk_begin;  // first 16-B chunk of the column within a tile
    uint32_t flags;        // bit0: bool column
};
struct FixStage {
    FixStageCol c[kStageCols];
    int32_t n;
    int32_t flags;         // bit0: some column is bool
};

// ---------------------------------------------------------------- decode ----
// DecNode.variable flags of a tuple
enum : uint8_t {
    DT_VARIABLE = 1,    // VariableLength: no arg-count check
    DT_NAMED = 2,       // TupleSchemaNamed: the arg-count check has no argCount > 0 guard
                        // (schema.go:1773 vs TupleSchema's :1607)
    DT_NAMES_BAD = 4,   // TupleSchemaNamed, len(FieldNames) != len(Schemas): Decode fails
                        // first with ErrConstraintViolated at position 0 (schema.go:1756-1758)
};

struct DecNode {
    int32_t kind;      // NodeKind
    int32_t width;     // scalar width, or SchemaString/SchemaBytes Width
    int32_t col;       // column, -1 for K_MATCH / K_ROOT
    int32_t nkids;
    int32_t kid0;      // first entry in the kid list
    uint8_t nullable;  // precheck nullable flag (schema IsNullable())
    uint8_t variable;  // tuples: DT_* flags
    uint8_t tag;
    uint8_t pad;
    uint32_t lit, lit_len;    // K_MATCH literal, or the Prefix / Suffix literal
    uint32_t check;           // CHK_* value checks
    uint32_t dlit, dlit_len;  // DefaultDecodeValue literal (CHK_DEFAULT)
    uint32_t pad2;
    int64_t rmin, rmax;       // CHK_MIN / CHK_MAX bounds
};

struct DecProgram {
    const DecNode* nodes;
    const int32_t* kids;
    const uint8_t* lits;
    int32_t root;
    int32_t n_nodes, n_kids, n_lits;   // table sizes (for staging into LDS)
    int32_t flat;      // F > 0: the chain is F leaves (no tuple / map), F <= 15: canonical fast path
    int32_t ext;       // PACKOS_MODE_EXTENDED: tag-2 containers are read (ADR-001)
    int32_t win;       // > 0: the decoder reads nothing past this many leading blob bytes but
                       // var views (no fixed field / header after the first var payload)
};

// Fixed-layout decode fast path.  A blob whose length is B and whose
// constant bytes (header words, MATCH literals, map keys) equal those of the
// schema's all-present layout walks the SeqGetAccess machine exactly like the
// canonical blob does, so its leaves sit at compile-time positions.
struct DecFix {
    int32_t col;
    uint32_t width;
    uint32_t blob_off;     // first payload byte of the leaf inside the blob
    uint32_t flags;        // bit0: bool (normalise to 0/1)
    uint32_t magic;        // ceil(2^32 / width) for width > 1 (division by width)
    uint32_t pad[3];
};

// Value check of a fixed leaf in the fixed-layout decode fast path: a row
// that fails it is re-decoded by the exact per-blob decoder (which reports it).
struct DecChk {
    uint32_t blob_off, width, flags, lit, lit_len, pad;
    int64_t rmin, rmax;
};

struct DecFixProgram {
    const DecFix* cols;
    const DecChk* vchk;    // n_vchk value checks
    const uint32_t* chk;   // n_chk triples {blob dword q, constant-byte mask, constant value}, mask != 0
    int32_t B, T, n_cols, pad;
    uint32_t q_magic;      // B % 4 == 0: ceil(2^32 / (B/4)) (0 when B/4 == 1)
    uint32_t b_magic;      // B % 4 != 0: ceil(2^32 / B)
    int32_t n_all_cols;    // every schema column (validity marking)
    int32_t n_chk;
    int32_t n_vchk;
};

// column pointer tables passed by value as kernel arguments
struct EncCols {
    const uint8_t* data[kMaxCols];
    const void* off[kMaxCols];      // var offsets: uint32_t[n+1], or uint64_t[n+1] when off64 bit c is set
    const uint8_t* valid[kMaxCols];
    uint64_t off64;
};

struct DecCols {
    uint8_t* data[kMaxCols];
    uint8_t* valid[kMaxCols];
    uint64_t* start[kMaxCols];
    uint32_t* length[kMaxCols];
};

}  // namespace packos
