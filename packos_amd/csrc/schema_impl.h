// schema_impl.h — host representation of a compiled schema (packos_schema).
#pragma once
#include <hip/hip_runtime_api.h>

#include <deque>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/packos.h"
#include "program.h"

namespace packos {

struct Node {
    int kind = 0;          // NodeKind
    int width = 0;         // scalar width / SchemaString|SchemaBytes Width
    bool nullable = false; // scalar Nullable / TupleSchema.Nullable
    bool variable = false; // TupleSchema.VariableLength
    bool named = false;    // TupleSchemaNamed (arg-count check without the argCount > 0 guard)
    bool names_bad = false; // TupleSchemaNamed with len(FieldNames) != len(Schemas)
    bool sorted = false;   // map pairs sorted by key (PackMapSorted)
    std::string literal;   // K_MATCH
    // value checks (schema.go:1172-1364 Range, :2188-2250 SDateRange,
    // :1070-1158 CheckFunc Prefix/Suffix, :284-286 DefaultDecodeValue)
    uint32_t check = 0;    // CHK_* bits (program.h)
    int64_t rmin = 0, rmax = 0;
    std::string check_lit; // Prefix / Suffix literal
    std::string dflt;      // SchemaString.DefaultDecodeVal
    std::vector<int> kids; // emission order
    std::string name;      // dotted field path
    int col = -1;
    int parent = -1;
    int depth = 0;
    int top = -1;
};

// Tuning / testing knobs, read ONCE when the schema is compiled (never on the
// launch path): PACKOS_VAR_PER (var staging pool bytes per blob of the
// variable-size encoder), PACKOS_SIZES_SCAN=1 (look-back size kernel even for
// closed-form layouts), PACKOS_DECODE_GENERIC=1 (thread-per-blob decoder even
// for fixed layouts), PACKOS_DEC_TILE_BYTES (staged bytes per fixed-decode
// tile), PACKOS_TILE_BYTES (fixed-encode tile bytes), PACKOS_ENC_FLAT
// (flat closed-form var encoder k_encode_flat: 0 never, 1 always, 2 = auto:
// when the output capacity averages >= 256 B per blob).
struct Tune {
    int var_per = 40;
    bool var_per_set = false;    // PACKOS_VAR_PER given: no data-sized pool
    bool sizes_scan = false;
    bool decode_generic = false;
    int dec_tile_bytes = 0;      // 0: 24 KB for B >= 128, else 16 KB
    int enc_flat = 2;            // PACKOS_ENC_FLAT: 0 never, 1 always, 2 auto (large blobs)
};

struct DeviceTables {
    int device = -1;
    void* block = nullptr;   // one allocation holding every table below
    EncProgram enc{};
    FixProgram fix{};
    DecProgram dec{};
    DecFixProgram dfix{};
    const EncCheck* echk = nullptr;
};

}  // namespace packos

struct packos_schema {
    int mode = 0;                      // PACKOS_MODE_PUTACCESS / PACKOS_MODE_PACKABLE
    bool ext = false;                  // PACKOS_MODE_EXTENDED (ADR-001 extended containers)
    std::vector<packos::Node> nodes;   // node 0 = K_ROOT (the chain)
    std::vector<int> col_node;         // column -> node
    std::vector<packos_column_info> col_info;
    int n_top = 0;
    // SchemaNamedChain whose len(FieldNames) != len(Schemas): len(FieldNames),
    // else 0.  EncodeValueNamed walks FieldNames (fewer: only that many fields
    // are written; more: a panic once the schemas are written), DecodeBufferNamed
    // fails every blob NewSeqGetAccess accepts (schema.go:948-995); ValidateBuffer
    // takes the plain SchemaChain (unchanged)
    int chain_names = 0;

    // encode program (host copies)
    std::vector<packos::EncItem> items;
    std::vector<uint32_t> ipk;           // packed per-item size / var slot (EncProgram::ipk)
    std::vector<uint32_t> ihr;           // per-item header-entry range (EncProgram::ihr)
    std::vector<packos::EncHdr> hdrs;
    std::vector<packos::EncCont> conts;
    std::vector<uint8_t> lits;
    std::vector<packos::EncCheck> echk;   // encode-time value checks (emission order)
    bool has_var = false;        // any var-width leaf
    bool has_nullable = false;   // any nullable leaf / container column
    int64_t all_present_size = -1;  // blob size when every nullable is present (no var leaves)
    bool all_present_overflow = false;

    // fixed layout (valid when fix_ok)
    bool fix_ok = false;
    std::vector<packos::FixSeg> fsegs;
    std::vector<uint32_t> fseg_index;
    std::vector<packos::FixCol> fcols;
    std::vector<packos::DwDesc> fdw;   // lane-invariant descriptors (B % 4 == 0)
    int fix_T = 0, fix_lds = 0, fix_chunks = 0;
    int fix_maxseg = 0;                 // max column segments of any output dword (fdw)
    std::vector<packos::DwDesc> ftdw, fxdw;  // k_encode_fixed_tile: single-source + X dwords
    std::vector<uint32_t> fxq;
    int fix_x_lds = 0, fix_tile_lds = 0;

    // decode program
    std::vector<packos::DecNode> dnodes;
    std::vector<int32_t> dkids;
    // fixed-layout decode fast path (B % 4 == 0, B <= 1024); dec_fast is set
    // when the canonical blob decodes cleanly (checked on first upload)
    std::vector<packos::DecFix> dfix;
    std::vector<packos::DecChk> dvchk;    // value checks of fixed leaves
    std::vector<uint32_t> dchk;
    std::vector<uint8_t> canon;       // all-present blob, zero payload bytes
    int dec_fast = 0;                 // 1: canonical blob decodes (set at compile)
    int64_t dec_prefix = 0;           // bytes of an all-present blob before its first var payload
    bool dec_tail_fixed = false;      // some header / fixed / literal item follows the first var item
    int64_t val_win = 0;              // > 0: ValidateBuffer reads nothing past this many leading bytes

    packos::Tune tune;

    std::string describe;

    std::mutex mu;
    std::deque<packos::DeviceTables> dev;   // deque: pointers handed out stay valid
    // host-resident batches: one cached pipeline per device (host_pipeline.cpp),
    // created on first use by packos_encode_host_batch / packos_decode_host_batch
    std::vector<packos_pipeline*> pipes;
};

namespace packos {
// thread-local last error string
void set_error(const std::string& m);
void read_tune(Tune& t);
int upload_tables(packos_schema* s, int device, DeviceTables** out);
// host run of the device decoder over the canonical blob (kernels.hip)
bool canonical_decodes(const packos_schema* s);
// extended mode (ADR-001): item sizes of one blob (nil = 0) -> the header
// items of containers written extended grow to ext_hdr_bytes (bottom-up,
// children first); returns the bit mask of extended containers
uint64_t ext_layout_host(const packos_schema* s, std::vector<int64_t>& sz);
// extended mode: bytes every container's extended header block may add to a blob
int64_t ext_overhead(const packos_schema* s);
// host pipelines (host_pipeline.cpp): free the schema's cached pipelines
void destroy_pipelines(packos_schema* s);
// tiny device helpers (kernels.hip) for the host pipelines
int launch_fill_offsets(uint64_t* offs, size_t n, uint64_t base, uint64_t B, hipStream_t st);
int launch_add_base(uint64_t* offs, size_t n, uint64_t add, hipStream_t st);
}  // namespace packos
