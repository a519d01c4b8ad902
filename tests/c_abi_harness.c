/* c_abi_harness.c — the cgo shim's call sequence, in C.
 *
 * What a Go caller of libpackos does, step by step, with nothing but the C
 * ABI of include/packos.h and the HIP runtime:
 *   1. compile the schema from the JSON Go's json.Marshal makes of a
 *      []schema.SchemaJSON (schemabuilder_json.go:8-30): every key but "type"
 *      is omitempty, and "extra" (UI metadata, map[string]any) may hold any
 *      JSON value, which BuildSchema never reads;
 *   2. lay the rows out as columns (packos_schema_column_info: one column per
 *      non-constant node, pre-order) in pinned memory from hipHostMalloc,
 *      which cgo allows (no Go pointers inside);
 *   3. packos_encode_host_batch — PutAccess Add* / Pack() for every row;
 *   4. compare every blob with the reference's own bytes for that row
 *      (access/put_test.go:12-41: 17 bytes, given on the command line from
 *      tests/golden/vectors.json "put_flat17");
 *   5. packos_decode_host_batch — DecodeBuffer of every blob back into host
 *      columns; values and views must be the row's;
 *   6. packos_validate_host_batch — ValidateBuffer of every blob, one of
 *      them corrupted.
 * Built by oracle/Makefile (test infrastructure), run by
 * tests/test_c_abi_harness.py on the GPU box.  Exit 0 and "c_abi_harness ok".
 *
 *   usage: c_abi_harness <expected blob hex> [n_blobs]
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "packos.h"

/* json.Marshal([]schema.SchemaJSON{{Type: "int16", Extra: ...}, {Type: "bool"},
 * {Type: "string"}, {Type: "bytes", Extra: map[string]any{}}}) — field order
 * of the struct, empty / zero keys dropped; an empty Extra map is omitted too */
static const char* kSchemaJSON =
    "[{\"type\":\"int16\",\"extra\":{\"label\":\"id\",\"order\":1,\"tags\":[\"a\",\"b\"],"
    "\"ui\":{\"widget\":\"spinner\",\"step\":0.5,\"hidden\":false,\"hint\":null}}},"
    "{\"type\":\"bool\"},{\"type\":\"string\"},{\"type\":\"bytes\"}]";

#define CHECK(c, ...)                                        \
    do {                                                     \
        if (!(c)) {                                          \
            fprintf(stderr, "c_abi_harness: " __VA_ARGS__);  \
            fprintf(stderr, "\n");                           \
            return 1;                                        \
        }                                                    \
    } while (0)

static void* pinned(size_t bytes) {
    void* p = NULL;
    if (hipHostMalloc(&p, bytes ? bytes : 16, 0) != hipSuccess) return NULL;
    memset(p, 0, bytes ? bytes : 16);
    return p;
}

static int unhex(const char* h, uint8_t* out, size_t cap) {
    size_t n = strlen(h) / 2;
    if (n > cap) return -1;
    for (size_t i = 0; i < n; i++) {
        unsigned v;
        if (sscanf(h + 2 * i, "%2x", &v) != 1) return -1;
        out[i] = (uint8_t)v;
    }
    return (int)n;
}

int main(int argc, char** argv) {
    CHECK(argc >= 2, "usage: c_abi_harness <expected blob hex> [n_blobs]");
    uint8_t want[64];
    const int B = unhex(argv[1], want, sizeof(want));
    CHECK(B > 0, "bad expected hex");
    const size_t n = argc > 2 ? (size_t)strtoull(argv[2], NULL, 10) : 100000;
    CHECK(packos_abi_version() >= 3, "ABI version %d", packos_abi_version());

    /* 1. schema */
    packos_schema* s = NULL;
    int rc = packos_schema_compile(kSchemaJSON, PACKOS_MODE_PUTACCESS, &s);
    CHECK(rc == 0, "compile: %s (%s)", packos_strerror(rc), packos_last_error());
    const int ncol = packos_schema_num_columns(s);
    CHECK(ncol == 4, "%d columns", ncol);
    static const int kinds[4] = {PACKOS_KIND_INT, PACKOS_KIND_BOOL, PACKOS_KIND_STRING, PACKOS_KIND_BYTES};
    static const int widths[4] = {2, 1, 0, 0};
    for (int c = 0; c < ncol; c++) {
        packos_column_info ci;
        CHECK(packos_schema_column_info(s, c, &ci) == 0, "column_info %d", c);
        CHECK(ci.kind == kinds[c] && ci.width == widths[c] && ci.top_index == c && ci.depth == 0,
              "column %d: kind %d width %d top %d depth %d", c, ci.kind, ci.width, ci.top_index, ci.depth);
    }
    CHECK(packos_schema_fixed_blob_size(s) == -1, "a var schema has no fixed size");

    /* 2. rows -> pinned columns: the row of access/put_test.go:12-41,
     * AddInt16(42) AddBool(true) AddString("go") AddBytes({0xAA, 0xBB}) */
    int16_t* c_int = (int16_t*)pinned(2 * n);
    uint8_t* c_bool = (uint8_t*)pinned(n);
    uint8_t* c_str = (uint8_t*)pinned(2 * n);
    uint32_t* o_str = (uint32_t*)pinned(4 * (n + 1));
    uint8_t* c_byt = (uint8_t*)pinned(2 * n);
    uint32_t* o_byt = (uint32_t*)pinned(4 * (n + 1));
    CHECK(c_int && c_bool && c_str && o_str && c_byt && o_byt, "hipHostMalloc failed");
    for (size_t i = 0; i < n; i++) {
        c_int[i] = 42;
        c_bool[i] = 1;
        c_str[2 * i] = 'g';
        c_str[2 * i + 1] = 'o';
        c_byt[2 * i] = 0xAA;
        c_byt[2 * i + 1] = 0xBB;
        o_str[i] = o_byt[i] = (uint32_t)(2 * i);
    }
    o_str[n] = o_byt[n] = (uint32_t)(2 * n);
    packos_column cols[4];
    memset(cols, 0, sizeof(cols));
    cols[0].data = c_int;
    cols[1].data = c_bool;
    cols[2].data = c_str;
    cols[2].offsets = o_str;
    cols[3].data = c_byt;
    cols[3].offsets = o_byt;

    /* 3. encode (host columns -> host arena; the library pipelines H2D / kernel / D2H) */
    const uint64_t cap = (uint64_t)B * n;
    uint8_t* arena = (uint8_t*)pinned(cap);
    uint64_t* offs = (uint64_t*)pinned(8 * (n + 1));
    uint32_t* st = (uint32_t*)pinned(4 * n);
    CHECK(arena && offs && st, "hipHostMalloc failed");
    rc = packos_encode_host_batch(s, cols, n, arena, cap, offs, st, 0);
    CHECK(rc == 0, "encode_host_batch: %s (%s)", packos_strerror(rc), packos_last_error());

    /* 4. every blob = the reference bytes */
    for (size_t i = 0; i < n; i++) {
        CHECK(offs[i] == (uint64_t)B * i, "offset %zu = %llu", i, (unsigned long long)offs[i]);
        CHECK(st[i] == 0, "status %zu = %#x", i, st[i]);
        CHECK(memcmp(arena + offs[i], want, (size_t)B) == 0, "blob %zu differs from the reference bytes", i);
    }
    CHECK(offs[n] == cap, "total %llu", (unsigned long long)offs[n]);

    /* 5. decode the host arena back (views are absolute arena offsets) */
    int16_t* d_int = (int16_t*)pinned(2 * n);
    uint8_t* d_bool = (uint8_t*)pinned(n);
    uint64_t* v_start[2] = {(uint64_t*)pinned(8 * n), (uint64_t*)pinned(8 * n)};
    uint32_t* v_len[2] = {(uint32_t*)pinned(4 * n), (uint32_t*)pinned(4 * n)};
    uint32_t* dst = (uint32_t*)pinned(4 * n);
    packos_column out[4];
    memset(out, 0, sizeof(out));
    out[0].data = d_int;
    out[1].data = d_bool;
    for (int v = 0; v < 2; v++) {
        out[2 + v].start = v_start[v];
        out[2 + v].length = v_len[v];
    }
    rc = packos_decode_host_batch(s, arena, offs, 0, n, out, dst, 0);
    CHECK(rc == 0, "decode_host_batch: %s (%s)", packos_strerror(rc), packos_last_error());
    for (size_t i = 0; i < n; i++) {
        CHECK(dst[i] == 0, "decode status %zu = %#x", i, dst[i]);
        CHECK(d_int[i] == 42 && d_bool[i] == 1, "decoded scalars of blob %zu", i);
        CHECK(v_len[0][i] == 2 && memcmp(arena + v_start[0][i], "go", 2) == 0, "decoded string of blob %zu", i);
        CHECK(v_len[1][i] == 2 && arena[v_start[1][i]] == 0xAA && arena[v_start[1][i] + 1] == 0xBB,
              "decoded bytes of blob %zu", i);
    }
    /* 6. packos_validate_host_batch — ValidateBuffer of every blob (status only);
     *    a blob whose first field header is cut to tag End fails precheck  */
    arena[(n / 2) * (size_t)B + 2] &= 0xF8;
    rc = packos_validate_host_batch(s, arena, offs, 0, n, dst, 0);
    CHECK(rc == 0, "validate_host_batch: %s (%s)", packos_strerror(rc), packos_last_error());
    for (size_t i = 0; i < n; i++)
        CHECK(i == n / 2 ? dst[i] != 0 : dst[i] == 0, "validate status %zu = %#x", i, dst[i]);
    packos_schema_free(s);
    printf("c_abi_harness ok: %zu blobs of %d bytes\n", n, B);
    return 0;
}
