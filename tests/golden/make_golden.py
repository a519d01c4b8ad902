#!/usr/bin/env python3
"""Build tests/golden/vectors.json from the reference's own tests.

Byte vectors are EXTRACTED from the reference test sources under
/root/reference (the `expected := []byte{...}` / `buf := []byte{...}` blocks
of access/put_test.go, packable/pack_test.go, access/get_test.go,
access/seqget_test.go and README.md): the parser below reads the hex and char
literals of the block that starts at the cited line.  What each test FEEDS the
API (the Add*/Pack* call sequence or the schema + value) is transcribed by
hand into the CASES table as a schema (SchemaJSON vocabulary) plus one row
value, with the same file:line citation.

Cross-API equalities the reference asserts without spelling out bytes
(e.g. schema.EncodeValue == packable.Pack) are recorded as "equal" groups.
"inputs" are blobs a reference test builds with pack.Pack(...) without
spelling out its bytes (the checker's encoder, pinned by the byte vectors
above, rebuilds them); "decode" cases then name what DecodeBuffer returns
for them.  Cases marked "derived" restate a reference behaviour no reference
test exercises (e.g. a Range violation): parity there rests on the cited code.

The reference is Go and no Go toolchain exists in this image, so nothing here
runs the reference; the JSON is data only.  Run: python tests/golden/make_golden.py
"""
import json
import os
import re
import sys

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "vectors.json")


def extract_bytes(relpath, line):
    """Hex/char literals of the []byte{...} block starting at `line` (1-based)."""
    with open(os.path.join(REF, relpath), encoding="utf-8") as f:
        lines = f.read().split("\n")
    i = line - 1
    if "[]byte{" not in lines[i]:
        raise ValueError(f"{relpath}:{line} is not a []byte{{ block: {lines[i]!r}")
    out = []
    depth = 0
    first = True
    while True:
        ln = lines[i]
        code = ln.split("//", 1)[0]
        if first:
            code = code.split("[]byte{", 1)[1]
            depth = 1
            first = False
        for tok in re.finditer(r"0x[0-9A-Fa-f]{1,2}|'(\\.|[^'])'|[{}]", code):
            t = tok.group(0)
            if t == "{":
                depth += 1
            elif t == "}":
                depth -= 1
                if depth == 0:
                    return bytes(out)
            elif t.startswith("0x"):
                out.append(int(t, 16))
            else:
                ch = tok.group(1)
                out.append(ord(ch.encode().decode("unicode_escape")))
        i += 1


def S(x):
    return {"s": x}


def B(x):
    return {"b": x.encode().hex() if isinstance(x, str) else x.hex()}


def F32(x):
    return {"f32": x}


# SchemaJSON snippets
I16 = {"type": "int16"}
I32 = {"type": "int32"}
I64 = {"type": "int64"}
F32T = {"type": "float32"}
BOOL = {"type": "bool"}
STR = {"type": "string"}
BYT = {"type": "bytes"}
I16R = {"type": "int16", "min": 0, "max": 20000}      # SInt16.RangeValues(0, 20000)
I32R = {"type": "int32", "min": 1, "max": 100}        # SInt32.RangeValues(1, 100)


def EX(k):
    return {"type": "string", "exact": k}


def MAP(*kv, sorted_=False):
    d = {"type": "map", "schema": list(kv)}
    if sorted_:
        d["sorted"] = True
    return d


def TUP(*kids, names=None):
    d = {"type": "tuple", "schema": list(kids)}
    if names:
        d["fieldNames"] = names
    elif names is not None:
        # STupleNamed(nil, ...): BuildSchema routes an empty fieldNames to STuple
        # (schemabuilder_json.go:245), so this build marks the named form itself
        d["named"] = True
    return d


META_SORTED = MAP(EX("user"), BYT, EX("role"), BYT, sorted_=True)
META_ORDERED = MAP(EX("role"), BYT, EX("user"), BYT)
ROW_META = {"user": B("alice"), "role": B("admin")}

ENCODE = [
    # id, source, mode, schema, row, bytes-source
    ("put_flat17", "access/put_test.go:12-41", "putaccess", [I16, BOOL, STR, BYT],
     [42, True, S("go"), B(b"\xaa\xbb")], ("access/put_test.go", 22)),
    ("put_map_sorted32", "access/put_test.go:44-75", "putaccess",
     [MAP(EX("user"), BYT, EX("role"), BYT, sorted_=True)], [ROW_META],
     ("access/put_test.go", 53)),
    ("put_int_nested_sorted60", "access/put_test.go:78-135", "putaccess",
     [I16, MAP(EX("meta"), META_SORTED, EX("name"), STR, sorted_=True)],
     [12345, {"meta": ROW_META, "name": S("gopher")}], ("access/put_test.go", 91)),
    ("put_nullables23", "access/put_test.go:138-177", "putaccess",
     [{"type": "int32", "nullable": True}, {"type": "int32", "nullable": True},
      {"type": "float32", "nullable": True}, {"type": "float32", "nullable": True},
      {"type": "bool", "nullable": True}, {"type": "bool", "nullable": True}],
     [None, 123456, None, F32(3.14159), None, True], ("access/put_test.go", 154)),
    ("put_ordered60", "access/put_test.go:180-245", "putaccess",
     [I16, MAP(EX("meta"), META_ORDERED, EX("name"), STR)],
     [12345, {"meta": ROW_META, "name": S("gopher")}], ("access/put_test.go", 202)),
    ("pack_flat17", "packable/pack_test.go:12-40", "packable", [I16, BOOL, STR, BYT],
     [42, True, S("go"), B(b"\xaa\xbb")], ("packable/pack_test.go", 17)),
    ("pack_sorted60", "packable/pack_test.go:42-97", "packable",
     [I16, MAP(EX("meta"), META_SORTED, EX("name"), STR, sorted_=True)],
     [12345, {"meta": ROW_META, "name": S("gopher")}], ("packable/pack_test.go", 54)),
    ("pack_two_tuples34", "packable/pack_test.go:120-171", "packable",
     [TUP(I32, BOOL, STR), TUP(I16, BOOL, STR)],
     [[2025, False, S("az")], [7, True, S("go")]], ("packable/pack_test.go", 134)),
    ("pack_ordered60", "packable/pack_test.go:173-232", "packable",
     [I16, MAP(EX("meta"), META_ORDERED, EX("name"), STR)],
     [12345, {"meta": ROW_META, "name": S("gopher")}], ("packable/pack_test.go", 191)),
    ("readme_flat17", "README.md:43-65", "putaccess", [I16, BOOL, STR, BYT],
     [42, True, S("go"), B(b"\xaa\xbb")], ("README.md", 52)),
    ("readme_sorted60", "README.md:69-115", "packable",
     [I16, MAP(EX("meta"), META_SORTED, EX("name"), STR, sorted_=True)],
     [12345, {"meta": ROW_META, "name": S("gopher")}], ("README.md", 80)),
    ("readme_two_tuples34", "README.md:119-156", "packable",
     [TUP(I32, BOOL, STR), TUP(I16, BOOL, STR)],
     [[2025, False, S("az")], [7, True, S("go")]], ("README.md", 132)),
    # schema.EncodeValue of the two tuples must give pack_test's bytes
    ("schema_two_tuples34", "schema/schema_test.go:781-818 (expected = pack.Pack(...) = packable/pack_test.go:134)",
     "putaccess",
     [TUP(I32, BOOL, {"type": "string", "width": 2}), TUP(I16, BOOL, {"type": "string", "width": 2})],
     [[2025, False, S("az")], [7, True, S("go")]], ("packable/pack_test.go", 134)),
    ("schema_named_tuples34", "schema/schema_test.go:1248-1303 (expected = packable/pack_test.go:134)",
     "putaccess",
     {"type": "chain", "fieldNames": ["firstTuple", "secondTuple"], "schema": [
         TUP(I32, BOOL, {"type": "string", "width": 2}, names=["year", "flag", "code"]),
         TUP(I16, BOOL, {"type": "string", "width": 2}, names=["num", "flag", "lang"])]},
     {"firstTuple": {"year": 2025, "flag": False, "code": S("az")},
      "secondTuple": {"num": 7, "flag": True, "lang": S("go")}}, ("packable/pack_test.go", 134)),
    # derived (schema.go:968-995): EncodeValueNamed walks FieldNames, so a
    # SchemaNamedChain with a third schema but two names writes the two named
    # tuples only -- the same 34 bytes as above
    ("derived_named_chain_fewer_names", "derived: schema/schema.go:968-995 (expected = packable/pack_test.go:134)",
     "putaccess",
     {"type": "chain", "fieldNames": ["firstTuple", "secondTuple"], "schema": [
         TUP(I32, BOOL, {"type": "string", "width": 2}, names=["year", "flag", "code"]),
         TUP(I16, BOOL, {"type": "string", "width": 2}, names=["num", "flag", "lang"]),
         TUP(I16, names=["extra"])]},
     {"firstTuple": {"year": 2025, "flag": False, "code": S("az")},
      "secondTuple": {"num": 7, "flag": True, "lang": S("go")}}, ("packable/pack_test.go", 134)),
]

# groups whose encodings the reference asserts equal (no literal bytes)
EQUAL = [
    ("putaccess_addpackable_eq_pack", "packable/pack_test.go:99-118", [
        ("putaccess", [I16, MAP(EX("meta"), META_SORTED, EX("name"), STR, sorted_=True), F32T]),
        ("packable", [I16, MAP(EX("meta"), META_SORTED, EX("name"), STR, sorted_=True), F32T])],
     [12345, {"meta": ROW_META, "name": S("gopher")}, F32(4.45)]),
    ("putaccess_addpackable_ordered_eq_pack", "packable/pack_test.go:234-256", [
        ("putaccess", [I16, MAP(EX("meta"), META_ORDERED, EX("name"), STR), F32T]),
        ("packable", [I16, MAP(EX("meta"), META_ORDERED, EX("name"), STR), F32T])],
     [12345, {"meta": ROW_META, "name": S("gopher")}, F32(4.45)]),
    ("schema_empty_tuples1", "schema/schema_test.go:820-839", [
        ("putaccess", [TUP(), TUP()]),
        ("packable", [TUP(), TUP()])],
     [None, None]),
    ("schema_empty_tuples2", "schema/schema_test.go:840-869", [
        ("putaccess", [I16, TUP(STR, STR, STR), TUP(), TUP(STR, names=["ok"]), TUP(names=[]), I16]),
        ("packable", [I16, TUP(), TUP(), TUP(), TUP(), I16])],
     [5, None, None, None, None, 5]),
    ("schema_empty_maps", "schema/schema_test.go:870-911 (SMap subset)", [
        ("putaccess", [I16, MAP(STR, STR), MAP(STR, STR), MAP(STR, STR), I16]),
        ("packable", [I16, MAP(), MAP(), MAP(), I16])],
     [5, None, None, None, 5]),
    ("schema_packed_structure", "schema/schema_test.go:1116-1173", [
        ("putaccess", [I16, F32T, I64, BOOL,
                       MAP(EX("meta"), MAP(EX("role"), {"type": "bytes", "width": 5},
                                           EX("user"), {"type": "bytes", "width": 5}),
                           EX("name"), {"type": "string", "width": 6})]),
        ("packable", [I16, F32T, I64, BOOL,
                      MAP(EX("meta"), META_SORTED, EX("name"), STR, sorted_=True)]),
        # the test's own schema: SInt16.RangeValues(0, 20000) (schema_test.go:1133-1134)
        ("putaccess", [I16R, F32T, I64, BOOL,
                       MAP(EX("meta"), MAP(EX("role"), {"type": "bytes", "width": 5},
                                           EX("user"), {"type": "bytes", "width": 5}),
                           EX("name"), {"type": "string", "width": 6})])],
     [12345, F32(3.14), 9876543210, True, {"meta": ROW_META, "name": S("gopher")}]),
]

# blobs built by pack.Pack(...) inside reference tests (no literal bytes there)
INPUTS = [
    ("pack_date_range_email_prefix_suffix", "schema/schema_test.go:407-413 (pack.Pack of five values)", "packable",
     [STR, I32, STR, STR, STR],
     [S("2025-09-10"), 42, S("alice@example.com"), S("prefix-hello"), S("world-suffix")]),
    ("pack_defaults_empty", "schema/schema_test.go:443-450 (pack.Pack with three empty strings)", "packable",
     [STR, I32, STR, STR, STR], [S("2025-09-10"), 42, S(""), S(""), S("")]),
    ("pack_four_tuples", "schema/schema_test.go:559-583 (pack.Pack of four tuples)", "packable",
     [TUP(I32, BOOL, STR), TUP(I16, BOOL, STR), TUP(I32, BOOL, STR), TUP(I32, BOOL, STR)],
     [[2025, False, S("az")], [7, True, S("go")], [111, True, S("xx")], [222, False, S("yy")]]),
    # derived: pack.Pack(pack.PackTuple(pack.PackInt16(7))) = 24 00 30 00 21 00 10 00 07 00
    ("pack_one_tuple_int16", "derived: pack.Pack(pack.PackTuple(pack.PackInt16(7)))", "packable",
     [TUP(I16)], [[7]]),
    # TestValidateChain_DateEmailPrefixSuffix_Success2: pack.Pack of seven values
    ("pack_optional_email_seven", "schema/schema_test.go:187-195 (pack.Pack of seven values)", "packable",
     [STR, STR, I32, STR, STR, STR, STR],
     [S(""), S("2025-09-10"), 42, S("alice@example.com"), S("prefix-hello"), S("world-suffix"), S("")]),
    # TestSDate_SuccessAndNullable: pack.Pack(pack.PackInt64(date.Unix())) for
    # 2025-09-10 (inside 2020..2030) and 2050-01-01 (outside), and
    # pack.Pack(pack.PackNullableInt64(nil)) (Q2: 8 bytes of slack after End)
    ("pack_date_2025", "schema/schema_test.go:1363-1364 (pack.Pack(PackInt64(2025-09-10)))", "packable",
     [I64], [1757462400]),
    ("pack_nullable_int64_nil", "schema/schema_test.go:1377 (pack.Pack(PackNullableInt64(nil)))", "packable",
     [{"type": "int64", "nullable": True}], [None]),
    ("pack_date_2050", "schema/schema_test.go:1386-1387 (pack.Pack(PackInt64(2050-01-01)))", "packable",
     [I64], [2524608000]),
    # derived: pack.Pack(pack.PackInt8(7)) = 04 00 29 00 07: a 1-byte Integer field
    ("pack_int8_7", "derived: pack.Pack(pack.PackInt8(7))", "packable",
     [{"type": "int8"}], [7]),
]

SDATE_2020_2030 = {"type": "date", "nullable": True, "dateFrom": "2020-01-01T00:00:00Z",
                   "dateTo": "2030-12-31T23:59:59Z"}     # SDate(true, from, to), schema_test.go:1356-1360
SEVEN_SCHEMA = [STR, STR, I32R, STR, {"type": "string", "prefix": "prefix-"}, {"type": "string", "suffix": "-suffix"},
                {"type": "string", "nullable": True, "suffix": "-suffix"}]
PACKED_MAP = MAP(EX("meta"), MAP(EX("role"), {"type": "bytes", "width": 5}, EX("user"), {"type": "bytes", "width": 5}),
                 EX("name"), {"type": "string", "width": 6})
PACKED_ROW = [12345, F32(3.14), 9876543210, True, {"meta": {"role": B("admin"), "user": B("alice")},
                                                   "name": S("gopher")}]

# random-access known answers: (pos path, want_tag, want_width, expected payload)
GET = [
    ("get_flat", "access/get_test.go:11-44", ("access/get_test.go", 12), [
        ([0], 1, 2, "2a00"), ([1], 5, 1, "01"), ([2], 6, -1, b"go".hex()), ([3], 6, -1, "aabb")]),
    ("get_map2", "access/get_test.go:46-63", ("access/get_test.go", 47), [
        ([0, 0], 6, -1, b"role".hex()), ([0, 1], 6, -1, b"admin".hex()),
        ([0, 2], 6, -1, b"user".hex()), ([0, 3], 6, -1, b"alice".hex())]),
    ("get_map_ordered", "access/get_test.go:65-96", ("access/get_test.go", 66), [
        ([0, 0], 6, -1, b"role".hex()), ([0, 3], 6, -1, b"alice".hex())]),
    ("get_int_then_map", "access/get_test.go:98-126", ("access/get_test.go", 99), [
        ([0], 1, 2, "3930"), ([1, 0], 6, -1, b"meta".hex()), ([1, 1, 1], 6, -1, b"admin".hex()),
        ([1, 1, 3], 6, -1, b"alice".hex()), ([1, 2], 6, -1, b"name".hex()),
        ([1, 3], 6, -1, b"gopher".hex())]),
]

# map-walk known answers (GetMapStr / GetMapAny / GetMapOrderedAny): (id,
# source, bytes, path, flags 0 = MAP_STR / 1 = MAP_ANY, expected pairs in wire
# order as (key, value tag, value payload))
INNER_MAP = bytes([0x56, 0x00, 0x26, 0x00, 0x4E, 0x00, 0x6E, 0x00, 0x90, 0x00]) + b"roleadminuseralice"
MAPS = [
    ("map_str", "access/get_test.go:46-63 (GetMapStr(0) == {role: admin, user: alice})",
     ("access/get_test.go", 47), [0], 0, [(b"role", 6, b"admin"), (b"user", 6, b"alice")]),
    ("map_ordered_any", "access/get_test.go:65-96 (GetMapOrderedAny(0): role, user in order)",
     ("access/get_test.go", 66), [0], 1, [(b"role", 6, b"admin"), (b"user", 6, b"alice")]),
    ("map_any_nested", "access/get_test.go:98-126 (GetMapAny(1): meta -> map, name -> gopher)",
     ("access/get_test.go", 99), [1], 1, [(b"meta", 7, INNER_MAP), (b"name", 6, b"gopher")]),
    ("map_any_inner", "access/get_test.go:98-126 (m[\"meta\"]: role -> admin, user -> alice)",
     ("access/get_test.go", 99), [1, 1], 1, [(b"role", 6, b"admin"), (b"user", 6, b"alice")]),
]

SEQ = [
    ("seq_nested_map", "access/seqget_test.go:11-101", ("access/seqget_test.go", 12)),
    ("seq_flat_end", "access/seqget_test.go:103-151", ("access/seqget_test.go", 104)),
]

# schema.DecodeBuffer known answers over bytes produced by the encoders above
DECODE = [
    ("decode_packed_structure", "schema/schema_test.go:244-316", "schema_packed_structure",
     [I16, F32T, I64, BOOL, MAP(EX("meta"), MAP(EX("role"), {"type": "bytes", "width": 5},
                                               EX("user"), {"type": "bytes", "width": 5}),
                               EX("name"), {"type": "string", "width": 6})],
     [12345, F32(3.14), 9876543210, True, {"meta": {"role": B("admin"), "user": B("alice")},
                                          "name": S("gopher")}], 0),
    ("decode_two_tuples", "schema/schema_test.go:363-404", "pack_two_tuples34",
     [TUP(I32, BOOL, {"type": "string", "width": 2}), TUP(I16, BOOL, {"type": "string", "width": 2})],
     [[2025, False, S("az")], [7, True, S("go")]], 0),
    ("decode_named_tuples", "schema/schema_test.go:478-531 (DecodeBufferNamed)", "pack_two_tuples34",
     {"type": "chain", "fieldNames": ["firstTuple", "secondTuple"], "schema": [
         TUP(I32, BOOL, {"type": "string", "width": 2}, names=["year", "flag", "code"]),
         TUP(I16, BOOL, {"type": "string", "width": 2}, names=["num", "flag", "lang"])]},
     {"firstTuple": {"year": 2025, "flag": False, "code": S("az")},
      "secondTuple": {"num": 7, "flag": True, "lang": S("go")}}, 0),
    ("decode_extra_tuples_ignored", "schema/schema_test.go:559-610", "pack_four_tuples",
     [TUP(I32, BOOL, {"type": "string", "width": 2}), TUP(I16, BOOL, {"type": "string", "width": 2})],
     [[2025, False, S("az")], [7, True, S("go")]], 0),
    # derived (schema.go:1607): STuple() with no schemas skips the arg-count
    # check (argCount > 0 guard), so a 1-field tuple decodes as an empty one
    ("derived_unnamed_empty_tuple_any_count", "derived: schema/schema.go:1604-1609", "pack_one_tuple_int16",
     [TUP()], [[]], 0),
    # derived (schema.go:1773-1775): STupleNamed(nil) has no such guard:
    # 1 field != 0 schemas -> ErrConstraintViolated at position 0
    ("derived_named_nil_tuple_count", "derived: schema/schema.go:1766-1775", "pack_one_tuple_int16",
     [TUP(names=[])], None, (3 | (1 << 8))),
    # derived (schema.go:1756-1758): a named tuple whose FieldNames and
    # Schemas differ in length fails before precheck, at position 0 even as
    # the second field of the chain
    ("derived_named_names_mismatch", "derived: schema/schema.go:1756-1758", "pack_two_tuples34",
     [TUP(I32, BOOL, {"type": "string", "width": 2}),
      TUP(I16, BOOL, {"type": "string", "width": 2}, names=["num", "flag"])], None, (3 | (1 << 8))),
    # derived (schema.go:948-956): DecodeBufferNamed fails every blob that
    # NewSeqGetAccess accepts when len(FieldNames) != len(Schemas), with
    # ErrConstraintViolated at position -1 -- fewer names and more names
    ("derived_named_chain_fewer_names_decode", "derived: schema/schema.go:948-956", "pack_two_tuples34",
     {"type": "chain", "fieldNames": ["firstTuple"], "schema": [
         TUP(I32, BOOL, {"type": "string", "width": 2}), TUP(I16, BOOL, {"type": "string", "width": 2})]},
     None, 3),
    ("derived_named_chain_more_names_decode", "derived: schema/schema.go:948-956", "pack_two_tuples34",
     {"type": "chain", "fieldNames": ["firstTuple", "secondTuple", "third"], "schema": [
         TUP(I32, BOOL, {"type": "string", "width": 2}), TUP(I16, BOOL, {"type": "string", "width": 2})]},
     None, 3),
    ("decode_empty_tuples2", "schema/schema_test.go:840-869", "schema_empty_tuples2",
     [I16, TUP(STR, STR, STR), TUP(), TUP(STR, names=["ok"]), TUP(names=[]), I16],
     [5, None, None, None, None, 5], 0),
    # wrong width for "admin": SBytes(6) -> error (ValidateBuffer fails; DecodeBuffer
    # reports the SMap at top-level position 4 wrapping ErrInvalidFormat)
    ("decode_failure_width", "schema/schema_test.go:52-89", "schema_packed_structure",
     [I16, F32T, I64, BOOL, MAP(EX("meta"), MAP(EX("role"), {"type": "bytes", "width": 6},
                                               EX("user"), {"type": "bytes", "width": 5}),
                               EX("name"), {"type": "string", "width": 6})],
     None, (1 | (5 << 8))),
    # TestDecodePackedStructure's own schema: SInt16.RangeValues(0, 20000)
    ("decode_packed_structure_range", "schema/schema_test.go:244-316", "schema_packed_structure",
     [I16R, F32T, I64, BOOL, PACKED_MAP], PACKED_ROW, 0),
    # TestDecodeChain_DateEmailPrefixSuffix_Success minus the two Pattern
    # (regexp) checks, which are outside the compiled subset and pass here
    ("decode_range_prefix_suffix", "schema/schema_test.go:405-443 (Pattern checks dropped)",
     "pack_date_range_email_prefix_suffix",
     [STR, I32R, STR, {"type": "string", "prefix": "prefix-"}, {"type": "string", "suffix": "-suffix"}],
     [S("2025-09-10"), 42, S("alice@example.com"), S("prefix-hello"), S("world-suffix")], 0),
    # TestDecodeChain_Default_Success minus the Pattern checks: empty payloads
    # decode as the DefaultDecodeValue, which then passes Prefix / Suffix
    ("decode_defaults", "schema/schema_test.go:445-483 (Pattern checks dropped)", "pack_defaults_empty",
     [STR, I32R, {"type": "string", "decodeDefault": "alice@example.com"},
      {"type": "string", "decodeDefault": "prefix-hello", "prefix": "prefix-"},
      {"type": "string", "decodeDefault": "world-suffix", "suffix": "-suffix"}],
     [S("2025-09-10"), 42, S("alice@example.com"), S("prefix-hello"), S("world-suffix")], 0),
    # derived (schema.go:1187-1201): 12345 outside RangeValues(0, 10000) ->
    # ErrOutOfRange at top-level position 0
    ("derived_range_violation", "derived: schema/schema.go:1187-1201", "schema_packed_structure",
     [{"type": "int16", "min": 0, "max": 10000}, F32T, I64, BOOL, PACKED_MAP], None, (13 | (1 << 8))),
    # derived (schema.go:1093-1108, 1144-1150): "prefix-hello" lacks "xyz-" ->
    # ErrStringPrefix at position 3
    ("derived_prefix_violation", "derived: schema/schema.go:1093-1108,1144-1150",
     "pack_date_range_email_prefix_suffix",
     [STR, I32R, STR, {"type": "string", "prefix": "xyz-"}, STR], None, (6 | (4 << 8))),
    # derived (schema.go:1152-1158): suffix mismatch -> ErrStringSuffix at 4
    ("derived_suffix_violation", "derived: schema/schema.go:1152-1158",
     "pack_date_range_email_prefix_suffix",
     [STR, I32R, STR, STR, {"type": "string", "suffix": "-nope"}], None, (7 | (5 << 8))),
    # derived (schema.go:2197-2210, 997-1013): a date (int64, not nullable)
    # schema over the 4-byte int32 field fails precheck's width test before
    # any range check: ErrConstraintViolated at position 1
    ("derived_date_width", "derived: schema/schema.go:2197-2210", "pack_date_range_email_prefix_suffix",
     [STR, {"type": "date", "dateFrom": "1970-01-01T00:01:00Z", "dateTo": "2000-01-01T00:00:00Z"}, STR, STR, STR],
     None, (3 | (2 << 8))),
    # TestSDate_SuccessAndNullable (DecodeBuffer legs): the date decodes, the
    # nil payload decodes as nil, 2050 fails ErrDateOutOfRange at position 0
    ("decode_sdate_in_range", "schema/schema_test.go:1361-1375", "pack_date_2025", [SDATE_2020_2030],
     [1757462400], 0),
    ("decode_sdate_nil", "schema/schema_test.go:1376-1384", "pack_nullable_int64_nil", [SDATE_2020_2030],
     [None], 0),
    ("decode_sdate_out_of_range", "schema/schema_test.go:1385-1393", "pack_date_2050", [SDATE_2020_2030],
     None, (14 | (1 << 8))),
    # derived: the ValidateBuffer/DecodeBuffer divergences (VALIDATE below)
    # SInt16(nullable) over a 1-byte Integer: DecodeBuffer panics in
    # binary.LittleEndian.Uint16 (schema.go:649-657)
    ("derived_short_nullable_int16", "derived: schema/schema.go:649-657", "pack_int8_7",
     [{"type": "int16", "nullable": True}], None, (0x40000000 | (1 << 8))),
    # SString.Optional().Suffix over "": DecodeFunc tests the empty string
    # (schema.go:1093-1108): ErrStringSuffix at position 6
    ("derived_optional_suffix_empty", "derived: schema/schema.go:1093-1108 over schema_test.go:187-207",
     "pack_optional_email_seven", SEVEN_SCHEMA, None, (7 | (7 << 8))),
    # SMap with an odd schema count: SizeExact -> ErrConstraintViolated at 4
    # (schema.go:369-377)
    ("derived_odd_map_decode", "derived: schema/schema.go:369-377", "schema_packed_structure",
     [I16, F32T, I64, BOOL, MAP(EX("meta"), MAP(EX("role"), {"type": "bytes", "width": 5},
                                               EX("user"), {"type": "bytes", "width": 5}), EX("name"))],
     None, (3 | (5 << 8))),
    # SString.Match("x") over "": DecodeFunc tests the empty string
    # (schema.go:1093-1108, 1136-1142): ErrStringMatch at position 2
    ("derived_match_empty_decode", "derived: schema/schema.go:1093-1108,1136-1142", "pack_defaults_empty",
     [STR, I32, {"type": "string", "exact": "x"}, STR, STR], None, (9 | (3 << 8))),
]

# schema.ValidateBuffer known answers (status only; the Validate methods'
# rules, schema.go:880-891).  Pattern / SEmail / SMapUnordered checks are
# outside the compiled subset: as in DECODE, they are dropped (a plain string)
VALIDATE = [
    ("validate_packed_structure", "schema/schema_test.go:15-50", "schema_packed_structure",
     [I16R, F32T, I64, BOOL, PACKED_MAP], 0),
    # wrong width for "admin": SBytes(6): the inner SMap's precheck fails,
    # wrapped by both maps as ErrInvalidFormat at top-level position 4
    ("validate_packed_structure_failure", "schema/schema_test.go:52-89", "schema_packed_structure",
     [I16, F32T, I64, BOOL, MAP(EX("meta"), MAP(EX("role"), {"type": "bytes", "width": 6},
                                               EX("user"), {"type": "bytes", "width": 5}),
                               EX("name"), {"type": "string", "width": 6})], (1 | (5 << 8))),
    ("validate_prefix_suffix", "schema/schema_test.go:166-185 (Pattern checks dropped)",
     "pack_date_range_email_prefix_suffix",
     [STR, I32R, STR, {"type": "string", "prefix": "prefix-"}, {"type": "string", "suffix": "-suffix"}], 0),
    # SString.Optional().Suffix("-suffix") over "" passes Validate
    # (schema.go:1085-1087); SEmail / Pattern dropped
    ("validate_optional_suffix_empty", "schema/schema_test.go:187-211 (SEmail / Pattern dropped)",
     "pack_optional_email_seven", SEVEN_SCHEMA, 0),
    ("validate_packed_tuples", "schema/schema_test.go:213-242", "pack_two_tuples34",
     [TUP(I32, BOOL, {"type": "string", "width": 2}), TUP(I16, BOOL, {"type": "string", "width": 2})], 0),
    ("validate_sdate_in_range", "schema/schema_test.go:1361-1368", "pack_date_2025", [SDATE_2020_2030], 0),
    ("validate_sdate_nil", "schema/schema_test.go:1376-1379", "pack_nullable_int64_nil", [SDATE_2020_2030], 0),
    ("validate_sdate_out_of_range", "schema/schema_test.go:1385-1389", "pack_date_2050", [SDATE_2020_2030],
     (14 | (1 << 8))),
    # derived: SInt16(nullable).Validate = validatePrimitive, which never reads
    # the payload (schema.go:646-648): a 1-byte Integer passes
    ("derived_validate_short_nullable_int16", "derived: schema/schema.go:646-648", "pack_int8_7",
     [{"type": "int16", "nullable": True}], 0),
    # derived: SDateRange's ValidateFunc reads the payload like its DecodeFunc
    # (schema.go:2198-2212): a 4-byte payload under a nullable date panics in both
    ("derived_validate_short_date_panics", "derived: schema/schema.go:2198-2212",
     "pack_date_range_email_prefix_suffix", [STR, {"type": "date", "nullable": True}, STR, STR, STR],
     (0x40000000 | (2 << 8))),
    # derived: SchemaMap.Validate has no odd-count check (schema.go:336-359):
    # the three schemas validate in sequence over the four fields
    ("derived_validate_odd_map", "derived: schema/schema.go:336-359", "schema_packed_structure",
     [I16, F32T, I64, BOOL, MAP(EX("meta"), MAP(EX("role"), {"type": "bytes", "width": 5},
                                               EX("user"), {"type": "bytes", "width": 5}), EX("name"))], 0),
    # derived: Match over "" passes ValidateFunc (nullable receiver SString)
    ("derived_validate_match_empty", "derived: schema/schema.go:1072-1091,1136-1142",
     "pack_defaults_empty", [STR, I32, {"type": "string", "exact": "x"}, STR, STR], 0),
]


def main():
    if not os.path.isdir(REF):
        sys.exit("reference not present; vectors.json is already committed")
    out = {"note": __doc__.strip().split("\n")[0], "encode": [], "equal": [], "get": [], "maps": [], "seq": [],
           "inputs": [], "decode": []}
    for cid, src, mode, schema, row, (bf, bl) in ENCODE:
        out["encode"].append({"id": cid, "source": src, "mode": mode, "schema": schema, "row": row,
                              "bytes_from": f"{bf}:{bl}", "hex": extract_bytes(bf, bl).hex()})
    for cid, src, variants, row in EQUAL:
        out["equal"].append({"id": cid, "source": src, "row": row,
                             "variants": [{"mode": m, "schema": s} for m, s in variants]})
    for cid, src, (bf, bl), queries in GET:
        out["get"].append({"id": cid, "source": src, "bytes_from": f"{bf}:{bl}",
                           "hex": extract_bytes(bf, bl).hex(),
                           "queries": [{"path": p, "tag": t, "width": w, "expect": e}
                                       for p, t, w, e in queries]})
    for cid, src, (bf, bl), path, flags, pairs in MAPS:
        out["maps"].append({"id": cid, "source": src, "bytes_from": f"{bf}:{bl}",
                            "hex": extract_bytes(bf, bl).hex(), "path": path, "flags": flags,
                            "pairs": [[k.hex(), t, v.hex()] for k, t, v in pairs]})
    for cid, src, (bf, bl) in SEQ:
        out["seq"].append({"id": cid, "source": src, "bytes_from": f"{bf}:{bl}",
                           "hex": extract_bytes(bf, bl).hex()})
    for cid, src, mode, schema, row in INPUTS:
        out["inputs"].append({"id": cid, "source": src, "mode": mode, "schema": schema, "row": row})
    for cid, src, from_case, schema, row, status in DECODE:
        out["decode"].append({"id": cid, "source": src, "input_from": from_case, "schema": schema,
                              "expect_row": row, "expect_status": status})
    out["validate"] = []
    for cid, src, from_case, schema, status in VALIDATE:
        out["validate"].append({"id": cid, "source": src, "input_from": from_case, "schema": schema,
                                "expect_status": status})
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {OUT}: {len(out['encode'])} encode, {len(out['equal'])} equal, "
          f"{len(out['get'])} get, {len(out['maps'])} maps, {len(out['seq'])} seq, {len(out['inputs'])} inputs, {len(out['decode'])} decode, "
          f"{len(out['validate'])} validate")


if __name__ == "__main__":
    main()
