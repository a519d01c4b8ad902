"""libpackos.so host-side checks (no GPU): the C ABI loads, exports every
symbol include/packos.h declares, and the schema compiler's layout agrees
with the oracle on blob sizes."""
import ctypes as C
import json
import os
import re

import numpy as np
import pytest

import oracle_bridge as ob
from golden_util import MODES, chain_of, load, unwrap
from packos_amd import _lib
from packos_amd.api import CompiledSchema
from packos_amd.columns import HostColumns
from packos_amd.configs import CONFIGS, make_columns
from schema_gen import rand_chain, rand_rows

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_exports_match_header():
    hdr = open(os.path.join(ROOT, "include", "packos.h")).read()
    declared = set(re.findall(r"\b(packos_[a-z_]+)\s*\(", hdr))
    declared -= {"packos_column", "packos_schema"}
    L = _lib.lib()
    for name in sorted(declared):
        assert hasattr(L, name), f"{name} declared in packos.h but not exported"
    assert set(_lib.EXPORTED) == declared
    assert L.packos_abi_version() == 4


def test_schema_errors():
    L = _lib.lib()
    h = C.c_void_p()
    assert L.packos_schema_compile(b"[{\"type\":\"email\"}]", 0, C.byref(h)) == -3
    assert b"outside" in L.packos_last_error()
    # map keys must be strings (the compiled subset)
    assert L.packos_schema_compile(b"[{\"type\":\"map\",\"schema\":[{\"type\":\"int16\"},{\"type\":\"int16\"}]}]",
                                   0, C.byref(h)) == -2
    # an odd SMap schema count compiles (Validate accepts it, schema.go:336-359);
    # encode of a present value fails, so the schema needs a status array
    assert L.packos_schema_compile(b"[{\"type\":\"map\",\"schema\":[{\"type\":\"string\"}]}]", 0,
                                   C.byref(h)) == 0
    assert L.packos_schema_has_checks(h) == 1
    L.packos_schema_free(h)
    assert L.packos_schema_compile(b"[{\"type\":", 0, C.byref(h)) == -2
    assert L.packos_schema_compile(b"[{\"type\":\"string\",\"pattern\":\"^a\"}]", 0, C.byref(h)) == -3
    assert L.packos_schema_compile(b"[{\"type\":\"int16\",\"min\":0.5}]", 0, C.byref(h)) == -2
    assert L.packos_schema_compile(b"[{\"type\":\"uint16\",\"min\":0}]", 0, C.byref(h)) == -3
    assert L.packos_schema_compile(b"[]", 7, C.byref(h)) == -1


def test_config_blob_sizes():
    assert CompiledSchema(CONFIGS["M"].chain).fixed_blob_size == 256
    assert CompiledSchema(CONFIGS["C1"].chain).fixed_blob_size == 17
    assert CompiledSchema(CONFIGS["C2"].chain).fixed_blob_size == 64
    assert CompiledSchema(CONFIGS["C4"].chain).fixed_blob_size == 256
    assert CompiledSchema(CONFIGS["C3"].chain).fixed_blob_size == -1
    assert CompiledSchema(CONFIGS["C5"].chain).fixed_blob_size == -1


def test_decode_fast_eligibility_configs():
    fast = {k: CompiledSchema(c.chain, c.mode).decode_fast for k, c in CONFIGS.items()}
    assert fast == {"M": True, "C1": True, "C2": True, "C3": False, "C4": True, "C5": False, "X1": False}
    from packos_amd.schema import SChain, STuple, SInt32
    # a present empty tuple is written as 10 00, which DecodeBuffer rejects
    assert not CompiledSchema(SChain(SInt32, STuple())).decode_fast


@pytest.mark.parametrize("seed", range(60))
def test_decode_fast_eligibility_vs_oracle(seed):
    """The compiler qualifies a fixed schema for the tiled decoder by running
    the (host-compiled) device decoder on the canonical blob; that must agree
    with the oracle's DecodeBuffer on an all-present blob of the schema."""
    chain = rand_chain(seed, allow_var=False)
    s = CompiledSchema(chain, 0)
    B = s.fixed_blob_size
    hc = HostColumns.from_rows(chain, rand_rows(chain, 1, seed, nil_p=0.0))
    arena, offs, _ = ob.encode(chain, hc, 0)
    _, st = ob.decode(chain, arena, offs, 1)
    depth = max((d for _, d, *_ in chain.walk()), default=0)
    expect = 0 < B <= 1024 and int(st[0]) == 0 and depth < 7
    assert s.decode_fast == expect, (B, hex(int(st[0])), depth)


def test_column_info_named():
    s = CompiledSchema(CONFIGS["C3"].chain)
    assert s.n_columns == 7
    info = [s.column_info(c) for c in range(7)]
    assert [i["name"] for i in info] == ["id", "ts", "score", "flag", "label", "code", "digest"]
    assert info[4]["width"] == 0 and info[4]["kind"] == "string"
    assert info[5]["width"] == 8


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("seed", range(40))
def test_blob_sizes_vs_oracle(seed, mode):
    chain = rand_chain(seed)
    rows = rand_rows(chain, 20, seed + 1000)
    hc = HostColumns.from_rows(chain, rows)
    s = CompiledSchema(chain, mode)
    _, offs, _ = ob.encode(chain, hc, mode)
    sizes = np.diff(offs.astype(np.int64))
    widths = hc.var_widths()
    for i in range(hc.n):
        valid = np.ones(len(hc.specs), np.uint8)
        for c in range(len(hc.specs)):
            if hc.valid[c] is not None:
                valid[c] = hc.valid[c][i]
        assert s.blob_size_host(widths[i], valid) == sizes[i], (seed, i, s.describe())


def test_golden_schemas_compile():
    g = load()
    for case in g["encode"]:
        s = CompiledSchema(chain_of(case["schema"]), MODES[case["mode"]])
        hc = HostColumns.from_rows(s.chain, [unwrap(case["row"])])
        widths = hc.var_widths()[0]
        valid = np.ones(len(hc.specs), np.uint8)
        for c in range(len(hc.specs)):
            if hc.valid[c] is not None:
                valid[c] = hc.valid[c][0]
        assert s.blob_size_host(widths, valid) == len(case["hex"]) // 2, case["id"]


@pytest.mark.parametrize("seed", range(40))
def test_checked_schema_bounds_match_compiler(seed):
    """The compiler's value checks (describe(): min/max/flags in emission
    order) equal the Python schema tree's, through the SchemaJSON text
    (RFC3339 dates for SDateRange, int64 min/max for Range)."""
    from schema_gen import rand_checked_chain
    chain = rand_checked_chain(seed)
    got = [tuple(int(kv.split("=")[1]) for kv in l.split()[4:7])
           for l in CompiledSchema(chain).describe().split("\n") if l.startswith("check ")]
    # a named tuple whose names and schemas differ in length adds a CHK_FAIL
    # (64) check ahead of its children's (schema.go:1808-1810)
    want = [(n.check, n.rmin, n.rmax) if n.kind != "tuple" else (64, 0, 0)
            for n, *_ in chain.walk()
            if n.check & 0x1B or (n.kind == "tuple" and n.names is not None and len(n.names) != len(n.children))]
    assert got == want


def test_rfc3339_dates():
    from packos_amd.schema import SDateRange, _parse_rfc3339
    L = _lib.lib()
    for txt, unix in [("2025-09-10T00:00:00Z", 1757462400), ("0913-11-12T02:00:13Z", -33328447187),
                      ("1970-01-01T01:00:00+01:00", 0), ("2000-02-29T12:00:00.75-05:30", 951845400),
                      ("913-11-12T02:00:13Z", -62135596800), ("2001-02-29T00:00:00Z", -62135596800),
                      ("bad", -62135596800)]:
        assert _parse_rfc3339(txt) == unix, txt
        s = CompiledSchema(json.dumps([{"type": "date", "dateFrom": txt, "dateTo": txt}]))
        line = next(l for l in s.describe().split("\n") if l.startswith("check "))
        assert f"min={unix} max={unix}" in line, (txt, line)


def test_flatten_tuple_compiles_as_plain():
    """BuildSchema's "flatten" (STupleValFlatten / STupleNamedValFlattened,
    schemabuilder_json.go:247-258) differs from the plain variable tuple only
    for SRepeatSchema children (schema.go:1616-1623): same compiled layout."""
    from packos_amd.schema import BuildChain
    kids = [{"type": "int32"}, {"type": "string"}, {"type": "bytes", "width": 4}]
    for named in (False, True):
        base = {"type": "tuple", "schema": kids, "variableLength": True}
        if named:
            base["fieldNames"] = ["a", "b", "c"]
        flat = dict(base, flatten=True)
        js_plain, js_flat = json.dumps([{"type": "int16"}, base]), json.dumps([{"type": "int16"}, flat])
        a, b = CompiledSchema(js_plain), CompiledSchema(js_flat)
        assert a.describe() == b.describe()
        assert BuildChain(js_flat).Schemas[1].flatten and b.chain.to_json()[1]["flatten"] is True
    # without variableLength, BuildSchema ignores "flatten" (plain STuple)
    js = json.dumps([{"type": "tuple", "schema": kids, "flatten": True}])
    assert not BuildChain(js).Schemas[0].flatten
    assert CompiledSchema(js).describe() == CompiledSchema(json.dumps([{"type": "tuple", "schema": kids}])).describe()


def test_has_checks():
    assert not CompiledSchema(CONFIGS["M"].chain).has_checks
    assert CompiledSchema(json.dumps([{"type": "int16", "min": 0, "max": 9}])).has_checks
    assert CompiledSchema(json.dumps([{"type": "string", "prefix": "ab"}])).has_checks
    assert not CompiledSchema(json.dumps([{"type": "string", "decodeDefault": "x"}])).has_checks


def test_get_batch_span_outputs_optional_only_for_typed_gathers():
    """packos_get_batch argument rules, checked before any device work (n = 0):
    start / len / tag may be NULL only when a typed value (out_values) carries
    the result; SPAN / ANY / no gather with NULL spans -> PACKOS_E_INVALID."""
    L = _lib.lib()
    path = (C.c_int32 * 1)(0)
    st = (C.c_uint8 * 4)()
    vals = (C.c_uint8 * 32)()
    s0 = (C.c_uint64 * 4)()
    ln = (C.c_uint32 * 4)()
    tg = (C.c_uint8 * 4)()
    arena = (C.c_uint8 * 16)()
    GET_SPAN, GET_INT, GET_ANY = 2, 3, 5
    call = lambda g, v, spans: L.packos_get_batch(arena, None, 16, 0, path, 1, g, 0, 0, v, 8 if v else 0,  # noqa: E731
                                                  *((s0, ln, tg) if spans else (None, None, None)), st, None)
    assert call(GET_INT, vals, False) == 0
    assert call(GET_INT, vals, True) == 0
    assert call(GET_SPAN, None, True) == 0
    assert call(GET_SPAN, None, False) == -1
    assert call(GET_ANY, None, False) == -1
    assert call(GET_INT, None, False) == -1


def test_json_marshal_shaped_schema_compiles():
    """The text Go's json.Marshal makes of []schema.SchemaJSON
    (schemabuilder_json.go:8-30): omitempty keys absent, "extra" holding any
    JSON (objects, arrays, null, floats) that BuildSchema never reads.  Same
    columns and layout as the bare schema."""
    extra = {"label": "id", "order": 1, "tags": ["a", "b"], "ui": {"step": 0.5, "hidden": False, "hint": None}}
    marshalled = json.dumps([{"type": "int16", "extra": extra}, {"type": "bool"}, {"type": "string"},
                             {"type": "bytes", "extra": {}}], separators=(",", ":"))
    bare = json.dumps([{"type": "int16"}, {"type": "bool"}, {"type": "string"}, {"type": "bytes"}])
    a, b = CompiledSchema(marshalled), CompiledSchema(bare)
    assert a.describe() == b.describe()
