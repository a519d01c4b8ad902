"""Pin the CPU oracle to the reference's own golden vectors (CPU only).

Every byte vector comes from the reference test sources via
tests/golden/make_golden.py; a failure here means the oracle is not a faithful
restatement and no GPU parity claim can rest on it.
"""
import json

import numpy as np
import pytest

from packos_amd.api import VIEW_DEFAULT

import oracle_bridge as ob
from golden_util import MODES, chain_of, load, unwrap
from packos_amd.columns import HostColumns, column_specs

G = load()


def _encode_one(schema_json, row, mode):
    chain = chain_of(schema_json)
    hc = HostColumns.from_rows(chain, [unwrap(row)])
    arena, offs, st = ob.encode(chain, hc, mode)
    return bytes(arena[int(offs[0]):int(offs[1])]), int(st[0])


@pytest.mark.parametrize("case", G["encode"], ids=[c["id"] for c in G["encode"]])
def test_encode_golden(case):
    got, st = _encode_one(case["schema"], case["row"], MODES[case["mode"]])
    assert got.hex() == case["hex"], f"{case['id']} ({case['source']})"
    assert st == 0


@pytest.mark.parametrize("case", G["equal"], ids=[c["id"] for c in G["equal"]])
def test_cross_api_equal(case):
    res = [_encode_one(v["schema"], case["row"], MODES[v["mode"]]) for v in case["variants"]]
    for o, st in res:
        assert o == res[0][0], f"{case['id']} ({case['source']})"
        assert st == 0


def test_empty_tuple_bytes():
    # schema_test.go:820: EncodeValue(nil, nil tuples) == Pack(PackTuple(), PackTuple())
    case = next(c for c in G["equal"] if c["id"] == "schema_empty_tuples1")
    got, _ = _encode_one(case["variants"][0]["schema"], case["row"], 0)
    assert got == bytes.fromhex("340004000000")


@pytest.mark.parametrize("case", G["get"], ids=[c["id"] for c in G["get"]])
def test_getaccess_golden(case):
    buf = np.frombuffer(bytes.fromhex(case["hex"]), np.uint8)
    offs = np.asarray([0, buf.size], np.uint64)
    for q in case["queries"]:
        s0, ln, tg, st = ob.get_field_batch(buf, offs, 1, q["path"], q["tag"], q["width"])
        assert st[0] == 0, q
        assert bytes(buf[int(s0[0]):int(s0[0]) + int(ln[0])]).hex() == q["expect"], q


def test_getaccess_wrong_type_and_width():
    case = next(c for c in G["get"] if c["id"] == "get_flat")
    buf = np.frombuffer(bytes.fromhex(case["hex"]), np.uint8)
    offs = np.asarray([0, buf.size], np.uint64)
    # GetInt32(0) on an int16 field -> decode error (tag ok, width 2 != 4)
    assert ob.get_field_batch(buf, offs, 1, [0], 1, 4)[3][0] == 1
    # GetBool(0) -> wrong tag
    assert ob.get_field_batch(buf, offs, 1, [0], 5, 1)[3][0] == 1
    # position past argCount -> rangeAt returns TypeEnd
    assert ob.get_field_batch(buf, offs, 1, [4], 1, 2)[3][0] == 1
    # nested access on a scalar -> "it's not nested type"
    assert ob.get_field_batch(buf, offs, 1, [0, 0], 6, -1)[3][0] == 1


def pack_fields(fields):
    """Lay fields [(tag, bytes)] out in the wire format (header block of
    uint16 offset<<3|tag, End entry holding the payload length;
    pack.go:9-60): h0 is absolute, later offsets relative to the payload."""
    base = 2 * (len(fields) + 1)
    hdr, pay = [], b""
    for i, (tag, b) in enumerate(fields):
        hdr.append(((base if i == 0 else len(pay)) << 3) | tag)
        pay += b
    hdr.append(len(pay) << 3)
    return b"".join(h.to_bytes(2, "little") for h in hdr) + pay


# Integer int16, nil Integer, Floating f32, Bool 7, String, nil Floating,
# 3-byte Integer, Integer int8 -5
NIL_FIELDS = [(1, (-300).to_bytes(2, "little", signed=True)), (1, b""), (3, bytes.fromhex("0000c03f")),
              (5, b"\x07"), (6, b"abc"), (3, b""), (1, b"\x01\x02\x03"), (1, bytes([0xFB]))]


@pytest.mark.parametrize("path,getter,tag,width,status,value", [
    ([1], 1, 1, 4, 4, None),            # GetNullableInt32 on nil -> nil, no error
    ([1], 1, 5, 1, 4, None),            # GetNullableBool on a nil Integer: nil before the tag check
    ([1], 0, 1, 4, 1, None),            # GetInt32 on nil -> width error
    ([0], 1, 1, 2, 0, "d4fe"),          # GetNullableInt16 on a value
    ([0], 3, 0, 0, 0, "d4feffffffffffff"),  # GetInt -> int16 sign-extended
    ([7], 3, 0, 0, 0, "fbffffffffffffff"),  # GetInt -> int8 -5
    ([6], 3, 0, 0, 1, None),            # GetInt on a 3-byte integer -> error
    ([1], 3, 0, 0, 4, None),            # GetInt on nil -> nil
    ([2], 3, 0, 0, 1, None),            # GetInt on Floating -> tag error
    ([2], 4, 0, 0, 0, "0000c03f00000000"),  # GetFloating -> float32 bits
    ([5], 4, 0, 0, 4, None),            # GetFloating on nil -> nil
    ([3], 0, 5, 1, 0, "01"),            # GetBool normalises to 0/1
    ([3], 1, 5, 1, 0, "01"),            # GetNullableBool
    ([4], 2, 6, 0, 0, None),            # GetString span
    ([5], 2, 6, 0, 1, None),            # GetBytes on a Floating -> tag error
    ([9], 1, 1, 4, 1, None),            # past argCount: TypeEnd, width -1 -> tag error
])
def test_get_batch_getters(path, getter, tag, width, status, value):
    blob = pack_fields(NIL_FIELDS)
    buf = np.frombuffer(blob, np.uint8)
    vals, s0, ln, tg, st = ob.get_batch(buf, np.asarray([0, len(blob)], np.uint64), 1, path, getter, tag, width)
    assert st[0] == status
    if value is not None:
        assert bytes(vals[0]).hex() == value
    if getter == 2 and status == 0:
        assert bytes(buf[int(s0[0]):int(s0[0]) + int(ln[0])]) == b"abc"


@pytest.mark.parametrize("path,status,tag,payload", [
    ([0], 0, 1, (-300).to_bytes(2, "little", signed=True)),   # GetTypeAndValue: any tag
    ([1], 0, 1, b""),                                          # nil value: empty, not invalid
    ([4], 0, 6, b"abc"),
    ([9], 3, 0, None),                                         # past argCount: buf[-2:-1] panics
])
def test_get_any_type_and_value(path, status, tag, payload):
    """GetTypeAndValue (access/get.go:504-510): (tag, buf[start:end]) for any
    tag; TypeInvalid + nil only when end < start (derived: no reference test
    calls it)."""
    blob = pack_fields(NIL_FIELDS)
    buf = np.frombuffer(blob, np.uint8)
    vals, s0, ln, tg, st = ob.get_batch(buf, np.asarray([0, len(blob)], np.uint64), 1, path, 5)
    assert vals is None and st[0] == status and tg[0] == tag
    if payload is not None:
        assert bytes(buf[int(s0[0]):int(s0[0]) + int(ln[0])]) == payload


@pytest.mark.parametrize("case", [c["id"] for c in G["maps"]])
def test_map_getters_golden(case):
    """GetMapStr / GetMapAny / GetMapOrderedAny known answers of
    access/get_test.go (pairs in wire order, nested map values as spans)."""
    c = next(x for x in G["maps"] if x["id"] == case)
    buf = np.frombuffer(bytes.fromhex(c["hex"]), np.uint8)
    offs = np.asarray([0, buf.size], np.uint64)
    pr, ks, kl, vs, vl, vt, st = ob.get_map_batch(buf, offs, 1, c["path"], c["flags"], 4)
    assert st[0] == 0 and pr[0] == len(c["pairs"])
    got = [(bytes(buf[int(ks[0, j]):int(ks[0, j]) + int(kl[0, j])]).hex(), int(vt[0, j]),
            bytes(buf[int(vs[0, j]):int(vs[0, j]) + int(vl[0, j])]).hex()) for j in range(pr[0])]
    assert got == [tuple(p) for p in c["pairs"]]
    # max_pairs smaller than the map: the first pairs, status 5
    pr, ks, kl, vs, vl, vt, st = ob.get_map_batch(buf, offs, 1, c["path"], c["flags"], 1)
    assert st[0] == 5 and pr[0] == len(c["pairs"])


def _map(pairs):
    """A map container of (key bytes, tag, value bytes) pairs."""
    fields = []
    for k, t, v in pairs:
        fields += [(6, k), (t, v)]
    return pack_fields(fields)


@pytest.mark.parametrize("name,blob,flags,status", [
    # GetMapStr needs String values; GetMapAny takes ints / floats / nested maps
    ("str_int_value", pack_fields([(7, _map([(b"a", 1, b"\x01\x00")]))]), 0, 1),
    ("any_int_value", pack_fields([(7, _map([(b"a", 1, b"\x01\x00")]))]), 1, 0),
    ("any_int3_value", pack_fields([(7, _map([(b"a", 1, b"\x01\x00\x00")]))]), 1, 1),
    ("any_nil_float", pack_fields([(7, _map([(b"a", 3, b"")]))]), 1, 0),
    ("any_bool_value", pack_fields([(7, _map([(b"a", 5, b"\x01")]))]), 1, 1),     # GetAny has no Bool case
    ("any_tuple_value", pack_fields([(7, _map([(b"a", 4, _map([]))]))]), 1, 1),
    ("any_nested_bad", pack_fields([(7, _map([(b"a", 7, _map([(b"k", 5, b"\x00")]))]))]), 1, 1),
    ("any_nested_nil", pack_fields([(7, _map([(b"a", 7, b"")]))]), 1, 0),
    ("key_not_string", pack_fields([(7, pack_fields([(1, b"\x01"), (6, b"v")]))]), 0, 1),
    ("odd_fields", pack_fields([(7, pack_fields([(6, b"k")]))]), 1, 1),
    ("nil_map", pack_fields([(7, b"")]), 0, 4),
    ("not_a_map", pack_fields([(4, _map([]))]), 0, 1),
    ("nested_short", pack_fields([(7, b"\x40\x00")]), 0, 3),   # NewGetAccess -> nil: panic
])
def test_map_getters_rules(name, blob, flags, status):
    """Derived from access/get.go:377-490 (GetAny's tag switch, GetMapStr's
    GetString on keys and values, nil map / nil accessor)."""
    buf = np.frombuffer(blob, np.uint8)
    pr, ks, kl, vs, vl, vt, st = ob.get_map_batch(buf, np.asarray([0, buf.size], np.uint64), 1, [0], flags, 2)
    assert st[0] == status, name
    if status:
        assert int(ks.sum()) == 0 and int(vl.sum()) == 0


def test_seqget_nested_map_golden():
    # access/seqget_test.go:11-101
    case = next(c for c in G["seq"] if c["id"] == "seq_nested_map")
    s = ob.Seq(bytes.fromhex(case["hex"]))
    assert s.err == 0
    p, t, e = s.next()
    assert (p, t, e) == (bytes([0x39, 0x30]), 1, False)
    t, w, e = s.peek()
    assert (t, w, e) == (7, 52, False)
    nested = s.nested()
    assert nested is not None
    p, t, e = nested.next()
    assert (p, t) == (b"meta", 6)
    meta = nested.nested()
    assert meta.next()[:2] == (b"role", 6)
    assert meta.next()[:2] == (b"admin", 6)
    assert nested.advance()
    assert nested.next()[:2] == (b"name", 6)
    assert nested.next()[:2] == (b"gopher", 6)


def test_seqget_flat_end_golden():
    # access/seqget_test.go:103-151: four fields then End -> error
    case = next(c for c in G["seq"] if c["id"] == "seq_flat_end")
    s = ob.Seq(bytes.fromhex(case["hex"]))
    assert s.next()[:2] == (bytes([0x2A, 0x00]), 1)
    assert s.next()[:2] == (bytes([0x01]), 5)
    assert s.next()[:2] == (b"go", 6)
    assert s.next()[:2] == (bytes([0xAA, 0xBB]), 6)
    p, t, err = s.next()
    assert t == 0 and err


def _golden_bytes(case_id):
    for c in G["encode"]:
        if c["id"] == case_id:
            return bytes.fromhex(c["hex"])
    for c in G["inputs"]:
        if c["id"] == case_id:
            return _encode_one(c["schema"], c["row"], MODES[c["mode"]])[0]
    eq = next(c for c in G["equal"] if c["id"] == case_id)
    v = eq["variants"][0]
    return _encode_one(v["schema"], eq["row"], MODES[v["mode"]])[0]


@pytest.mark.parametrize("case", G["decode"], ids=[c["id"] for c in G["decode"]])
def test_decode_golden(case):
    blob = _golden_bytes(case["input_from"])
    chain = chain_of(case["schema"])
    arena = np.frombuffer(blob, np.uint8)
    out, st = ob.decode(chain, arena, np.asarray([0, len(blob)], np.uint64), 1)
    assert int(st[0]) == case["expect_status"], hex(int(st[0]))
    if case["expect_row"] is None:
        return
    # re-encoding the decoded columns must reproduce the expected row's encoding
    exp = HostColumns.from_rows(chain, [unwrap(case["expect_row"])])
    for c, sp in enumerate(column_specs(chain)):
        if sp.fixed:
            valid = exp.valid[c] is None or exp.valid[c][0]
            if valid:
                assert bytes(out.data[c][:sp.width]) == bytes(exp.data[c][:sp.width]), sp.path
        if sp.has_valid:
            assert int(out.valid[c][0]) == int(exp.valid[c][0]), (c, sp.kind)
        if sp.var:
            s0, ln = int(out.start[c][0]), int(out.length[c][0])
            o = exp.offsets[c]
            got = sp.node.default[:ln] if s0 == VIEW_DEFAULT else blob[s0:s0 + ln]
            assert got == bytes(exp.data[c][o[0]:o[1]]), (case["id"], c)


@pytest.mark.parametrize("case", G["validate"], ids=[c["id"] for c in G["validate"]])
def test_validate_golden(case):
    """ValidateBuffer known answers (schema_test.go) and the derived cases
    where Validate's rules differ from DecodeBuffer's."""
    blob = _golden_bytes(case["input_from"])
    chain = chain_of(case["schema"])
    st = ob.validate(chain, np.frombuffer(blob, np.uint8), np.asarray([0, len(blob)], np.uint64), 1)
    assert int(st[0]) == case["expect_status"], hex(int(st[0]))


def test_validate_vs_decode_divergences():
    """Each derived Validate case whose schema also appears in DECODE gives the
    two different answers the reference's two code paths give."""
    dec = {(c["input_from"], json.dumps(c["schema"], sort_keys=True)): c["expect_status"] for c in G["decode"]}
    pairs = 0
    for c in G["validate"]:
        k = (c["input_from"], json.dumps(c["schema"], sort_keys=True))
        if k in dec:
            pairs += 1
            blob = _golden_bytes(c["input_from"])
            chain = chain_of(c["schema"])
            a = np.frombuffer(blob, np.uint8)
            o = np.asarray([0, len(blob)], np.uint64)
            assert int(ob.validate(chain, a, o, 1)[0]) == c["expect_status"]
            assert int(ob.decode(chain, a, o, 1)[1][0]) == dec[k]
    assert pairs >= 6
