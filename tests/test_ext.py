"""ADR-001 extended containers (PACKOS_MODE_EXTENDED, include/packos.h).

A FORMAT EXTENSION beyond the reference: PackOS reserves tag 2
(typetags.TypeExtendedTagContainer, typetags/types.go:11) and links ADR 001
(README.md:34) with no code, test or wire format, so this build defines the
format and parity is **unpinned** for the extended bytes themselves: the
oracle's extended encoder (oracle/packos_oracle.c x_encode, written
independently of its PutAccess / packable restatements) is pinned indirectly —
whenever no container payload exceeds 8191 bytes it must reproduce the
reference-pinned plain bytes exactly, which the CPU tests below check — and the
extended layout is checked against hand-built vectors from the spec.

CPU tests (oracle only) run everywhere; GPU tests compare libpackos with the
oracle bit for bit.
"""
import random

import numpy as np
import pytest

import oracle_bridge as ob
from packos_amd.columns import HostColumns
from packos_amd.schema import (SBool, SChain, SInt16, SInt32, SInt64, SMapSorted, SString, SStringLen,
                               STuple, SVariableBytes, SVariableString, SBytes)
from schema_gen import rand_chain, rand_rows

EXT = ob.MODE_EXTENDED
BIG = [0, 5, 2000, 5000, 8185, 8191, 8192, 9000, 17000]


def big_rows(chain, n, seed, p=0.35, nil_p=0.15):
    """rand_rows with some var strings / bytes made long enough (up to 17 KB)
    that their containers pass 8191 bytes."""
    rows = rand_rows(chain, n, seed, nil_p)
    rng = random.Random(seed * 7 + 1)

    def fix(node, v):
        k = node.kind
        if k in ("string", "bytes") and node.width <= 0 and v is not None and rng.random() < p:
            L = rng.choice(BIG)
            return "".join(chr(rng.randint(0x20, 0x7E)) for _ in range(L)) if k == "string" else rng.randbytes(L)
        if k in ("tuple", "map") and v is not None:
            return [fix(ch, x) for ch, x in zip(node.children, v)]
        return v

    return [[fix(s, v) for s, v in zip(chain.Schemas, r)] for r in rows]


def u16(v):
    return int(v).to_bytes(2, "little")


def u32(v):
    return int(v).to_bytes(4, "little")


def hdr(off, tag):
    return u16(((off << 3) & 0xFFFF) | tag)


def ext_block(own_tag, tags, starts, pay_len):
    """the spec's extended header block for fields with these tags / starts"""
    n = len(tags)
    b = u16(0x0002) + u16(own_tag) + u32(((4 + 4 * (n + 1)) << 3) | tags[0])
    for j in range(1, n):
        b += u32((starts[j] << 3) | tags[j])
    return b + u32(pay_len << 3)


def enc(chain, rows, mode):
    hc = HostColumns.from_rows(chain, rows)
    return ob.encode(chain, hc, mode, nthreads=8)


# ----------------------------------------------------------------- CPU -----
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("seed", range(30))
def test_ext_oracle_equals_plain_below_8k(seed, mode):
    """No payload over 8191 bytes: extended mode == the reference bytes."""
    chain = rand_chain(seed)
    hc = HostColumns.from_rows(chain, rand_rows(chain, 200, seed + 5))
    a0, o0, s0 = ob.encode(chain, hc, mode, nthreads=8)
    a1, o1, s1 = ob.encode(chain, hc, mode | EXT, nthreads=8)
    assert np.array_equal(o0, o1) and np.array_equal(a0, a1)
    assert not (s1 & 0x80000000).any()


@pytest.mark.parametrize("mode", [0, 1])
def test_ext_known_flat(mode):
    chain = SChain(SInt16, SVariableBytes())
    payload = bytes(range(256)) * 36   # 9216 bytes
    arena, offs, st = enc(chain, [[0x1234, payload]], mode | EXT)
    want = ext_block(4, [1, 6], [0, 2], 2 + len(payload)) + u16(0x1234) + payload
    assert bytes(arena) == want
    assert int(st[0]) == 0
    # the plain mode truncates End (Q1) and flags it
    a0, _, s0 = enc(chain, [[0x1234, payload]], mode)
    assert bytes(a0[:6]) == hdr(6, 1) + hdr(2, 6) + hdr(2 + len(payload), 0)
    assert int(s0[0]) & 0x80000000


def test_ext_known_nested():
    """inner tuple over 8191 B -> extended; the chain grows past 8191 B too,
    and its entry for the tuple carries tag 2.  A small sibling tuple stays
    plain."""
    chain = SChain(SInt16, STuple(SVariableString(), SInt32), STuple(SBool))
    s = "x" * 9000
    arena, offs, st = enc(chain, [[7, [s, 0x01020304], [True]]], 0 | EXT)
    inner_pay = s.encode() + u32(0x01020304)
    inner = ext_block(4, [6, 1], [0, 9000], len(inner_pay)) + inner_pay
    small = hdr(4, 5) + hdr(1, 0) + b"\x01"
    pay = u16(7) + inner + small
    want = ext_block(4, [1, 2, 4], [0, 2, 2 + len(inner)], len(pay)) + pay
    assert bytes(arena) == want


def test_ext_known_map_child():
    """a sorted map whose value is large: the map container is extended (own
    tag 7 in its lead) and its parent entry carries tag 2"""
    chain = SChain(SMapSorted(SString.Match("k"), SVariableBytes()))
    v = b"\xAB" * 8200
    arena, _, _ = enc(chain, [[[None, v]]], 0 | EXT)
    mpay = b"k" + v
    m = ext_block(7, [6, 6], [0, 1], len(mpay)) + mpay
    want = ext_block(4, [2], [0], len(m)) + m
    assert bytes(arena) == want


def rebuild_columns(chain, out, arena, n):
    """decoded columns (oracle layout, numpy) -> HostColumns for re-encoding"""
    back = HostColumns(chain, n)
    for c, sp in enumerate(back.specs):
        if sp.fixed:
            back.data[c] = out.data[c][: n * sp.width].copy()
        if sp.var:
            st0 = out.start[c][:n].astype(np.int64)
            ln = out.length[c][:n].astype(np.int64)
            o = np.zeros(n + 1, np.int64)
            np.cumsum(ln, out=o[1:])
            idx = (np.repeat(st0 - o[:-1], ln) + np.arange(o[-1])) if o[-1] else np.zeros(0, np.int64)
            back.data[c] = arena[idx] if o[-1] else np.zeros(0, np.uint8)
            back.offsets[c] = o.astype(np.uint32)
        if sp.has_valid:
            v = out.valid[c][:n].copy()
            v[v == 255] = 0
            back.valid[c] = v
    return back


def no_empty_containers(chain):
    # BeginX/EndNested writes a present EMPTY container as 10 00, which
    # NewSeqGetAccess rejects (seqget.go:23): not decodable in any mode
    return not any(n.kind in ("tuple", "map") and not n.children for n, *_ in chain.walk())


@pytest.mark.parametrize("seed", range(20))
def test_ext_oracle_roundtrip(seed):
    chain = rand_chain(seed)
    if not no_empty_containers(chain):
        pytest.skip("schema with an empty container")
    rows = big_rows(chain, 60, seed)
    arena, offs, st = enc(chain, rows, EXT)
    n = len(rows)
    out, dst = ob.decode(chain, arena, offs, n, nthreads=8, mode=EXT)
    assert (dst == 0).all(), dst
    back = rebuild_columns(chain, out, arena, n)
    a2, o2, _ = ob.encode(chain, back, EXT, nthreads=8)
    assert np.array_equal(o2, offs) and np.array_equal(a2, arena)


def test_ext_oracle_plain_decoder_rejects_extended():
    """the reference's decoder (plain mode) cannot read an extended blob; the
    extended-mode decoder reads plain blobs exactly like the plain one"""
    chain = SChain(SInt16, SVariableBytes())
    arena, offs, _ = enc(chain, [[1, b"z" * 9000], [2, b"small"]], EXT)
    _, st_plain = ob.decode(chain, arena, offs, 2)
    _, st_ext = ob.decode(chain, arena, offs, 2, mode=EXT)
    assert st_plain[0] != 0 and st_plain[1] == 0
    assert (st_ext == 0).all()


# ----------------------------------------------------------------- GPU -----
def _torch():
    import torch
    return torch


def gpu_encode(chain, hc, mode, via_host=False):
    from packos_amd.api import CompiledSchema, DeviceColumns, encode_batch, encode_host_batch
    T = _torch()
    s = CompiledSchema(chain, mode)
    if via_host:
        a, o, st = encode_host_batch(s, hc, chunk_blobs=37)
        return np.asarray(a), np.asarray(o, np.uint64), np.asarray(st, np.uint32)
    r = encode_batch(s, DeviceColumns.from_host(s, hc, "cuda:0"))
    T.cuda.synchronize()
    n = hc.n
    offs = (r.offsets.cpu().numpy().astype(np.uint64) if r.offsets is not None
            else np.arange(n + 1, dtype=np.uint64) * np.uint64(r.blob_size))
    return r.arena[: r.total].cpu().numpy(), offs, r.status.cpu().numpy().astype(np.uint32)


def assert_gpu_matches(chain, hc, mode, what, via_host=False):
    a0, o0, s0 = ob.encode(chain, hc, mode, nthreads=8)
    a1, o1, s1 = gpu_encode(chain, hc, mode, via_host)
    assert np.array_equal(o0, o1), f"{what}: offsets differ"
    if not np.array_equal(a0, a1):
        bad = int(np.nonzero(a0 != a1)[0][0])
        blob = int(np.searchsorted(o0, bad, side="right")) - 1
        raise AssertionError(f"{what}: byte {bad} (blob {blob}, +{bad - int(o0[blob])}) "
                             f"oracle {a0[bad]:#x} gpu {a1[bad]:#x}")
    assert np.array_equal(s0, s1), f"{what}: status differs"
    return a0, o0


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("seed", range(24))
def test_gpu_ext_encode_random(seed, mode):
    chain = rand_chain(seed)
    hc = HostColumns.from_rows(chain, big_rows(chain, 150, seed))
    assert_gpu_matches(chain, hc, mode | EXT, f"seed {seed} mode {mode}")


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(8))
def test_gpu_ext_small_equals_plain(seed):
    """extended mode on blobs with no large container: the reference bytes"""
    chain = rand_chain(seed + 100)
    hc = HostColumns.from_rows(chain, rand_rows(chain, 500, seed))
    a0, o0, _ = ob.encode(chain, hc, 0, nthreads=8)
    a1, o1, s1 = gpu_encode(chain, hc, EXT)
    assert np.array_equal(o0, o1) and np.array_equal(a0, a1)
    assert not (s1 & 0x80000000).any()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
def test_gpu_ext_fixed_schema_over_8k(mode):
    """a fixed schema whose blobs are 9 KB: the fixed path would truncate, the
    extended mode takes the offsets path"""
    chain = SChain(SInt64, STuple(SStringLen(4000), SBytes(4500)), SBool)
    rng = random.Random(3)
    rows = [[rng.getrandbits(63), ["a" * 4000, rng.randbytes(4500)], rng.random() < 0.5] for _ in range(257)]
    hc = HostColumns.from_rows(chain, rows)
    a0, o0 = assert_gpu_matches(chain, hc, mode | EXT, "fixed 9 KB")
    assert a0[0] == 2 and a0[1] == 0   # extended top level


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_gpu_ext_host_batch(seed):
    chain = rand_chain(seed + 40)
    hc = HostColumns.from_rows(chain, big_rows(chain, 300, seed))
    assert_gpu_matches(chain, hc, EXT, f"host seed {seed}", via_host=True)


def gpu_decode(chain, arena, offs, n, mode):
    from packos_amd.api import CompiledSchema, decode_batch
    T = _torch()
    s = CompiledSchema(chain, mode)
    a = T.from_numpy(arena if arena.size else np.zeros(16, np.uint8)).to("cuda:0")
    o = T.from_numpy(offs.astype(np.int64)).to("cuda:0")
    out, st = decode_batch(s, a, o, n)
    T.cuda.synchronize()
    return out, st.cpu().numpy().astype(np.uint32)


def assert_same_decode(chain, arena, offs, n, mode, what):
    o_out, o_st = ob.decode(chain, arena, offs, n, nthreads=8, mode=mode)
    g_out, g_st = gpu_decode(chain, arena, offs, n, mode)
    if not np.array_equal(o_st, g_st):
        bad = int(np.nonzero(o_st != g_st)[0][0])
        raise AssertionError(f"{what}: status blob {bad}: oracle {o_st[bad]:#x} gpu {g_st[bad]:#x}")
    ok = o_st[:n] == 0
    for c, sp in enumerate(o_out.specs):
        for name in ("data", "valid", "start", "length"):
            a = getattr(o_out, name)[c]
            if a is None:
                continue
            b = getattr(g_out, name)[c].cpu().numpy()
            if name == "start":
                b = b.astype(np.uint64)
            if name == "length":
                b = b.astype(np.uint32)
            if name == "data":
                w = sp.width
                assert np.array_equal(a[: n * w].reshape(n, w)[ok], b[: n * w].reshape(n, w)[ok]), (what, c, name)
            else:
                assert np.array_equal(a[:n][ok], b[:n][ok]), (what, c, name)
    return g_st


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(20))
def test_gpu_ext_decode_random(seed):
    chain = rand_chain(seed)
    rows = big_rows(chain, 120, seed)
    arena, offs, _ = enc(chain, rows, EXT)
    st = assert_same_decode(chain, arena, offs, len(rows), EXT, f"seed {seed}")
    if no_empty_containers(chain):
        assert (st == 0).all()
    # the plain-mode decoder on the same arena: the reference's reading
    assert_same_decode(chain, arena, offs, len(rows), 0, f"plain seed {seed}")


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(12))
def test_gpu_ext_decode_corrupted(seed):
    """flipped lead / entry bytes and truncations of extended blobs: every
    status (code, position) matches the oracle"""
    rng = np.random.default_rng(seed)
    chain = rand_chain(seed + 7)
    rows = big_rows(chain, 80, seed, p=0.6)
    arena, offs, _ = enc(chain, rows, EXT)
    arena = arena.copy()
    n = len(rows)
    offs = offs.copy()
    for i in range(n):
        a, b = int(offs[i]), int(offs[i + 1])
        r = rng.random()
        if r < 0.3 and b - a > 2:
            k = int(rng.integers(0, min(b - a, 48)))
            arena[a + k] ^= np.uint8(1 << int(rng.integers(0, 8)))
        elif r < 0.45 and b - a > 1:
            offs[i + 1] = offs[i] + np.uint64(rng.integers(0, b - a))   # truncated (gap after)
    assert_same_decode(chain, arena, offs, n, EXT, f"corrupted seed {seed}")


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_gpu_ext_roundtrip(seed):
    """GPU extended encode -> GPU extended decode -> GPU re-encode: same bytes"""
    chain = rand_chain(seed + 300)
    if not no_empty_containers(chain):
        pytest.skip("schema with an empty container")
    rows = big_rows(chain, 100, seed)
    hc = HostColumns.from_rows(chain, rows)
    arena, offs, _ = gpu_encode(chain, hc, EXT)
    out, st = gpu_decode(chain, arena, offs, hc.n, EXT)
    assert (st == 0).all()

    class O:   # decoded columns as numpy, the oracle's layout
        pass
    o = O()
    o.data = [None if x is None else x.cpu().numpy() for x in out.data]
    o.valid = [None if x is None else x.cpu().numpy() for x in out.valid]
    o.start = [None if x is None else x.cpu().numpy().view(np.uint64) for x in out.start]
    o.length = [None if x is None else x.cpu().numpy().view(np.uint32) for x in out.length]
    back = rebuild_columns(chain, o, arena, hc.n)
    a2, o2, _ = gpu_encode(chain, back, EXT)
    assert np.array_equal(o2, offs) and np.array_equal(a2, arena)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("seed", range(10))
def test_ext_host_sizes_match_oracle(seed, mode):
    """packos_schema_blob_size_host (shard planning) applies the extended
    rule exactly like the encoders; packos_schema_ext_overhead bounds it"""
    from packos_amd.api import CompiledSchema
    chain = rand_chain(seed + 60)
    rows = big_rows(chain, 40, seed)
    hc = HostColumns.from_rows(chain, rows)
    _, offs, _ = ob.encode(chain, hc, mode | EXT, nthreads=4)
    s = CompiledSchema(chain, mode | EXT)
    ncol = len(s.specs)
    over = s.ext_overhead
    plain = CompiledSchema(chain, mode)
    for i in range(hc.n):
        w = np.zeros(max(ncol, 1), np.uint32)
        v = np.ones(max(ncol, 1), np.uint8)
        for c in range(ncol):
            if hc.offsets[c] is not None:
                w[c] = int(hc.offsets[c][i + 1]) - int(hc.offsets[c][i])
            if hc.valid[c] is not None:
                v[c] = hc.valid[c][i]
        got = s.blob_size_host(w, v)
        assert got == int(offs[i + 1] - offs[i]), i
        assert got <= plain.blob_size_host(w, v) + over


GETTERS = [(0, 1, 2), (0, 1, 8), (1, 1, 4), (1, 3, 8), (2, 6, 0), (3, 0, 0), (4, 0, 0), (0, 5, 1)]


def test_ext_oracle_get_reads_extended():
    """GetAccess over an extended blob (PACKOS_GET_EXTENDED): the nested
    extended tuple's fields are reached through its tag-2 entry"""
    chain = SChain(SInt16, STuple(SVariableString(), SInt32), STuple(SBool))
    s = "x" * 9000
    arena, offs, _ = enc(chain, [[7, [s, 0x01020304], [True]]], EXT)
    X = 0x100
    v, st0, ln, tg, stt = ob.get_batch(arena, offs, 1, [1, 1], 0 | X, 1, 4)
    assert stt[0] == 0 and int.from_bytes(bytes(v[0]), "little") == 0x01020304
    v, st0, ln, tg, stt = ob.get_batch(arena, offs, 1, [1, 0], 2 | X, 6, 0)
    assert stt[0] == 0 and ln[0] == 9000 and bytes(arena[st0[0]:st0[0] + 9000]) == s.encode()
    v, st0, ln, tg, stt = ob.get_batch(arena, offs, 1, [0], 3 | X)
    assert stt[0] == 0 and int.from_bytes(bytes(v[0]), "little") == 7
    assert ob.get_batch(arena, offs, 1, [1], 2 | X, 6, 0)[3][0] == 2      # the field's own tag: 2
    # without the flag the reference's GetAccess sees h0 offset 0 (argCount
    # -1): every Get* is a decode error
    assert ob.get_batch(arena, offs, 1, [0], 3)[4][0] == 1


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(12))
def test_gpu_ext_get_batch(seed):
    """packos_get_batch | PACKOS_GET_EXTENDED vs the oracle on extended
    batches (every getter family, random nested paths, some corrupted blobs)"""
    from packos_amd.api import get_batch
    T = _torch()
    rng = np.random.default_rng(500 + seed)
    chain = rand_chain(seed)
    rows = big_rows(chain, 150, seed)
    arena, offs, _ = enc(chain, rows, int(rng.integers(0, 2)) | EXT)
    arena = arena.copy()
    for i in range(0, len(rows), 4):
        a, b = int(offs[i]), int(offs[i + 1])
        if b > a:
            arena[a + int(rng.integers(0, min(12, b - a)))] = rng.integers(0, 256)
    da = T.from_numpy(arena).to("cuda:0")
    do = T.from_numpy(offs.astype(np.int64)).to("cuda:0")
    for _ in range(12):
        depth = int(rng.integers(1, 3))
        path = [int(rng.integers(0, 6)) for _ in range(depth)]
        getter, tag, width = GETTERS[int(rng.integers(0, len(GETTERS)))]
        o = ob.get_batch(arena, offs, len(rows), path, getter | 0x100, tag, width)
        g = [None if x is None else x.cpu().numpy()
             for x in get_batch(da, do, len(rows), path, getter | 0x100, tag, width)]
        what = (path, getter, tag, width)
        assert np.array_equal(o[4], g[4]), what
        assert np.array_equal(o[3], g[3]), what
        assert np.array_equal(o[1], g[1].astype(np.uint64)), what
        assert np.array_equal(o[2], g[2].astype(np.uint32)), what
        if o[0] is not None:
            assert np.array_equal(o[0], g[0]), what


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_gpu_ext_decode_host_batch(seed):
    """packos_decode_host_batch in extended mode (host arena -> chunked H2D ->
    decode -> host columns) vs the oracle"""
    from packos_amd.api import CompiledSchema, decode_host_batch
    chain = rand_chain(seed + 80)
    rows = big_rows(chain, 200, seed)
    arena, offs, _ = enc(chain, rows, EXT)
    n = len(rows)
    got, g_st = decode_host_batch(CompiledSchema(chain, EXT), arena, offs, n, chunk_blobs=37)
    o_out, o_st = ob.decode(chain, arena, offs, n, nthreads=8, mode=EXT)
    assert np.array_equal(o_st, g_st)
    ok = o_st[:n] == 0
    for c, sp in enumerate(o_out.specs):
        if sp.fixed:
            w = sp.width
            assert np.array_equal(o_out.data[c][: n * w].reshape(n, w)[ok], got.data[c][: n * w].reshape(n, w)[ok])
        if sp.var:
            assert np.array_equal(o_out.start[c][:n][ok], got.start[c][:n][ok])
            assert np.array_equal(o_out.length[c][:n][ok], got.length[c][:n][ok])
