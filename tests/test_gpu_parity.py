"""HIP path vs CPU oracle, bit-exact (integer/byte work: no tolerance).

Every test calls libpackos.so through the C ABI on cuda:0 and compares with
the oracle on the same seeded inputs (oracle pinned by test_oracle_golden.py)
or with the reference's golden bytes directly.
"""
import ctypes as C
import random

import numpy as np
import pytest

import oracle_bridge as ob
from packos_amd import _lib
from golden_util import MODES, chain_of, load, unwrap
from packos_amd.api import (CompiledSchema, DeviceColumns, decode_batch, encode_batch, get_batch, get_field_batch,
                           get_map_batch, GET_ANY, GET_INT, GET_SPAN)
from packos_amd.columns import HostColumns
from packos_amd.configs import CONFIGS, make_columns
from packos_amd.schema import SBool, SChain, SInt16, SInt32, SInt64, SStringLen, SVariableString, STuple, SMap, SString
from schema_gen import rand_chain, rand_checked_chain, rand_checked_rows, rand_rows

pytestmark = pytest.mark.gpu
G = load()


def torch():
    import torch as t
    return t


def gpu_encode(chain, hc, mode=0, flags=0, fused=False, poison=False):
    """fused=True: size the arena with the size pass, then encode WITHOUT
    PACKOS_ENC_OFFSETS_READY into poisoned offsets, so the single-pass kernel's
    own sizes + look-back scan must produce them.  poison: the arena starts
    filled with 0xCD (bytes an encoder never stores stay visible)."""
    T = torch()
    s = CompiledSchema(chain, mode)
    dc = DeviceColumns.from_host(s, hc, "cuda:0")
    out = None
    if poison:
        a0, o0, _ = ob.encode(chain, hc, mode, nthreads=8)
        out = T.full((max(int(o0[hc.n]), 16),), 0xCD, dtype=T.uint8, device="cuda:0")
    r = encode_batch(s, dc, flags=flags, out=out)
    if fused and r.blob_size < 0 and hc.n:
        L = _lib.lib()
        n = hc.n
        wsb = L.packos_encode_workspace_size(s.handle, n)
        ws = T.full((wsb,), 0xAB, dtype=T.uint8, device="cuda:0")
        r.offsets.fill_(-1)
        r.arena.fill_(0xCD)
        assert L.packos_encode_batch(s.handle, dc.ctypes_array(), n, r.arena.data_ptr(), r.arena.numel(),
                                     r.offsets.data_ptr(), r.status.data_ptr(), ws.data_ptr(), wsb, flags,
                                     None) == 0, L.packos_last_error().decode()
    T.cuda.synchronize()
    arena = r.arena[: r.total].cpu().numpy()
    offs = r.offsets.cpu().numpy().astype(np.uint64)
    st = r.status.cpu().numpy().astype(np.uint32)
    return arena, offs, st


def assert_same_encoding(chain, hc, mode, what="", flags=0, fused=False):
    a0, o0, s0 = ob.encode(chain, hc, mode, nthreads=8)
    a1, o1, s1 = gpu_encode(chain, hc, mode, flags, fused)
    assert np.array_equal(o0, o1), f"{what}: offsets differ"
    if not np.array_equal(a0, a1):
        bad = int(np.nonzero(a0 != a1)[0][0])
        blob = int(np.searchsorted(o0, bad, side="right") - 1)
        raise AssertionError(f"{what}: first diff at byte {bad} (blob {blob}, +{bad - int(o0[blob])})")
    assert np.array_equal(s0, s1), f"{what}: status differs"


# --------------------------------------------------------------- golden ----
@pytest.mark.parametrize("case", G["encode"], ids=[c["id"] for c in G["encode"]])
def test_golden_encode(case):
    chain = chain_of(case["schema"])
    hc = HostColumns.from_rows(chain, [unwrap(case["row"])])
    a, o, st = gpu_encode(chain, hc, MODES[case["mode"]])
    assert bytes(a).hex() == case["hex"]
    assert st[0] == 0


@pytest.mark.parametrize("case", G["equal"], ids=[c["id"] for c in G["equal"]])
def test_golden_cross_api(case):
    outs = []
    for v in case["variants"]:
        chain = chain_of(v["schema"])
        hc = HostColumns.from_rows(chain, [unwrap(case["row"])])
        a, _, st = gpu_encode(chain, hc, MODES[v["mode"]])
        outs.append(bytes(a))
        assert int(st[0]) == 0
    assert all(o == outs[0] for o in outs)


# --------------------------------------------------------------- encode ----
# k_encode_tiles knobs (read when the schema compiles): PACKOS_VAR_PER = var
# staging pool bytes per blob (0: no var column is ever staged -> every value
# > 16 B is a hole, shorter ones take the HBM slow path; 8: tiles stage some
# columns and not others; 256: everything staged), PACKOS_SIZES_SCAN = the
# look-back size pass + loaded offsets instead of the closed form
VAR_KNOBS = [{}, {"PACKOS_VAR_PER": "0"}, {"PACKOS_VAR_PER": "8"}, {"PACKOS_VAR_PER": "256"},
             {"PACKOS_SIZES_SCAN": "1"}, {"PACKOS_SIZES_SCAN": "1", "PACKOS_VAR_PER": "0"}]


@pytest.mark.parametrize("fused", [False, True], ids=["offsets_ready", "single_pass"])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("seed", range(60))
def test_random_schema_encode(seed, mode, fused):
    # default var path: k_encode_tiles (caller offsets, or its own layout)
    chain = rand_chain(seed)
    hc = HostColumns.from_rows(chain, rand_rows(chain, 257 + 300 * (seed % 3), seed * 7 + 1))
    assert_same_encoding(chain, hc, mode, f"seed {seed}", fused=fused)


@pytest.mark.parametrize("scan", [False, True], ids=["closed_form", "lookback"])
@pytest.mark.parametrize("n,seed", [(0, 1), (1, 2), (1023, 3), (1024, 4), (1025, 5), (5000, 6), (70001, 7)])
def test_size_pass_var_base_and_counts(n, seed, scan, monkeypatch):
    """Size pass for data-independent presence (k_sizes_affine:
    offs[i] = i*C + sum_v off_v[i] - off_v[0]) vs the look-back scan
    (PACKOS_SIZES_SCAN): var columns whose offsets start past 0 (a column
    slice), block-boundary counts; offsets and bytes equal the oracle's."""
    T = torch()
    if scan:
        monkeypatch.setenv("PACKOS_SIZES_SCAN", "1")
    chain = SChain(SInt16, SVariableString(), SStringLen(5), SVariableString(), STuple(SInt16, SVariableString()))
    rng = np.random.default_rng(seed)
    rows = [[int(rng.integers(-30000, 30000)), "x" * int(rng.integers(0, 60)), "abcde",
             bytes(rng.integers(32, 127, int(rng.integers(0, 300))).astype(np.uint8)).decode(),
             [7, "y" * int(rng.integers(0, 9))]] for _ in range(n)]
    hc = HostColumns.from_rows(chain, rows)
    s = CompiledSchema(chain, 0)
    dc = DeviceColumns.from_host(s, hc, "cuda:0")
    for c, o in enumerate(dc.offsets):
        if o is not None:   # shift every var column by a different base
            k = 1000 + 37 * c
            dc.data[c] = T.cat([T.full((k,), 0xEE, dtype=T.uint8, device="cuda:0"), dc.data[c]])
            dc.offsets[c] = o + k
    r = encode_batch(s, dc)
    T.cuda.synchronize()
    a0, o0, s0 = ob.encode(chain, hc, 0, nthreads=8)
    assert np.array_equal(r.offsets.cpu().numpy().astype(np.uint64), o0)
    assert np.array_equal(r.arena[: r.total].cpu().numpy(), a0)
    assert np.array_equal(r.status.cpu().numpy().astype(np.uint32), s0)


@pytest.mark.parametrize("knobs", VAR_KNOBS[1:], ids=lambda k: ",".join(f"{a[7:]}={b}" for a, b in k.items()))
@pytest.mark.parametrize("seed", range(0, 60, 6))
def test_random_schema_encode_var_knobs(seed, knobs, monkeypatch):
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    chain = rand_chain(seed)
    hc = HostColumns.from_rows(chain, rand_rows(chain, 700, seed * 7 + 3))
    assert_same_encoding(chain, hc, seed % 2, f"knobs {knobs} seed {seed}", fused=True)


@pytest.mark.parametrize("fields,tuples,nest", [(43, 0, 0), (44, 0, 0), (45, 0, 0), (60, 0, 0), (6, 15, 0),
                                               (6, 16, 0), (6, 0, 12)])
def test_stream_plan_limits(fields, tuples, nest):
    """Schemas at and past the tile encoder's plan limits (48 items, 16
    containers): past them the call routes to k_encode_var; both must
    match the oracle.  Items = one header block per container + the leaves:
    `fields` flat leaves, `tuples` one-leaf tuples (one container each), and a
    tuple nested `nest` deep (12 is the compiler's depth limit)."""
    import random
    rng = random.Random(fields * 31 + tuples * 7 + nest)
    leaves = [SInt16 if k % 3 else SVariableString() for k in range(fields)]
    tups = [STuple(SVariableString()) for _ in range(tuples)]
    node = STuple(SInt16, SVariableString())
    for _ in range(nest):   # a chain of tuples inside tuples
        node = STuple(SInt16, node)
    chain = SChain(*leaves, *tups, node)
    rows = []
    for i in range(600):
        r = [rng.getrandbits(16) if k % 3 else "v" * rng.randint(0, 90) for k in range(fields)]
        t = [["t" * rng.randint(0, 60)] for _ in range(tuples)]
        inner = [rng.getrandbits(16), "w" * rng.randint(0, 70)]
        for _ in range(nest):
            inner = [rng.getrandbits(16), inner]
        rows.append(r + t + [inner])
    hc = HostColumns.from_rows(chain, rows)
    for mode in (0, 1):
        assert_same_encoding(chain, hc, mode, f"fields {fields} nest {nest} mode {mode}")
        assert_same_encoding(chain, hc, mode, f"fields {fields} nest {nest} mode {mode} fused", fused=True)


@pytest.mark.parametrize("name,n,chunk,pinned", [("C3", 20000, 3000, False), ("C3", 20000, 0, True),
                                                 ("M", 10001, 4096, False), ("M", 10001, 4096, True),
                                                 ("C5", 3000, 700, False), ("C1", 1000, 0, False),
                                                 ("C4", 5001, 1024, True), ("C2", 7777, 1000, False)])
def test_encode_host_batch(name, n, chunk, pinned):
    """packos_encode_host_batch (host columns -> chunked H2D / encode / D2H on
    two streams -> host arena) vs the oracle, pageable and pinned inputs,
    many chunks (both pipeline slots reused)."""
    from packos_amd.api import encode_host_batch
    T = torch()
    cfg = CONFIGS[name]
    hc = make_columns(cfg, n=n)
    if pinned:
        for lst in (hc.data, hc.offsets, hc.valid):
            for c, a in enumerate(lst):
                if a is not None:
                    lst[c] = T.from_numpy(np.ascontiguousarray(a)).pin_memory().numpy()
    s = CompiledSchema(cfg.chain, cfg.mode)
    a1, o1, s1 = encode_host_batch(s, hc, chunk_blobs=chunk)
    a0, o0, s0 = ob.encode(cfg.chain, hc, cfg.mode, nthreads=8)
    assert np.array_equal(o0, o1) and np.array_equal(a0, a1) and np.array_equal(s0, s1.astype(np.uint32))


@pytest.mark.parametrize("seed", range(0, 60, 5))
def test_encode_host_batch_random(seed):
    from packos_amd.api import encode_host_batch
    chain = rand_chain(seed)
    hc = HostColumns.from_rows(chain, rand_rows(chain, 2500, seed * 3 + 2))
    for mode in (0, 1):
        s = CompiledSchema(chain, mode)
        a1, o1, s1 = encode_host_batch(s, hc, chunk_blobs=600)
        a0, o0, s0 = ob.encode(chain, hc, mode, nthreads=8)
        assert np.array_equal(o0, o1) and np.array_equal(a0, a1) and np.array_equal(s0, s1.astype(np.uint32))


@pytest.mark.parametrize("fused", [False, True], ids=["offsets_ready", "single_pass"])
@pytest.mark.parametrize("knobs", VAR_KNOBS, ids=lambda k: ",".join(f"{a[7:]}={b}" for a, b in k.items()) or "default")
def test_var_holes_and_budgets(knobs, fused, monkeypatch):
    """k_encode_tiles: values around the 16-B hole threshold at every 16-B
    alignment (a chunk = tail of one hole + frame bytes + head of the next),
    adjacent long values, nil containers, staged / unstaged var columns, the
    HBM slow path for short unstaged values."""
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    img = knobs.get("PACKOS_VAR_PER")
    longv = knobs.get("PACKOS_SIZES_SCAN")
    chain = SChain(SInt16, SVariableString(), SVariableString(), STuple(SVariableString(), SInt16),
                   SStringLen(100))
    rng = np.random.default_rng(11)
    rows = []
    lens = [0, 1, 15, 16, 17, 31, 32, 33, 48, 63, 64, 65, 66, 79, 80, 81, 95, 96, 97, 127, 128, 129, 200, 513]
    for i in range(1100):
        a = lens[int(rng.integers(0, len(lens)))] + (i % 3)
        b = lens[int(rng.integers(0, len(lens)))]
        c = int(rng.integers(0, 300)) if i % 7 else 4000
        rows.append([i, "a" * a, bytes(rng.integers(32, 127, b, dtype=np.uint8)).decode(),
                     None if rng.random() < 0.15 else ["t" * c, -i], "p" * 100])
    hc = HostColumns.from_rows(chain, rows)
    for mode in (0, 1):
        assert_same_encoding(chain, hc, mode, f"var_per={img} scan={longv} mode={mode}", fused=fused)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("seed", range(20))
def test_random_schema_encode_wave_kernel(seed, mode):
    # PACKOS_ENC_FORCE_GENERIC: the one-wavefront-per-blob kernel (the tiled
    # kernel's fallback) on its own
    chain = rand_chain(seed)
    hc = HostColumns.from_rows(chain, rand_rows(chain, 257, seed * 7 + 1))
    assert_same_encoding(chain, hc, mode, f"wave seed {seed}", flags=_lib.ENC_FORCE_GENERIC)


@pytest.mark.parametrize("kernel", ["tiles", "tiles_fused", "tiles_no_pool"])
@pytest.mark.parametrize("mode", [0, 1])
def test_var_tile_runs_and_fallbacks(mode, kernel, monkeypatch):
    """Tiled var encode: long values (holes), blobs > 64 KiB (whole-tile
    per-blob fallback), nil containers, and ragged last tiles."""
    chain = SChain(SInt16, SVariableString(), STuple(SVariableString(), SInt16))
    rng = np.random.default_rng(5)
    rows = []
    for i in range(333):
        r = rng.random()
        ln = int(rng.integers(0, 40)) if r < 0.7 else int(rng.integers(3000, 12000)) if r < 0.97 else 70_000
        rows.append([i, "s" * ln, None if rng.random() < 0.1 else ["t" * int(rng.integers(0, 300)), -i]])
    hc = HostColumns.from_rows(chain, rows)
    if kernel == "tiles_no_pool":
        monkeypatch.setenv("PACKOS_VAR_PER", "0")
    assert_same_encoding(chain, hc, mode, f"tile edges {kernel}", fused=kernel == "tiles_fused")


def test_var_encode_capacity_overrun():
    T = torch()
    cfg = CONFIGS["C3"]
    hc = make_columns(cfg, n=5000)
    a0, o0, _ = ob.encode(cfg.chain, hc, 0, nthreads=8)
    s = CompiledSchema(cfg.chain, 0)
    dc = DeviceColumns.from_host(s, hc, "cuda:0")
    L = _lib.lib()
    n = hc.n
    cap = int(o0[n]) - 1000
    out = T.zeros(cap, dtype=T.uint8, device="cuda:0")
    offs = T.empty(n + 1, dtype=T.int64, device="cuda:0")
    st = T.empty(n, dtype=T.int32, device="cuda:0")
    wsb = L.packos_encode_workspace_size(s.handle, n)
    ws = T.empty(wsb, dtype=T.uint8, device="cuda:0")
    assert L.packos_encode_batch(s.handle, dc.ctypes_array(), n, out.data_ptr(), cap, offs.data_ptr(),
                                 st.data_ptr(), ws.data_ptr(), wsb, 0, None) == 0
    T.cuda.synchronize()
    fits = o0[1:] <= cap
    stn = st.cpu().numpy()
    assert (stn[fits] == 0).all() and (stn[~fits] == 4).all()
    last = int(o0[int(fits.sum())])
    assert np.array_equal(out.cpu().numpy()[:last], a0[:last])


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("nil", [False, True])
def test_var_wide_fixed_holes(mode, nil):
    """Fixed leaves wider than 16 B in a var schema stay in HBM as holes
    (copied by the chunk pass straight from their column rows), next to var
    values, literals and nullable scalars."""
    chain = SChain(SInt16, SVariableString(), SStringLen(40), STuple(SStringLen(17), SInt16), SStringLen(100),
                   SMap(SString.Match("key"), SStringLen(33)), SInt32)
    rng = np.random.default_rng(3 + mode + 2 * nil)
    rows = []
    for i in range(2100):
        rows.append([i, "v" * int(rng.integers(0, 70)), "a" * 40,
                     None if (nil and rng.random() < 0.2) else ["b" * 17, -i], "c" * 100,
                     None if (nil and rng.random() < 0.2) else {"key": "d" * 33}, 7 * i])
    hc = HostColumns.from_rows(chain, rows)
    assert_same_encoding(chain, hc, mode, f"wide fixed holes mode={mode} nil={nil}")
    assert_same_encoding(chain, hc, mode, f"wide fixed holes mode={mode} nil={nil} fused", fused=True)


@pytest.mark.parametrize("shift", [1, 3, 7, 8, 13])
def test_var_unaligned_columns(shift):
    """Column data at arbitrary byte alignment (views at an offset): every
    staged row array and every hole source is misaligned differently."""
    T = torch()
    cfg = CONFIGS["C3"]
    hc = make_columns(cfg, n=3001)
    s = CompiledSchema(cfg.chain, cfg.mode)
    dc = DeviceColumns.from_host(s, hc, "cuda:0")
    for c, d in enumerate(dc.data):
        if d is not None:
            k = shift + 2 * c
            buf = T.zeros(d.numel() + 64, dtype=T.uint8, device="cuda:0")
            buf[k:k + d.numel()] = d
            dc.data[c] = buf[k:k + d.numel()]
    r = encode_batch(s, dc)
    T.cuda.synchronize()
    a0, o0, s0 = ob.encode(cfg.chain, hc, cfg.mode, nthreads=8)
    assert np.array_equal(r.offsets.cpu().numpy().astype(np.uint64), o0)
    assert np.array_equal(r.arena[: r.total].cpu().numpy(), a0)


@pytest.mark.parametrize("base_gib", [0, 4.25])
def test_var_offsets64(base_gib):
    """64-bit var offsets (packos_column.offsets64): the C5 schema with its var
    arenas placed `base_gib` GiB into one device allocation, so the offsets
    have high bits set; bytes and offsets equal the oracle's (which reads the
    same values through 32-bit offsets relative to the arena start)."""
    T = torch()
    cfg = CONFIGS["C5"]
    n = 4099
    hc = make_columns(cfg, n=n)
    s = CompiledSchema(cfg.chain, cfg.mode)
    dc = DeviceColumns.from_host(s, hc, "cuda:0")
    base = int(base_gib * 2 ** 30)
    var_cols = [c for c, o in enumerate(dc.offsets) if o is not None]
    total_var = sum(int(hc.offsets[c][-1]) for c in var_cols)
    big = T.empty(base + total_var + 64, dtype=T.uint8, device="cuda:0")
    arr = dc.ctypes_array()
    keep = []
    pos = base
    for c in var_cols:
        ln = int(hc.offsets[c][-1])
        big[pos:pos + ln] = dc.data[c][:ln]
        o64 = T.from_numpy(hc.offsets[c].astype(np.int64) + pos).to("cuda:0")
        keep.append(o64)
        arr[c].data = big.data_ptr()
        arr[c].offsets = None
        arr[c].offsets64 = o64.data_ptr()
        pos += ln
    L = _lib.lib()
    a0, o0, s0 = ob.encode(cfg.chain, hc, cfg.mode, nthreads=8)
    out = T.zeros(int(o0[n]) + 16, dtype=T.uint8, device="cuda:0")
    offs = T.empty(n + 1, dtype=T.int64, device="cuda:0")
    st = T.empty(n, dtype=T.int32, device="cuda:0")
    wsb = L.packos_encode_workspace_size(s.handle, n)
    ws = T.empty(max(wsb, 16), dtype=T.uint8, device="cuda:0")
    for flags in (0, _lib.ENC_FORCE_GENERIC):
        assert L.packos_encode_batch(s.handle, arr, n, out.data_ptr(), out.numel(), offs.data_ptr(), st.data_ptr(),
                                     ws.data_ptr(), wsb, flags, None) == 0, L.packos_last_error()
        T.cuda.synchronize()
        assert np.array_equal(offs.cpu().numpy().astype(np.uint64), o0)
        assert np.array_equal(out[: int(o0[n])].cpu().numpy(), a0)
    del big


@pytest.mark.parametrize("seed", range(30))
def test_random_fixed_schema_encode(seed):
    # no var leaves, no nils: exercises the LDS-tiled fixed-layout kernel
    chain = rand_chain(1000 + seed, allow_var=False, allow_null=False)
    hc = HostColumns.from_rows(chain, rand_rows(chain, 1500, seed, nil_p=0.0))
    hc.valid = [None] * len(hc.valid)
    assert_same_encoding(chain, hc, 0, f"fixed seed {seed}")


@pytest.mark.parametrize("variant", [13, 2, 8])
@pytest.mark.parametrize("seed", range(16))
def test_fixed_kernel_variants(seed, variant):
    """Every fixed-layout kernel on random fixed schemas padded (one extra
    StringLen field) to a blob size the tile kernel takes (B % 4 == 0,
    16 <= B <= 1024), with batch sizes that leave partial last tiles."""
    chain = rand_chain(3000 + seed, allow_var=False, allow_null=False)
    B = CompiledSchema(chain, 0).fixed_blob_size
    pad = (-(B + 2)) % 4 + 4 * (seed % 4)
    if pad == 0:
        pad = 4
    while B + 2 + pad < 16:
        pad += 4
    chain2 = SChain(*chain.Schemas, SStringLen(pad))
    assert CompiledSchema(chain2, 0).fixed_blob_size % 4 == 0
    n = [1, 63, 1000, 4097, 20001, 257][seed % 6]
    hc = HostColumns.from_rows(chain2, rand_rows(chain2, n, seed, nil_p=0.0))
    hc.valid = [None] * len(hc.valid)
    assert_same_encoding(chain2, hc, 0, f"variant {variant} seed {seed} n {n}",
                         flags=_lib.ENC_FIXED_VARIANT(variant))


@pytest.mark.parametrize("n", [1, 2, 15, 16, 17, 63, 64, 65, 1000, 4097])
def test_fixed_tail_tiles(n):
    cfg = CONFIGS["M"]
    assert_same_encoding(cfg.chain, make_columns(cfg, n=n), 0, f"M n={n}")


@pytest.mark.parametrize("name,n", [("C1", 1000), ("C2", 100_003), ("M", 100_001), ("C3", 50_000),
                                    ("C4", 65_537), ("C5", 20_000)])
def test_configs_vs_oracle(name, n):
    cfg = CONFIGS[name]
    hc = make_columns(cfg, n=n)
    assert_same_encoding(cfg.chain, hc, cfg.mode, name)
    assert_same_encoding(cfg.chain, hc, cfg.mode, name + " single pass", fused=True)


def test_overflow_13bit_and_large_blob():
    # offsets >= 8192 are truncated exactly like typetags.EncodeHeader (Q1)
    chain = SChain(SInt16, SVariableString(), SInt16, STuple(SVariableString(), SInt16))
    rows = [[1, "x" * 9000, 2, ["y" * 10, 3]], [4, "short", 5, ["z" * 8200, 6]], [7, "", 8, None]]
    hc = HostColumns.from_rows(chain, rows)
    a0, o0, s0 = ob.encode(chain, hc, 0)
    a1, o1, s1 = gpu_encode(chain, hc, 0)
    assert np.array_equal(a0, a1) and np.array_equal(o0, o1) and np.array_equal(s0, s1)
    assert s1[0] & 0x80000000 and s1[1] & 0x80000000 and s1[2] == 0


def test_empty_batch_and_empty_chain():
    T = torch()
    s = CompiledSchema(SChain(), 0)
    hc = HostColumns.from_rows(SChain(), [[], []])
    a, o, st = gpu_encode(SChain(), hc, 0)
    assert bytes(a) == bytes.fromhex("1000") * 2  # Pack() of an empty PutAccess
    a, o, st = gpu_encode(SChain(), hc, 1)
    assert a.size == 0  # packable.Pack() with no args
    del s, T


# --------------------------------------------------------------- decode ----
def gpu_decode(chain, arena_np, offs_np, n, stride=0):
    T = torch()
    s = CompiledSchema(chain, 0)
    arena = T.from_numpy(arena_np if arena_np.size else np.zeros(16, np.uint8)).to("cuda:0")
    offs = None if stride else T.from_numpy(offs_np.astype(np.int64)).to("cuda:0")
    out, st = decode_batch(s, arena, offs, n, stride=stride)
    T.cuda.synchronize()
    return out, st.cpu().numpy().astype(np.uint32)


def assert_same_decode(chain, arena, offs, n, what="", stride=0, gpu=None):
    """Statuses must match for every blob; leaf columns for every blob that
    decodes (status 0).  DecodeBuffer returns (nil, err) on failure
    (schema/schema.go:900-903), so a failing blob's columns are unspecified
    (the fixed-layout fast path may leave tile data in them)."""
    o_out, o_st = ob.decode(chain, arena, offs, n, stride=stride, nthreads=8)
    g_out, g_st = gpu_decode(chain, arena, offs, n, stride) if gpu is None else gpu
    if not np.array_equal(o_st, g_st):
        bad = int(np.nonzero(o_st != g_st)[0][0])
        raise AssertionError(f"{what}: status blob {bad}: oracle {o_st[bad]:#x} gpu {g_st[bad]:#x}")
    ok = o_st[:n] == 0
    for c, sp in enumerate(o_out.specs):
        for name in ("data", "valid", "start", "length"):
            a = getattr(o_out, name)[c]
            b = getattr(g_out, name)[c]
            if a is None:
                continue
            bn = b.cpu().numpy()
            if name == "start":
                bn = bn.astype(np.uint64)
            if name == "length":
                bn = bn.astype(np.uint32)
            if name == "data":
                w = sp.width
                a2, b2 = a[: n * w].reshape(n, w), bn[: n * w].reshape(n, w)
                same = np.array_equal(a2[ok], b2[ok])
            else:
                same = np.array_equal(a[:n][ok], bn[:n][ok])
            assert same, f"{what}: column {c} {name}"
    return g_st


@pytest.mark.parametrize("case", G["decode"], ids=[c["id"] for c in G["decode"]])
def test_golden_decode(case):
    src = next((c for c in G["encode"] if c["id"] == case["input_from"]), None)
    inp = next((c for c in G["inputs"] if c["id"] == case["input_from"]), None)
    if src is not None:
        blob = bytes.fromhex(src["hex"])
    elif inp is not None:
        ch = chain_of(inp["schema"])
        blob = bytes(ob.encode(ch, HostColumns.from_rows(ch, [unwrap(inp["row"])]), MODES[inp["mode"]])[0])
    else:
        eq = next(c for c in G["equal"] if c["id"] == case["input_from"])
        v = eq["variants"][0]
        ch = chain_of(v["schema"])
        blob = bytes(ob.encode(ch, HostColumns.from_rows(ch, [unwrap(eq["row"])]), MODES[v["mode"]])[0])
    chain = chain_of(case["schema"])
    arena = np.frombuffer(blob, np.uint8).copy()
    st = assert_same_decode(chain, arena, np.asarray([0, len(blob)], np.uint64), 1, case["id"])
    assert int(st[0]) == case["expect_status"]


@pytest.mark.parametrize("seed", range(40))
def test_random_decode_roundtrip(seed):
    chain = rand_chain(seed)
    hc = HostColumns.from_rows(chain, rand_rows(chain, 300, seed + 99))
    arena, offs, _ = ob.encode(chain, hc, 0)
    st = assert_same_decode(chain, arena, offs, hc.n, f"seed {seed}")
    # Reference quirk: a present EMPTY tuple/map is written by BeginX/EndNested
    # as the 2-byte blob 10 00 (access/put.go:637-652), which NewSeqGetAccess
    # rejects (len < 4, seqget.go:23), so DecodeBuffer cannot read it back.
    has_empty = any(n.kind in ("tuple", "map") and not n.children for n, *_ in chain.walk())
    if not has_empty:
        assert (st == 0).all()


@pytest.mark.parametrize("nested", [False, True])
def test_named_tuple_rules(nested):
    """TupleSchemaNamed (schema.go:1726-1810), explicit statuses as well as
    the oracle's: FieldNames shorter than Schemas -> encoding a present value
    fails (ErrEncode wrapping ErrConstraintViolated, or ErrInvalidFormat when a
    parent tuple wraps it), a nil one encodes; every decode fails at position
    0 (top level) or as ErrInvalidFormat at the parent's position (nested)."""
    from packos_amd.schema import STupleNamed
    bad = STupleNamed(["a"], SInt32, SInt16)
    chain = SChain(SInt16, STuple(bad) if nested else bad, SInt16)
    rows = [[1, [[7, 8]] if nested else [7, 8], 2], [3, [None] if nested else None, 4]] * 50
    hc = HostColumns.from_rows(chain, rows)
    assert_same_encoding(chain, hc, 0, "named mismatch")
    _, _, st = gpu_encode(chain, hc, 0)
    enc_present = 4 | ((1 if nested else 3) << 24)
    assert st[0] == enc_present and st[1] == 0
    good = STupleNamed(["a", "b"], SInt32, SInt16)
    ok_chain = SChain(SInt16, STuple(good) if nested else good, SInt16)
    arena, offs, _ = ob.encode(ok_chain, HostColumns.from_rows(ok_chain, rows), 0)
    st = assert_same_decode(chain, arena, offs, len(rows), "named mismatch decode")
    # the names check runs before precheck: a nil named tuple fails too
    want = (1 | (2 << 8)) if nested else (3 | (1 << 8))
    assert int(st[0]) == want and int(st[1]) == want


@pytest.mark.parametrize("k,w", [(6, 8), (12, 8), (15, 8), (15, 4), (13, 8)])
def test_decode_long_static_prefix(k, w):
    """A flat chain whose static prefix (header block + k fixed fields) is
    longer than the decoder's per-blob LDS window, then a trailing var field:
    blobs large enough for per-blob windows, at unaligned arena offsets.  The
    flat fast path must not read the prefix's tail from the (short) window."""
    leaf = SInt64 if w == 8 else SInt32
    chain = SChain(*([leaf] * k), SVariableString())
    rng = random.Random(k * 31 + w)
    rows = [[rng.getrandbits(8 * w) for _ in range(k)] +
            ["".join(chr(rng.randint(0x20, 0x7E)) for _ in range(rng.randint(0, 300)))] for _ in range(3000)]
    hc = HostColumns.from_rows(chain, rows)
    arena, offs, _ = ob.encode(chain, hc, 0)
    st = assert_same_decode(chain, arena, offs, hc.n, f"k={k} w={w}")
    assert (st == 0).all()


@pytest.mark.parametrize("seed", range(40))
def test_random_decode_corrupted(seed):
    # flip header bytes / truncate blobs: every error code, position and panic
    # must match the oracle's SeqGetAccess restatement
    rng = np.random.default_rng(seed)
    chain = rand_chain(seed)
    hc = HostColumns.from_rows(chain, rand_rows(chain, 400, seed + 5))
    arena, offs, _ = ob.encode(chain, hc, 0)
    arena = arena.copy()
    offs = offs.copy()
    n = hc.n
    for i in range(n):
        a, b = int(offs[i]), int(offs[i + 1])
        r = rng.random()
        if r < 0.4 and b - a > 0:
            k = int(rng.integers(0, min(b - a, 24)))
            arena[a + k] = rng.integers(0, 256)
        elif r < 0.5 and b - a > 0:
            arena[a + int(rng.integers(0, b - a))] ^= 1 << int(rng.integers(0, 8))
    # truncate some blobs by shifting their end offsets inward (keeps monotone)
    cut = rng.random(n) < 0.1
    ends = offs[1:].astype(np.int64)
    starts = offs[:-1].astype(np.int64)
    ends_cut = np.where(cut, starts + (ends - starts) // 2, ends)
    # decode with an explicit [start, end) per blob: build a gapped arena
    pieces, noffs = [], [0]
    for i in range(n):
        pieces.append(arena[starts[i]:ends_cut[i]])
        noffs.append(noffs[-1] + int(ends_cut[i] - starts[i]))
    arena2 = np.concatenate(pieces) if pieces else np.zeros(0, np.uint8)
    assert_same_decode(chain, arena2, np.asarray(noffs, np.uint64), n, f"corrupt seed {seed}")


class _RawDevBuf:
    """An exactly sized hipMalloc allocation (torch's caching allocator
    rounds up to 2 MiB segments, hiding over-reads past an arena's end)."""

    def __init__(self, data: np.ndarray):
        T = torch()
        self.hip = C.CDLL("libamdhip64.so")
        self.size = (data.size + 4095) // 4096 * 4096
        p = C.c_void_p()
        assert self.hip.hipMalloc(C.byref(p), C.c_size_t(self.size)) == 0
        self.base = p.value
        self.ptr = self.base + self.size - data.size   # arena ends at the allocation's (page) end
        assert self.hip.hipMemcpy(C.c_void_p(self.ptr), data.ctypes.data_as(C.c_void_p),
                                  C.c_size_t(data.size), 1) == 0
        self.device = T.device("cuda:0")

    def data_ptr(self):
        return self.ptr

    def free(self):
        self.hip.hipDeviceSynchronize()
        self.hip.hipFree(C.c_void_p(self.base))


@pytest.mark.parametrize("cfg,seed", [("M", 0), ("M", 1), ("C1", 2)])
def test_decode_fixed_truncated_exact_alloc(cfg, seed):
    """A fixed-schema batch whose blobs are truncated (end offsets pulled
    inward) decoded from an arena that ends exactly at the end of its
    allocation, on a page boundary: the fixed-layout tile staging must stop
    at the tile's last offset, and statuses match the oracle (tiles with a
    truncated blob are not contiguous: the per-blob path)."""
    T = torch()
    rng = np.random.default_rng(seed)
    c = CONFIGS[cfg]
    if CompiledSchema(c.chain, 0).fixed_blob_size <= 0:
        pytest.skip("not a fixed schema")
    n = 3000
    hc = make_columns(c, n=n, seed=seed)
    arena, offs, _ = ob.encode(c.chain, hc, 0, nthreads=8)
    starts, ends = offs[:-1].astype(np.int64), offs[1:].astype(np.int64)
    cut = rng.random(n) < 0.02
    cut[-1] = True                                   # the last tile runs short too
    ends_cut = np.where(cut, starts + (ends - starts) // 3, ends)
    pieces, noffs = [], [0]
    for i in range(n):
        pieces.append(arena[starts[i]:ends_cut[i]])
        noffs.append(noffs[-1] + int(ends_cut[i] - starts[i]))
    pad = (-noffs[-1]) % 16                          # keep the arena base 16-B aligned
    arena2 = np.concatenate(pieces + [np.zeros(0, np.uint8)])
    buf = np.concatenate([np.zeros(pad, np.uint8), arena2])
    noffs = np.asarray(noffs, np.uint64) + np.uint64(pad)
    raw = _RawDevBuf(buf)
    try:
        s = CompiledSchema(c.chain, 0)
        do = T.from_numpy(noffs.astype(np.int64)).to("cuda:0")
        out, st = decode_batch(s, raw, do, n)
        T.cuda.synchronize()
        g = (out, st.cpu().numpy().astype(np.uint32))
    finally:
        raw.free()
    got = assert_same_decode(c.chain, buf, noffs, n, f"truncated {cfg}", gpu=g)
    assert (got[~cut] == 0).all()


@pytest.mark.parametrize("seed", range(12))
def test_decode_generic_kernel(seed, monkeypatch):
    """PACKOS_DECODE_GENERIC: the thread-per-blob decoder (k_decode_win) even
    where the fixed-layout fast path applies, on clean and corrupted batches."""
    monkeypatch.setenv("PACKOS_DECODE_GENERIC", "1")
    rng = np.random.default_rng(77 + seed)
    chain = rand_chain(seed)
    hc = HostColumns.from_rows(chain, rand_rows(chain, 300, seed + 3))
    arena, offs, _ = ob.encode(chain, hc, 0)
    assert_same_decode(chain, arena, offs, hc.n, f"nowin seed {seed}")
    arena = arena.copy()
    for i in range(0, hc.n, 4):
        a, b = int(offs[i]), int(offs[i + 1])
        if b > a:
            arena[a + int(rng.integers(0, min(b - a, 16)))] ^= np.uint8(1 << int(rng.integers(0, 8)))
    assert_same_decode(chain, arena, offs, hc.n, f"nowin corrupt seed {seed}")


@pytest.mark.parametrize("seed", range(30))
def test_fixed_decode_fast_path(seed):
    """Fixed-size schemas take the tiled fast path (k_decode_fixed).  In-place
    corruption keeps the tiles contiguous, so corrupted blobs go through the
    constant-byte check and fall back to decode_blob inside the same tile.
    Covers offsets and stride addressing and ragged last tiles."""
    rng = np.random.default_rng(1000 + seed)
    chain = rand_chain(seed, allow_var=False, allow_null=False)
    s = CompiledSchema(chain, 0)
    B = s.fixed_blob_size
    if B <= 0:
        pytest.skip("schema has no fixed layout")
    n = int(rng.integers(1, 3000))
    hc = HostColumns.from_rows(chain, rand_rows(chain, n, seed + 7))
    arena, offs, _ = ob.encode(chain, hc, 0)
    arena = arena.copy()
    for i in np.nonzero(rng.random(n) < 0.05)[0]:
        a, b = int(offs[i]), int(offs[i + 1])
        if b > a:
            arena[a + int(rng.integers(0, b - a))] ^= np.uint8(1 << int(rng.integers(0, 8)))
    st = assert_same_decode(chain, arena, offs, n, f"fast offs seed {seed}")
    if np.all(np.diff(offs.astype(np.int64)) == B):  # no nil containers: stride addressing
        st2 = assert_same_decode(chain, arena, offs, n, f"fast stride seed {seed}", stride=B)
        assert np.array_equal(st, st2)



@pytest.mark.parametrize("tile", [None, "1024", "49152"], ids=["tile_default", "tile_1k", "tile_48k"])
@pytest.mark.parametrize("B", [32, 64, 128, 256, 512, 1024, 48, 272])
def test_fixed_decode_blob_sizes(B, tile, monkeypatch):
    """k_decode_fixed across blob sizes (power-of-two 32..1024 B and two
    others; tile T = 16 * floor(1024 / B) blobs): narrow columns (int16 /
    bool / int32 / int64) next to a string filling the blob, a ragged last
    tile, corrupted blobs in the mix, offsets and stride addressing; decode
    tiles of 1 KB / 48 KB staged bytes (PACKOS_DEC_TILE_BYTES) besides the
    default."""
    if tile:
        monkeypatch.setenv("PACKOS_DEC_TILE_BYTES", tile)
    L = B - 2 * 6 - (2 + 1 + 4 + 8)
    chain = SChain(SInt16, SBool, SInt32, SInt64, SStringLen(L))
    s = CompiledSchema(chain, 0)
    assert s.fixed_blob_size == B
    rng = np.random.default_rng(B)
    n = 3001
    rows = [[int(rng.integers(-32768, 32767)), bool(rng.integers(0, 2)), int(rng.integers(-2**31, 2**31 - 1)),
             int(rng.integers(-2**62, 2**62)), bytes(rng.integers(32, 127, L).astype(np.uint8)).decode()]
            for _ in range(n)]
    hc = HostColumns.from_rows(chain, rows)
    arena, offs, _ = ob.encode(chain, hc, 0)
    arena = arena.copy()
    for i in np.nonzero(rng.random(n) < 0.03)[0]:
        arena[int(offs[i]) + int(rng.integers(0, B))] ^= np.uint8(1 << int(rng.integers(0, 8)))
    st = assert_same_decode(chain, arena, offs, n, f"B={B}")
    st2 = assert_same_decode(chain, arena, offs, n, f"B={B} stride", stride=B)
    assert np.array_equal(st, st2)


@pytest.mark.parametrize("seed", range(10))
def test_fixed_decode_random_gap(seed):
    """k_decode_fixed on random fixed schemas: in-place corruption (check
    failures inside contiguous tiles), a gap between two blobs (one tile not
    contiguous), offsets and stride addressing."""
    rng = np.random.default_rng(5000 + seed)
    chain = rand_chain(seed + 100, allow_var=False, allow_null=False)
    s = CompiledSchema(chain, 0)
    B = s.fixed_blob_size
    if B <= 0:
        pytest.skip("schema has no fixed layout")
    n = int(rng.integers(2000, 12000))
    hc = HostColumns.from_rows(chain, rand_rows(chain, n, seed + 9))
    arena, offs, _ = ob.encode(chain, hc, 0)
    arena = arena.copy()
    for i in np.nonzero(rng.random(n) < 0.02)[0]:
        a, b = int(offs[i]), int(offs[i + 1])
        if b > a:
            arena[a + int(rng.integers(0, b - a))] ^= np.uint8(1 << int(rng.integers(0, 8)))
    st = assert_same_decode(chain, arena, offs, n, f"fixed offs seed {seed}")
    if np.all(np.diff(offs.astype(np.int64)) == B):
        st2 = assert_same_decode(chain, arena, offs, n, f"fixed stride seed {seed}", stride=B)
        assert np.array_equal(st, st2)
    # 16 zero bytes between blobs g - 1 and g: g's tile is not contiguous
    g = int(rng.integers(1, n))
    cut = int(offs[g])
    arena2 = np.concatenate([arena[:cut], np.zeros(16, np.uint8), arena[cut:]])
    offs2 = offs.astype(np.uint64).copy()
    offs2[g:] += np.uint64(16)
    assert_same_decode(chain, arena2, offs2, n, f"fixed gap seed {seed}")


@pytest.mark.parametrize("name", ["M", "C2", "C4"])
def test_fixed_decode_fast_matches_generic(name, monkeypatch):
    """Fast path and the generic thread-per-blob kernel give identical columns."""
    T = torch()
    cfg = CONFIGS[name]
    n = 5000
    hc = make_columns(cfg, n=n)
    arena, offs, _ = ob.encode(cfg.chain, hc, 0, nthreads=8)
    f_out, f_st = gpu_decode(cfg.chain, arena, offs, n)
    monkeypatch.setenv("PACKOS_DECODE_GENERIC", "1")
    g_out, g_st = gpu_decode(cfg.chain, arena, offs, n)
    assert (f_st == 0).all() and (g_st == 0).all()
    for c in range(len(f_out.schema.specs)):
        for name_ in ("data", "valid"):
            a, b = getattr(f_out, name_)[c], getattr(g_out, name_)[c]
            if a is not None:
                assert T.equal(a, b), f"{name} column {c} {name_}"


@pytest.mark.parametrize("name,n", [("C1", 1000), ("C2", 100_003), ("C3", 30_000), ("C4", 30_000), ("M", 30_000),
                                    ("C5", 5000)])
def test_config_decode(name, n):
    cfg = CONFIGS[name]
    hc = make_columns(cfg, n=n)
    arena, offs, _ = ob.encode(cfg.chain, hc, cfg.mode, nthreads=8)
    st = assert_same_decode(cfg.chain, arena, offs, n, name)
    assert (st == 0).all()


@pytest.mark.parametrize("name,n", [("C1", 1000), ("C2", 20_001), ("C3", 20_001), ("C4", 9_999), ("M", 20_001),
                                    ("C5", 3000)])
def test_config_roundtrip(name, n):
    """encode -> decode -> re-encode on the GPU reproduces the bytes
    (access/put_test.go:12-42, packable/pack_test.go:99-118 round trips; C1
    is the reference's 1k-tuple plumbing case at full size)."""
    T = torch()
    cfg = CONFIGS[name]
    hc = make_columns(cfg, n=n)
    s = CompiledSchema(cfg.chain, cfg.mode)
    r = encode_batch(s, DeviceColumns.from_host(s, hc, "cuda:0"))
    offs = r.offsets if r.offsets is not None else T.arange(n + 1, device="cuda:0", dtype=T.int64) * r.blob_size
    out, st = decode_batch(s, r.arena, offs, n)
    T.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    arena = r.arena[: r.total].cpu().numpy()
    back = HostColumns(cfg.chain, n)
    for c, sp in enumerate(back.specs):
        if sp.fixed:
            back.data[c] = out.data[c][: n * sp.width].cpu().numpy().copy()
        if sp.var:
            st0 = out.start[c][:n].cpu().numpy().view(np.uint64)
            ln = out.length[c][:n].cpu().numpy().view(np.uint32).astype(np.int64)
            o = np.zeros(n + 1, np.int64)
            np.cumsum(ln, out=o[1:])
            idx = (np.repeat(st0.astype(np.int64) - o[:-1], ln) + np.arange(o[-1])) if o[-1] else np.zeros(0, np.int64)
            back.data[c] = arena[idx] if o[-1] else np.zeros(0, np.uint8)
            back.offsets[c] = o.astype(np.uint32)
        if sp.has_valid:
            back.valid[c] = out.valid[c][:n].cpu().numpy().copy()
    a2, o2, s2 = gpu_encode(cfg.chain, back, cfg.mode)
    assert np.array_equal(a2, arena)
    assert np.array_equal(o2, offs.cpu().numpy().astype(np.uint64))


def test_full_size_c4_vs_oracle():
    """Config C4 at its full 4,194,304 blobs (1 GiB of output) against the
    oracle, byte for byte."""
    cfg = CONFIGS["C4"]
    hc = make_columns(cfg, n=cfg.shard)
    assert hc.n == 4_194_304
    assert_same_encoding(cfg.chain, hc, cfg.mode, "C4 full")


# ------------------------------------------------------------ GetAccess ----
@pytest.mark.parametrize("case", G["get"], ids=[c["id"] for c in G["get"]])
def test_golden_get(case):
    T = torch()
    buf = np.frombuffer(bytes.fromhex(case["hex"]), np.uint8).copy()
    arena = T.from_numpy(buf).to("cuda:0")
    offs = T.tensor([0, buf.size], dtype=T.int64, device="cuda:0")
    for q in case["queries"]:
        s0, ln, tg, st = get_field_batch(arena, offs, 1, q["path"], q["tag"], q["width"])
        T.cuda.synchronize()
        assert int(st[0]) == 0
        a = int(s0[0])
        assert bytes(buf[a:a + int(ln[0])]).hex() == q["expect"]


@pytest.mark.parametrize("seed", range(20))
def test_random_get(seed):
    T = torch()
    rng = np.random.default_rng(seed)
    chain = rand_chain(seed)
    hc = HostColumns.from_rows(chain, rand_rows(chain, 200, seed))
    arena, offs, _ = ob.encode(chain, hc, 0)
    arena = arena.copy()
    for i in range(0, hc.n, 3):  # corrupt a third of the blobs
        a, b = int(offs[i]), int(offs[i + 1])
        if b > a:
            arena[a + int(rng.integers(0, min(8, b - a)))] = rng.integers(0, 256)
    da = T.from_numpy(arena).to("cuda:0")
    do = T.from_numpy(offs.astype(np.int64)).to("cuda:0")
    for _ in range(12):
        depth = int(rng.integers(1, 4))
        path = [int(rng.integers(0, 6)) for _ in range(depth)]
        tag = int(rng.choice([1, 3, 4, 5, 6, 7]))
        width = int(rng.choice([-1, 1, 2, 4, 8]))
        o = ob.get_field_batch(arena, offs, hc.n, path, tag, width)
        g = get_field_batch(da, do, hc.n, path, tag, width)
        T.cuda.synchronize()
        gs = [x.cpu().numpy() for x in g]
        assert np.array_equal(o[3], gs[3]), (path, tag, width)
        okm = o[3] == 0
        assert np.array_equal(o[0][okm], gs[0].astype(np.uint64)[okm])
        assert np.array_equal(o[1][okm], gs[1].astype(np.uint32)[okm])


GETTERS = [(0, 1, 1), (0, 1, 2), (0, 1, 4), (0, 1, 8), (0, 3, 4), (0, 3, 8), (0, 5, 1),
           (1, 1, 4), (1, 1, 8), (1, 3, 8), (1, 5, 1), (2, 6, 0), (2, 4, 0), (2, 7, 0),
           (3, 0, 0), (4, 0, 0), (5, 0, 0)]


@pytest.mark.parametrize("seed", range(16))
def test_random_get_batch(seed):
    """packos_get_batch vs or_get_batch for every getter family (FIXED,
    NULLABLE, SPAN, INT, FLOAT) with typed gather, on random schemas whose
    nullable columns hold nils (width-0 fields) and a third of the blobs
    corrupted."""
    T = torch()
    rng = np.random.default_rng(100 + seed)
    chain = rand_chain(seed)
    hc = HostColumns.from_rows(chain, rand_rows(chain, 300, seed))
    arena, offs, _ = ob.encode(chain, hc, int(rng.integers(0, 2)))
    arena = arena.copy()
    for i in range(0, hc.n, 3):
        a, b = int(offs[i]), int(offs[i + 1])
        if b > a:
            arena[a + int(rng.integers(0, min(8, b - a)))] = rng.integers(0, 256)
    da = T.from_numpy(arena).to("cuda:0")
    do = T.from_numpy(offs.astype(np.int64)).to("cuda:0")
    for _ in range(10):
        depth = int(rng.integers(1, 3))
        path = [int(rng.integers(0, 6)) for _ in range(depth)]
        getter, tag, width = GETTERS[int(rng.integers(0, len(GETTERS)))]
        o = ob.get_batch(arena, offs, hc.n, path, getter, tag, width)
        g = [None if x is None else x.cpu().numpy() for x in get_batch(da, do, hc.n, path, getter, tag, width)]
        what = (path, getter, tag, width)
        assert np.array_equal(o[4], g[4]), what
        assert np.array_equal(o[3], g[3]), what
        assert np.array_equal(o[1], g[1].astype(np.uint64)), what
        assert np.array_equal(o[2], g[2].astype(np.uint32)), what
        if o[0] is None:
            assert g[0] is None
        else:
            assert np.array_equal(o[0], g[0]), what
            # GetInt-style call: value + status only, spans not written
            v = get_batch(da, do, hc.n, path, getter, tag, width, spans=False)
            assert v[1] is None and v[2] is None and v[3] is None
            assert np.array_equal(o[0], v[0].cpu().numpy()), what
            assert np.array_equal(o[4], v[4].cpu().numpy()), what


def test_get_batch_spans_required_without_gather():
    """spans=False is refused where no typed value carries the result (SPAN,
    ANY, values=False): the C ABI returns PACKOS_E_INVALID."""
    T = torch()
    da = T.zeros(64, dtype=T.uint8, device="cuda:0")
    for getter in (GET_SPAN, GET_ANY):
        with pytest.raises(ValueError):
            get_batch(da, None, 4, [0], getter, 0, 0, stride=16, spans=False)
    with pytest.raises(ValueError):
        get_batch(da, None, 4, [0], GET_INT, 0, 0, stride=16, values=False, spans=False)
    st = T.zeros(4, dtype=T.uint8, device="cuda:0")
    path = (C.c_int32 * 1)(0)
    rc = _lib.lib().packos_get_batch(da.data_ptr(), None, 16, 4, path, 1, GET_SPAN, 0, 0, None, 0,
                                     None, None, None, st.data_ptr(), None)
    assert rc == -1   # PACKOS_E_INVALID


def test_get_batch_nullable_and_any_width():
    """Hand-built blob with nil (width-0) fields: GetNullable* returns nil
    before checking the tag, GetInt/GetFloating take any legal width."""
    T = torch()
    blob = _blob_with_nils()
    buf = np.frombuffer(blob * 3, np.uint8).copy()
    offs = np.arange(4, dtype=np.uint64) * len(blob)
    da = T.from_numpy(buf).to("cuda:0")
    for path, getter, tag, width in [([1], 1, 5, 1), ([1], 3, 0, 0), ([7], 3, 0, 0), ([2], 4, 0, 0),
                                     ([5], 4, 0, 0), ([3], 0, 5, 1), ([6], 3, 0, 0), ([4], 2, 6, 0)]:
        o = ob.get_batch(buf, offs, 3, path, getter, tag, width)
        g = get_batch(da, None, 3, path, getter, tag, width, stride=len(blob))
        T.cuda.synchronize()
        assert np.array_equal(o[4], g[4].cpu().numpy())
        if o[0] is not None:
            assert np.array_equal(o[0], g[0].cpu().numpy())


@pytest.mark.parametrize("vw", [4, 8, 16, 24])
def test_get_batch_wide_value_narrow_buffer(vw):
    """A 16-B FIXED value gathered into rows of value_width bytes: the first
    min(16, vw) payload bytes, zero-padded (never the 8-B register path)."""
    T = torch()
    chain = SChain(SInt16, SStringLen(16))
    rows = [[i, "".join(chr(0x41 + (i + k) % 26) for k in range(16))] for i in range(300)]
    hc = HostColumns.from_rows(chain, rows)
    arena, offs, _ = ob.encode(chain, hc, 0)
    da = T.from_numpy(arena).to("cuda:0")
    n = hc.n
    vals = T.zeros((n, vw), dtype=T.uint8, device="cuda:0")
    st = T.zeros(n, dtype=T.uint8, device="cuda:0")
    p = (C.c_int32 * 1)(1)
    B = int(offs[1])
    assert _lib.lib().packos_get_batch(da.data_ptr(), None, B, n, p, 1, 0, 6, 16, vals.data_ptr(), vw,
                                       None, None, None, st.data_ptr(), None) == 0
    T.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    got = vals.cpu().numpy()
    for i in range(n):
        want = rows[i][1].encode()[:vw].ljust(vw, b"\0")
        assert bytes(got[i]) == want, i


def _rand_map_value(rng, depth):
    """(tag, payload) of a random GetAny-relevant value: ints of legal and
    illegal widths, floats, strings, bools, tuples, nil / nested maps."""
    from test_oracle_golden import pack_fields
    k = int(rng.integers(0, 10))
    if k < 3:
        return 1, bytes(rng.integers(0, 256, int(rng.choice([0, 1, 2, 3, 4, 8])), dtype=np.uint8))
    if k == 3:
        return 3, bytes(rng.integers(0, 256, int(rng.choice([0, 4, 8, 2])), dtype=np.uint8))
    if k < 6:
        return 6, bytes(rng.integers(97, 123, int(rng.integers(0, 12)), dtype=np.uint8))
    if k == 6:
        return int(rng.choice([5, 4])), b"\x01"
    if depth >= 3 or k == 7:
        return 7, b""
    return 7, _rand_map(rng, depth + 1)


def _rand_map(rng, depth=0):
    from test_oracle_golden import pack_fields
    fields = []
    for _ in range(int(rng.integers(0, 5))):
        fields.append((6 if rng.random() > 0.05 else 1, bytes(rng.integers(97, 123, int(rng.integers(1, 6)),
                                                                               dtype=np.uint8))))
        fields.append(_rand_map_value(rng, depth))
    if rng.random() < 0.05 and fields:
        fields.pop()   # odd field count
    return pack_fields(fields)


@pytest.mark.parametrize("seed", range(6))
def test_random_get_map_batch(seed):
    """packos_get_map_batch vs or_get_map_batch (GetMapStr / GetMapAny) on
    random blobs holding maps of mixed values (nested maps, bools, tuples,
    illegal int widths, nil maps), a fifth of the blobs corrupted."""
    from test_oracle_golden import pack_fields
    T = torch()
    rng = np.random.default_rng(700 + seed)
    blobs = []
    for i in range(2000):
        fields = [(1, b"\x01\x00"), (7, _rand_map(rng)), (4, pack_fields([(7, _rand_map(rng))]))]
        b = bytearray(pack_fields(fields))
        if i % 5 == 0 and b:
            b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
        blobs.append(bytes(b))
    offs = np.zeros(len(blobs) + 1, np.uint64)
    np.cumsum([len(b) for b in blobs], out=offs[1:])
    arena = np.frombuffer(b"".join(blobs), np.uint8).copy()
    da = T.from_numpy(arena).to("cuda:0")
    do = T.from_numpy(offs.astype(np.int64)).to("cuda:0")
    for path in ([1], [2, 0], [0], [3]):
        for flags in (0, 1):
            for mp in (0, 2, 8):
                o = ob.get_map_batch(arena, offs, len(blobs), path, flags, mp)
                g = [x.cpu().numpy() for x in get_map_batch(da, do, len(blobs), path, flags, mp)]
                what = (path, flags, mp)
                assert np.array_equal(o[6], g[6]), what
                assert np.array_equal(o[0], g[0].astype(np.uint32)), what
                for a, b_ in zip(o[1:6], g[1:6]):
                    assert np.array_equal(a, b_.astype(a.dtype)), what
    st = ob.get_map_batch(arena, offs, len(blobs), [1], 1, 8)[6]
    assert len(set(st.tolist())) >= 3   # the mix exercises ok, error and nil-map outcomes


def test_get_map_golden():
    """The reference's map known answers (access/get_test.go:46-126) on the GPU."""
    T = torch()
    for c in G["maps"]:
        buf = np.frombuffer(bytes.fromhex(c["hex"]), np.uint8)
        reps = np.concatenate([buf] * 3)
        da = T.from_numpy(reps).to("cuda:0")
        pr, ks, kl, vs, vl, vt, st = [x.cpu().numpy() for x in
                                      get_map_batch(da, None, 3, c["path"], c["flags"], 4, stride=buf.size)]
        for i in range(3):
            assert st[i] == 0 and pr[i] == len(c["pairs"]), c["id"]
            got = [(bytes(reps[int(ks[i, j]):int(ks[i, j]) + int(kl[i, j])]).hex(), int(vt[i, j]),
                    bytes(reps[int(vs[i, j]):int(vs[i, j]) + int(vl[i, j])]).hex()) for j in range(pr[i])]
            assert got == [tuple(p) for p in c["pairs"]], c["id"]


def _blob_with_nils():
    from test_oracle_golden import pack_fields
    return pack_fields(NIL_FIELDS)


from test_oracle_golden import NIL_FIELDS  # noqa: E402


# ---------------------------------------------------------- value checks ----
# Range (SInt*.Range, schema.go:1172-1364), SDateRange (:2188-2250), Prefix /
# Suffix (:1144-1158), DefaultDecodeValue (:1131, 283-285): the encode status
# (ErrEncode + top-level field + the leaf's code), decode statuses and default
# views must match the oracle blob for blob.
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("seed", range(24))
def test_checked_schema_encode(seed, mode):
    chain = rand_checked_chain(seed)
    hc = HostColumns.from_rows(chain, rand_checked_rows(chain, 700, seed + 5))
    assert_same_encoding(chain, hc, mode, f"checked seed {seed}")


@pytest.mark.parametrize("seed", range(16))
def test_checked_schema_encode_fixed(seed):
    chain = rand_checked_chain(seed, allow_var=False, allow_null=False)
    hc = HostColumns.from_rows(chain, rand_checked_rows(chain, 3001, seed + 7, nil_p=0.0))
    assert CompiledSchema(chain).fixed_blob_size > 0
    assert_same_encoding(chain, hc, 0, f"checked fixed seed {seed}")


@pytest.mark.parametrize("seed", range(24))
def test_checked_schema_decode(seed):
    chain = rand_checked_chain(seed)
    hc = HostColumns.from_rows(chain, rand_checked_rows(chain, 700, seed + 11))
    arena, offs, _ = ob.encode(chain, hc, 0)
    assert_same_decode(chain, arena, offs, hc.n, f"checked seed {seed}")


@pytest.mark.parametrize("seed", range(16))
def test_checked_schema_decode_fast(seed):
    """Fixed layouts with value checks keep the tiled decoder; rows failing a
    check are re-decoded exactly (status from decode_blob)."""
    chain = rand_checked_chain(seed, allow_var=False, allow_null=False)
    # a named tuple whose names and schemas differ in length fails every
    # decode (schema.go:1756-1758): such a schema never takes the fast path
    names_bad = any(n.kind == "tuple" and n.names is not None and len(n.names) != len(n.children)
                    for n, *_ in chain.walk())
    assert CompiledSchema(chain).decode_fast == (not names_bad)
    hc = HostColumns.from_rows(chain, rand_checked_rows(chain, 3001, seed + 13, nil_p=0.0))
    arena, offs, _ = ob.encode(chain, hc, 0)
    B = CompiledSchema(chain).fixed_blob_size
    assert_same_decode(chain, arena, offs, hc.n, f"checked fast seed {seed}")
    assert_same_decode(chain, arena, None, hc.n, f"checked fast stride seed {seed}", stride=B)


def test_decode_default_views_resolve():
    """DecodedColumns.var_values resolves PACKOS_VIEW_DEFAULT to the literal."""
    chain = SChain(SString.DefaultDecodeValue("fallback"), SString)
    hc = HostColumns.from_rows(chain, [["", "a"], ["xy", ""], ["", ""]])
    s = CompiledSchema(chain)
    dc = DeviceColumns.from_host(s, hc, "cuda:0")
    r = encode_batch(s, dc)
    out, st = decode_batch(s, r.arena, r.offsets, hc.n)
    torch().cuda.synchronize()
    assert st.cpu().tolist() == [0, 0, 0]
    assert out.var_values(0, r.arena[: r.total]) == [b"fallback", b"xy", b"fallback"]
    assert out.var_values(1, r.arena[: r.total]) == [b"a", b"", b""]


# ------------------------------------------------------ host-resident decode ----
def _same_host_decode(chain, arena, offs, n, got, g_st, what, stride=0):
    o_out, o_st = ob.decode(chain, arena, offs, n, stride=stride, nthreads=8)
    assert np.array_equal(o_st, g_st), what
    ok = o_st[:n] == 0
    for c, sp in enumerate(o_out.specs):
        for name in ("data", "valid", "start", "length"):
            a = getattr(o_out, name)[c]
            if a is None:
                continue
            b = getattr(got, name)[c]
            if name == "data":   # rows of nil values: zero on both sides
                w = sp.width
                assert np.array_equal(a[: n * w].reshape(n, w)[ok], b[: n * w].reshape(n, w)[ok]), (what, c)
            else:
                assert np.array_equal(a[:n][ok], b[:n][ok]), (what, c, name)


@pytest.mark.parametrize("name,n,chunk,pinned", [("C3", 20000, 3000, False), ("C3", 20000, 0, True),
                                                 ("M", 10001, 4096, False), ("M", 10001, 4096, True),
                                                 ("C5", 3000, 700, False), ("C1", 1000, 0, False),
                                                 ("C4", 5001, 1024, True), ("C2", 7777, 1000, False)])
def test_decode_host_batch(name, n, chunk, pinned):
    """packos_decode_host_batch (host arena -> chunked H2D / decode / D2H ->
    host columns) vs the oracle: views are absolute host-arena offsets."""
    from packos_amd.api import decode_host_batch
    T = torch()
    cfg = CONFIGS[name]
    hc = make_columns(cfg, n=n)
    arena, offs, _ = ob.encode(cfg.chain, hc, cfg.mode, nthreads=8)
    if pinned:
        arena = T.from_numpy(np.ascontiguousarray(arena)).pin_memory().numpy()
    s = CompiledSchema(cfg.chain, cfg.mode)
    got, st = decode_host_batch(s, arena, offs, n, chunk_blobs=chunk)
    _same_host_decode(cfg.chain, arena, offs, n, got, st, name)
    B = s.fixed_blob_size
    if B > 0:   # fixed stride, no offsets
        got, st = decode_host_batch(s, arena, None, n, stride=B, chunk_blobs=chunk)
        _same_host_decode(cfg.chain, arena, None, n, got, st, name + " stride", stride=B)


def test_pipeline_reuse_across_calls():
    """One explicit packos_pipeline for many calls: more chunks than slots,
    batches that grow (buffers reallocated) and shrink (reused), pinned and
    pageable inputs, 32- and 64-bit host var offsets whose first value is not
    0, then decode of each result on the same pipeline, all vs the oracle."""
    from packos_amd.api import Pipeline
    T = torch()
    cfg = CONFIGS["C3"]
    s = CompiledSchema(cfg.chain, cfg.mode)
    p = Pipeline(s, chunk_blobs=1000, slots=3)
    for n, lo, pinned, w64 in ((5000, 0, False, False), (23456, 777, True, False), (1500, 5, False, True),
                               (9000, 123457, True, True)):
        hc = make_columns(cfg, n=n, lo=lo)
        a0, o0, s0 = ob.encode(cfg.chain, hc, cfg.mode, nthreads=8)
        for c, o in enumerate(hc.offsets):
            if o is not None:   # offsets into a bigger host arena: values start past 0
                shift = 4096 + 3 * c
                hc.data[c] = np.concatenate([np.full(shift, 0xAB, np.uint8), hc.data[c]])
                hc.offsets[c] = (o.astype(np.uint64) + shift).astype(np.uint64 if w64 else np.uint32)
        if pinned:
            for lst in (hc.data, hc.offsets):
                for c, a in enumerate(lst):
                    if a is not None:
                        lst[c] = T.from_numpy(np.ascontiguousarray(a).view(np.int64 if a.dtype == np.uint64 else a.dtype)
                                              ).pin_memory().numpy().view(a.dtype)
        a1, o1, s1 = p.encode(hc)
        assert np.array_equal(o0, o1) and np.array_equal(a0, a1) and np.array_equal(s0, s1.astype(np.uint32)), n
        got, st = p.decode(a1, o1, n)
        _same_host_decode(cfg.chain, a1, o1, n, got, st, f"pipeline n={n}")
    p.close()


def test_decode_host_batch_nonmonotone_offsets():
    """Offsets that go backwards inside a chunk: the chunk's staged range is
    [min, max) of its offsets, so every blob reads staged bytes; a blob whose
    end precedes its start fails like the oracle's."""
    from packos_amd.api import decode_host_batch
    cfg = CONFIGS["C3"]
    n = 4000
    hc = make_columns(cfg, n=n)
    arena, offs, _ = ob.encode(cfg.chain, hc, cfg.mode, nthreads=8)
    offs = offs.copy()
    rng = np.random.default_rng(5)
    for i in rng.integers(1, n - 1, size=40):   # swap a blob boundary with its neighbour's
        offs[i], offs[i + 1] = offs[i + 1], offs[i]
    offs[1000] = offs[3500]                     # a jump forward, then back
    s = CompiledSchema(cfg.chain, cfg.mode)
    got, st = decode_host_batch(s, arena, offs, n, chunk_blobs=512)
    _same_host_decode(cfg.chain, arena, offs, n, got, st, "nonmonotone")
    assert (st != 0).any() and (st == 0).any()


@pytest.mark.parametrize("seed", range(0, 40, 4))
def test_decode_host_batch_random(seed):
    """Random schemas, checked schemas and corrupted blobs; offsets that start
    past 0 at odd positions (chunk arenas staged from a 16-B aligned start)."""
    from packos_amd.api import decode_host_batch
    for chain, rows in ((rand_chain(seed), None), (rand_checked_chain(seed), "checked")):
        rr = rand_checked_rows(chain, 2100, seed + 1) if rows else rand_rows(chain, 2100, seed + 1)
        hc = HostColumns.from_rows(chain, rr)
        a0, o0, _ = ob.encode(chain, hc, 0)
        rng = np.random.default_rng(seed)
        pad = int(rng.integers(1, 40))
        arena = np.concatenate([np.full(pad, 0xEE, np.uint8), a0, np.zeros(8, np.uint8)])
        offs = o0 + pad
        for k in rng.integers(0, a0.size, size=30):   # corrupt some header bytes
            arena[pad + int(k)] ^= np.uint8(rng.integers(1, 255))
        s = CompiledSchema(chain, 0)
        got, st = decode_host_batch(s, arena, offs, hc.n, chunk_blobs=333)
        _same_host_decode(chain, arena, offs, hc.n, got, st, f"seed {seed} {rows}")
