"""k_encode_flat (encode_flat.inc, the default for flat closed-form chains)
vs the CPU oracle, bit-exact: flat closed-form chains — random leaf mixes with empty, short,
chunk-straddling and multi-page var values, tile-edge counts, column slices
(var offsets starting past 0), 64-bit offsets, the 13-bit overflow status and
a capacity overrun (ErrEncode per blob that does not fit)."""
import random

import numpy as np
import pytest

import oracle_bridge as ob
from packos_amd import _lib
from packos_amd.api import CompiledSchema, DeviceColumns
from packos_amd.columns import HostColumns
from packos_amd.configs import CONFIGS, make_columns
from packos_amd.schema import (SBool, SBytes, SChain, SInt16, SInt32, SInt64, SStringLen, SUint8,
                               SVariableBytes, SVariableString)

pytestmark = pytest.mark.gpu

# fixed leaves of at most 16 B (k_encode_flat stages them; longer ones send the
# chain to k_encode_tiles)
LEAVES = [lambda: SBool, lambda: SUint8, lambda: SInt16, lambda: SInt32, lambda: SInt64, lambda: SStringLen(5),
          lambda: SBytes(13), lambda: SStringLen(16)]
LENS = [0, 1, 3, 7, 15, 16, 17, 31, 33, 80, 255, 1000, 4000]


def torch():
    import torch as t
    return t


def flat_chain(rng):
    k = rng.randint(1, 12)
    leaves, nvar = [], 0
    for _ in range(k):
        if rng.random() < 0.4 and nvar < 4:   # k_encode_flat takes <= 4 var leaves
            leaves.append(SVariableString() if rng.random() < 0.5 else SVariableBytes())
            nvar += 1
        else:
            leaves.append(rng.choice(LEAVES)())
    if nvar == 0:
        leaves.insert(rng.randint(0, len(leaves)), SVariableBytes())
    # >= 15 static bytes before the first var value (flat_plan's condition):
    # header words of the leading fixed leaves + their widths, else an SInt64 lead
    while True:
        nlead = next(j for j, x in enumerate(leaves) if x.width <= 0 and x.kind in ("string", "bytes"))
        if 2 * (len(leaves) + 1) + sum(x.width for x in leaves[:nlead]) >= 15:
            break
        leaves.insert(0, SInt64)
    return SChain(*leaves)


def value(rng, node, lens):
    k = node.kind
    if k in ("int", "uint"):
        return rng.getrandbits(8 * node.width)
    if k == "bool":
        return rng.random() < 0.5
    n = node.width if node.width > 0 else rng.choice(lens)
    if k == "string":
        return "".join(chr(rng.randint(0x20, 0x7E)) for _ in range(n))
    return rng.randbytes(n)


def rows(chain, n, seed, lens=LENS):
    rng = random.Random(seed)
    return [[value(rng, s, lens) for s in chain.Schemas] for _ in range(n)]


def check(chain, hc, mode, what, shift=False, off64=False, kernel=None, cap_scale=1, flags=0):
    T = torch()
    s = CompiledSchema(chain, mode)
    dc = DeviceColumns.from_host(s, hc, "cuda:0")
    keep = []
    for c, o in enumerate(dc.offsets):
        if o is not None and shift:   # a column slice: offsets start past 0
            k = 1000 + 37 * c
            dc.data[c] = T.cat([T.full((k,), 0xEE, dtype=T.uint8, device="cuda:0"), dc.data[c]])
            dc.offsets[c] = o + k
    arr = dc.ctypes_array()
    if off64:   # 64-bit offsets columns (packos_column.offsets64)
        for c, o in enumerate(dc.offsets):
            if o is not None:
                o64 = o.to(T.int64).contiguous()
                keep.append(o64)
                arr[c].offsets = None
                arr[c].offsets64 = o64.data_ptr()
    a0, o0, s0 = ob.encode(chain, hc, mode, nthreads=8)
    n = hc.n
    L = _lib.lib()
    out = T.zeros(int(o0[n]) * cap_scale + 16, dtype=T.uint8, device="cuda:0")
    offs = T.full((n + 1,), -1, dtype=T.int64, device="cuda:0")
    st = T.full((n,), -1, dtype=T.int32, device="cuda:0")
    assert L.packos_encode_batch(s.handle, arr, n, out.data_ptr(), out.numel(), offs.data_ptr(), st.data_ptr(),
                                 None, 0, flags, None) == 0, L.packos_last_error()
    T.cuda.synchronize()
    if kernel:   # the encoder under test actually ran (not a silent fallback)
        ok = (kernel,) if isinstance(kernel, str) else kernel
        assert L.packos_last_encoder().decode() in ok, (what, L.packos_last_encoder())
    o1 = offs.cpu().numpy().astype(np.uint64)
    assert np.array_equal(o1, o0), f"{what}: offsets differ"
    a1 = out[: int(o0[n])].cpu().numpy()
    if not np.array_equal(a0, a1):
        bad = int(np.nonzero(a0 != a1)[0][0])
        blob = int(np.searchsorted(o0, bad, side="right") - 1)
        raise AssertionError(f"{what}: first diff at byte {bad} (blob {blob}, +{bad - int(o0[blob])})")
    assert np.array_equal(st.cpu().numpy().astype(np.uint32), s0), f"{what}: status differs"


@pytest.fixture(autouse=True)
def flat_on(monkeypatch):
    monkeypatch.setenv("PACKOS_ENC_FLAT", "1")   # read when the schema compiles
    return "flat"


@pytest.mark.parametrize("seed", range(40))
def test_flat_random_flat(seed, flat_on):
    rng = random.Random(seed)
    chain = flat_chain(rng)
    n = [1, 127, 128, 129, 300, 1000, 2049][seed % 7]
    hc = HostColumns.from_rows(chain, rows(chain, n, seed * 11 + 5))
    check(chain, hc, seed % 2, f"seed {seed}", shift=seed % 3 == 1, off64=seed % 4 == 3, kernel=flat_on)


def test_flat_wide_fixed_leaf_falls_back():
    """A fixed leaf over 16 B is outside k_encode_flat's plan: the tile
    encoder takes the chain, bit-exact."""
    chain = SChain(SInt64, SVariableString(), SStringLen(40), SBytes(17))
    hc = HostColumns.from_rows(chain, rows(chain, 700, 3))
    check(chain, hc, 0, "wide fixed", kernel=("tiles", "tiles6"))


@pytest.mark.parametrize("lens", [[0], [0, 1], [16], [4000, 0], [7000, 9000]], ids=str)
def test_flat_length_regimes(lens, flat_on):
    """All-empty values, 16-B values, multi-page values and blobs past the
    13-bit header range (status PACKOS_STATUS_OVERFLOW13)."""
    # SInt64 first: >= 15 static bytes ahead of the first var value (flat_plan)
    chain = SChain(SInt64, SInt16, SVariableString(), SInt64, SVariableBytes(), SBool)
    hc = HostColumns.from_rows(chain, rows(chain, 600, 99, lens))
    check(chain, hc, 0, f"lens {lens}", kernel=flat_on)


@pytest.mark.parametrize("flat", ["1", "0"])
@pytest.mark.parametrize("name,n", [("C3", 20000), ("C5", 5000)])
def test_flat_configs(name, n, flat, monkeypatch, flat_on):
    """The configs through k_encode_flat and (PACKOS_ENC_FLAT=0) through
    k_encode_tiles, both modes."""
    monkeypatch.setenv("PACKOS_ENC_FLAT", flat)
    cfg = CONFIGS[name]
    hc = make_columns(cfg, n=n)
    for mode in (0, 1):
        check(cfg.chain, hc, mode, f"{name} flat={flat} mode {mode}",
              kernel=flat_on if flat == "1" else ("tiles", "tiles6"))


def test_flat_capacity_overrun():
    T = torch()
    cfg = CONFIGS["C5"]
    hc = make_columns(cfg, n=3000)
    a0, o0, _ = ob.encode(cfg.chain, hc, 0, nthreads=8)
    s = CompiledSchema(cfg.chain, 0)
    dc = DeviceColumns.from_host(s, hc, "cuda:0")
    L = _lib.lib()
    n = hc.n
    for cut in (1000, int(o0[n]) // 2 + 7):
        cap = int(o0[n]) - cut
        out = T.zeros(cap, dtype=T.uint8, device="cuda:0")
        offs = T.empty(n + 1, dtype=T.int64, device="cuda:0")
        st = T.empty(n, dtype=T.int32, device="cuda:0")
        assert L.packos_encode_batch(s.handle, dc.ctypes_array(), n, out.data_ptr(), cap, offs.data_ptr(),
                                     st.data_ptr(), None, 0, 0, None) == 0
        T.cuda.synchronize()
        fits = o0[1:] <= cap
        stn = st.cpu().numpy()
        assert (stn[fits] == 0).all() and (stn[~fits] == 4).all()
        last = int(o0[int(fits.sum())])
        assert np.array_equal(out.cpu().numpy()[:last], a0[:last])
        assert np.array_equal(offs.cpu().numpy().astype(np.uint64), o0)


@pytest.mark.parametrize("name,cap_scale,flags,want", [
    # no exact capacity and >= 256 B per blob of it: both kernels launched,
    # the device picks (flat for C5's 969-B mean, tiles for C3's 85 B)
    ("C5", 1, 0, ("flat|tiles", "flat|tiles6")), ("C5", 3, 0, ("flat|tiles", "flat|tiles6")), ("C5", 1, 4, "flat"),
    ("C3", 1, 0, "tiles"), ("C3", 4, 0, ("flat|tiles", "flat|tiles6")),
    # C3 declared exact: 24 var bytes per blob, a 32-B staging pool, six
    # workgroups per CU (k_encode_tiles<true, 1, 6>)
    ("C3", 1, 4, "tiles6"),
    # C3 with a capacity of 4x its size, declared exact: the caller's word is taken
    ("C3", 4, 4, "flat")])
def test_flat_auto_dispatch(name, cap_scale, flags, want, monkeypatch):
    """PACKOS_ENC_FLAT unset: the flat / tiles choice follows the batch's mean
    blob size (static bytes + var bytes), not the arena the caller passed:
    PACKOS_ENC_CAP_EXACT (4) takes out_capacity / n on the host; without it a
    capacity of >= 256 B per blob launches both kernels and the device decides
    (no read-back)."""
    monkeypatch.delenv("PACKOS_ENC_FLAT", raising=False)
    cfg = CONFIGS[name]
    hc = make_columns(cfg, n=3000)
    check(cfg.chain, hc, 0, f"{name} x{cap_scale} flags {flags}", kernel=want, cap_scale=cap_scale, flags=flags)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("n", [1000, 3000 + 77])
def test_tiles6_pool_overflow_and_tail(mode, n, monkeypatch):
    """The six-workgroup tile encoder (exact capacity, <= 28 var bytes per
    blob on average: a 32-B staging pool) on tiles whose var bytes overflow
    the pool (their values become holes, the kernel's spilled path), mixed
    with staged tiles and a ragged last tile; bit-exact against the oracle."""
    monkeypatch.delenv("PACKOS_ENC_FLAT", raising=False)
    chain = SChain(SInt32, SVariableString(), SInt64, SStringLen(8))
    rng = random.Random(n + mode)
    rws = []
    for i in range(n):
        t = i // 128
        ln = rng.randint(0, 120) if t % 5 == 2 else rng.randint(0, 24)   # every 5th tile overflows
        rws.append([i - 500, "x" * ln, (i * 7919) - 10 ** 12, "abcdefgh"])
    hc = HostColumns.from_rows(chain, rws)
    check(chain, hc, mode, f"tiles6 n={n} mode {mode}", kernel="tiles6", flags=_lib.ENC_CAP_EXACT)


def _graph_replay(T, fn):
    """fn() captured into a HIP graph on a side stream, replayed twice."""
    s = T.cuda.Stream()
    s.wait_stream(T.cuda.current_stream())
    with T.cuda.stream(s):
        fn()   # warm-up outside the capture (schema tables, pipelines)
    T.cuda.current_stream().wait_stream(s)
    T.cuda.synchronize()
    g = T.cuda.CUDAGraph()
    with T.cuda.graph(g):
        fn()
    for _ in range(2):
        g.replay()
    T.cuda.synchronize()


@pytest.mark.parametrize("name", ["C3", "C5"])
def test_encode_plan_graph_capture_oversized_arena(name, monkeypatch):
    """EncodePlan.run() with an `out` twice the batch's size, captured in a
    graph and replayed: no host sync inside the call (a hipStreamSynchronize
    on a capturing stream would fail the capture), bytes identical to the
    oracle's."""
    monkeypatch.delenv("PACKOS_ENC_FLAT", raising=False)
    from packos_amd.api import EncodePlan
    T = torch()
    cfg = CONFIGS[name]
    hc = make_columns(cfg, n=5000)
    a0, o0, _ = ob.encode(cfg.chain, hc, cfg.mode, nthreads=8)
    s = CompiledSchema(cfg.chain, cfg.mode)
    dc = DeviceColumns.from_host(s, hc, "cuda:0")
    big = T.zeros(2 * int(o0[hc.n]) + 64, dtype=T.uint8, device="cuda:0")
    plan = EncodePlan(s, dc, out=big)
    plan.offsets.fill_(-1)
    _graph_replay(T, plan.run)
    assert np.array_equal(plan.offsets.cpu().numpy().astype(np.uint64), o0)
    assert np.array_equal(big[: int(o0[hc.n])].cpu().numpy(), a0)


@pytest.mark.parametrize("name,cap_scale", [("C3", 4), ("C5", 2)])
def test_device_pick_graph_capture(name, cap_scale, monkeypatch):
    """packos_encode_batch with neither PACKOS_ENC_CAP_EXACT nor a small
    capacity: the flat / tiles choice is made on the device (both kernels
    launched), inside a graph capture, bit-exact against the oracle."""
    monkeypatch.delenv("PACKOS_ENC_FLAT", raising=False)
    T = torch()
    cfg = CONFIGS[name]
    hc = make_columns(cfg, n=4000)
    a0, o0, s0 = ob.encode(cfg.chain, hc, 0, nthreads=8)
    s = CompiledSchema(cfg.chain, 0)
    dc = DeviceColumns.from_host(s, hc, "cuda:0")
    arr = dc.ctypes_array()
    n = hc.n
    L = _lib.lib()
    out = T.zeros(int(o0[n]) * cap_scale + 16, dtype=T.uint8, device="cuda:0")
    offs = T.full((n + 1,), -1, dtype=T.int64, device="cuda:0")
    st = T.full((n,), -1, dtype=T.int32, device="cuda:0")

    def call():
        rc = L.packos_encode_batch(s.handle, arr, n, out.data_ptr(), out.numel(), offs.data_ptr(), st.data_ptr(),
                                   None, 0, 0, T.cuda.current_stream().cuda_stream)
        assert rc == 0, L.packos_last_error()
    _graph_replay(T, call)
    assert L.packos_last_encoder().decode() in ("flat|tiles", "flat|tiles6")
    assert np.array_equal(offs.cpu().numpy().astype(np.uint64), o0)
    assert np.array_equal(out[: int(o0[n])].cpu().numpy(), a0)
    assert np.array_equal(st.cpu().numpy().astype(np.uint32), s0)
