"""ValidateBuffer on the GPU (packos_validate_batch / packos_validate_host_batch)
vs the CPU oracle's restatement (or_validate_batch), bit-exact status words.

schema.ValidateBuffer (schema/schema.go:880-891) runs each schema's Validate
method; in the compiled subset its rules differ from DecodeBuffer's in three
places (include/packos.h): short nullable scalars are not read (no panic),
a nullable string under Prefix / Suffix / Match passes when empty, and an odd
SMap schema count is not checked.  The mutation sweep below builds blobs that
hit all three, and every test also checks the property the reference's code
implies: a blob DecodeBuffer accepts is accepted by ValidateBuffer.
"""
import random
from dataclasses import replace

import numpy as np
import pytest

import oracle_bridge as ob
from golden_util import MODES, chain_of, load, unwrap
from packos_amd.api import CompiledSchema, Pipeline, decode_batch, validate_batch, validate_host_batch
from packos_amd.columns import HostColumns
from packos_amd.configs import CONFIGS, make_columns
from packos_amd.schema import CHK_PREFIX, CHK_SUFFIX, SChain, Schema
from schema_gen import rand_chain, rand_checked_chain, rand_checked_rows, rand_rows

pytestmark = pytest.mark.gpu
G = load()


def torch():
    import torch as t
    return t


def gpu_validate(chain, arena_np, offs_np, n, stride=0, mode=0):
    T = torch()
    s = CompiledSchema(chain, mode)
    arena = T.from_numpy(arena_np if arena_np.size else np.zeros(16, np.uint8)).to("cuda:0")
    offs = None if stride else T.from_numpy(np.asarray(offs_np).astype(np.int64)).to("cuda:0")
    st = validate_batch(s, arena, offs, n, stride=stride)
    T.cuda.synchronize()
    return st.cpu().numpy().astype(np.uint32)


def gpu_decode_status(chain, arena_np, offs_np, n, stride=0):
    T = torch()
    s = CompiledSchema(chain, 0)
    arena = T.from_numpy(arena_np if arena_np.size else np.zeros(16, np.uint8)).to("cuda:0")
    offs = None if stride else T.from_numpy(np.asarray(offs_np).astype(np.int64)).to("cuda:0")
    _, st = decode_batch(s, arena, offs, n, stride=stride)
    T.cuda.synchronize()
    return st.cpu().numpy().astype(np.uint32)


def assert_same_validate(chain, arena, offs, n, what="", stride=0, mode=0):
    o_st = ob.validate(chain, arena, offs, n, stride=stride, nthreads=8, mode=mode)
    g_st = gpu_validate(chain, arena, offs, n, stride, mode)
    if not np.array_equal(o_st, g_st):
        bad = int(np.nonzero(o_st != g_st)[0][0])
        raise AssertionError(f"{what}: validate status blob {bad}: oracle {o_st[bad]:#x} gpu {g_st[bad]:#x}")
    return g_st


def _golden_blob(case_id):
    src = next((c for c in G["encode"] if c["id"] == case_id), None)
    if src is not None:
        return bytes.fromhex(src["hex"])
    inp = next((c for c in G["inputs"] if c["id"] == case_id), None)
    if inp is not None:
        ch = chain_of(inp["schema"])
        return bytes(ob.encode(ch, HostColumns.from_rows(ch, [unwrap(inp["row"])]), MODES[inp["mode"]])[0])
    eq = next(c for c in G["equal"] if c["id"] == case_id)
    v = eq["variants"][0]
    ch = chain_of(v["schema"])
    return bytes(ob.encode(ch, HostColumns.from_rows(ch, [unwrap(eq["row"])]), MODES[v["mode"]])[0])


@pytest.mark.parametrize("case", G["validate"], ids=[c["id"] for c in G["validate"]])
def test_golden_validate(case):
    """schema_test.go's ValidateBuffer known answers (TestValidatePackedStructure
    (+_Failure), ..._DateEmailPrefixSuffix_Success(2), TestValidatePackedTuples,
    TestSDate_SuccessAndNullable) and the derived divergence cases."""
    blob = _golden_blob(case["input_from"])
    chain = chain_of(case["schema"])
    # the blob at several arena offsets (per-blob windows start unaligned)
    for pad in (0, 5, 16):
        arena = np.concatenate([np.zeros(pad, np.uint8), np.frombuffer(blob, np.uint8)])
        st = assert_same_validate(chain, arena, np.asarray([pad, pad + len(blob)], np.uint64), 1, case["id"])
        assert int(st[0]) == case["expect_status"], hex(int(st[0]))


@pytest.mark.parametrize("case", [c for c in G["decode"] if c["id"].startswith(("decode_sdate", "derived_short",
                                                                               "derived_optional", "derived_odd",
                                                                               "derived_match"))],
                         ids=lambda c: c["id"])
def test_golden_decode_side_of_divergences(case):
    """The DecodeBuffer answers paired with the validate cases, on the GPU."""
    blob = _golden_blob(case["input_from"])
    chain = chain_of(case["schema"])
    st = gpu_decode_status(chain, np.frombuffer(blob, np.uint8).copy(), np.asarray([0, len(blob)], np.uint64), 1)
    assert int(st[0]) == case["expect_status"], hex(int(st[0]))


# ------------------------------------------------------------ mutations ----
_WIDER = {("int", 1): 2, ("int", 2): 4, ("int", 4): 8, ("uint", 1): 2, ("uint", 2): 4, ("uint", 4): 8,
          ("float", 4): 8}


def mutate(node: Schema, rng: random.Random) -> Schema:
    """A schema that reads blobs written under `node` where Validate and
    Decode disagree: scalars widened and made nullable (a short payload),
    strings given a check on a nullable receiver, maps with the last schema
    dropped (odd count)."""
    k = node.kind
    if k in ("int", "uint", "float") and not node.check and (k, node.width) in _WIDER and rng.random() < 0.5:
        return replace(node, width=_WIDER[(k, node.width)], nullable=True)
    if k == "string" and node.width <= 0 and not node.check and rng.random() < 0.5:
        lit = bytes(rng.choice(b"abcxyz") for _ in range(rng.randint(1, 3)))
        r = rng.random()
        if r < 0.35:
            return replace(node, check=CHK_PREFIX, check_lit=lit)
        if r < 0.7:
            return replace(node, check=CHK_SUFFIX, check_lit=lit)
        return Schema("match", width=node.width, nullable=True, literal=lit)
    if k in ("tuple", "map"):
        kids = tuple(mutate(c, rng) for c in node.children)
        if k == "map" and len(kids) >= 2 and rng.random() < 0.4:
            kids = kids[:-1]
        return replace(node, children=kids)
    return node


def _divergence_batch(seed, n=500):
    rng = random.Random(seed * 7 + 1)
    chain = rand_chain(seed)
    hc = HostColumns.from_rows(chain, rand_rows(chain, n, seed + 3, nil_p=0.2))
    # empty strings make the nullable-empty check rule fire
    arena, offs, _ = ob.encode(chain, hc, rng.choice([0, 1]))
    mchain = SChain(*[mutate(s, rng) for s in chain.Schemas])
    return mchain, arena, offs, hc.n


@pytest.mark.parametrize("seed", range(40))
def test_validate_mutated_schemas(seed):
    mchain, arena, offs, n = _divergence_batch(seed)
    v = assert_same_validate(mchain, arena, offs, n, f"mutated seed {seed}")
    d = ob.decode(mchain, arena, offs, n, nthreads=8)[1]
    g_d = gpu_decode_status(mchain, arena, offs, n)
    assert np.array_equal(d, g_d), f"mutated seed {seed}: decode status"
    # DecodeBuffer accepting implies ValidateBuffer accepting
    assert (v[d == 0] == 0).all()


@pytest.mark.parametrize("seed", range(40))
def test_validate_corrupted(seed):
    """Flipped header bytes and truncated blobs: every error code, position
    and panic bit of ValidateBuffer matches the oracle."""
    rng = np.random.default_rng(seed + 1000)
    chain = rand_chain(seed)
    hc = HostColumns.from_rows(chain, rand_rows(chain, 400, seed + 5))
    arena, offs, _ = ob.encode(chain, hc, 0)
    arena = arena.copy()
    n = hc.n
    for i in range(n):
        a, b = int(offs[i]), int(offs[i + 1])
        r = rng.random()
        if r < 0.4 and b - a > 0:
            arena[a + int(rng.integers(0, min(b - a, 24)))] = rng.integers(0, 256)
        elif r < 0.5 and b - a > 0:
            arena[a + int(rng.integers(0, b - a))] ^= 1 << int(rng.integers(0, 8))
    cut = rng.random(n) < 0.1
    starts = offs[:-1].astype(np.int64)
    ends = offs[1:].astype(np.int64)
    ends = np.where(cut, starts + (ends - starts) // 2, ends)
    pieces, noffs = [], [0]
    for i in range(n):
        pieces.append(arena[starts[i]:ends[i]])
        noffs.append(noffs[-1] + int(ends[i] - starts[i]))
    arena2 = np.concatenate(pieces) if pieces else np.zeros(0, np.uint8)
    noffs = np.asarray(noffs, np.uint64)
    v = assert_same_validate(chain, arena2, noffs, n, f"corrupt seed {seed}")
    d = ob.decode(chain, arena2, noffs, n, nthreads=8)[1]
    assert (v[d == 0] == 0).all()


@pytest.mark.parametrize("seed", range(24))
def test_validate_checked_schemas(seed):
    """Range / SDateRange / Prefix / Suffix / default schemas, ~25 % failing
    values (the checked payloads widen the validate window)."""
    chain = rand_checked_chain(seed)
    hc = HostColumns.from_rows(chain, rand_checked_rows(chain, 700, seed + 11))
    arena, offs, _ = ob.encode(chain, hc, 0)
    assert_same_validate(chain, arena, offs, hc.n, f"checked seed {seed}")


@pytest.mark.parametrize("seed", range(12))
def test_validate_checked_fixed_stride(seed):
    chain = rand_checked_chain(seed, allow_var=False, allow_null=False)
    hc = HostColumns.from_rows(chain, rand_checked_rows(chain, 3001, seed + 13, nil_p=0.0))
    arena, offs, _ = ob.encode(chain, hc, 0)
    B = CompiledSchema(chain).fixed_blob_size
    assert_same_validate(chain, arena, offs, hc.n, f"fixed seed {seed}")
    assert_same_validate(chain, arena, None, hc.n, f"fixed stride seed {seed}", stride=B)


@pytest.mark.parametrize("name,n", [("C1", 1000), ("C2", 50_001), ("C3", 30_000), ("C4", 20_000), ("M", 50_001),
                                    ("C5", 4_000), ("X1", 64)])
def test_validate_configs(name, n):
    cfg = CONFIGS[name]
    hc = make_columns(cfg, n=n)
    arena, offs, _ = ob.encode(cfg.chain, hc, cfg.mode)
    st = assert_same_validate(cfg.chain, arena, offs, n, name, mode=cfg.mode & 0x100)
    assert (st == 0).all()


@pytest.mark.parametrize("name,n,chunk", [("C3", 20000, 3000), ("M", 10001, 0), ("C2", 30000, 7000)])
def test_validate_host_batch(name, n, chunk):
    cfg = CONFIGS[name]
    hc = make_columns(cfg, n=n)
    arena, offs, _ = ob.encode(cfg.chain, hc, cfg.mode)
    arena = arena.copy()
    # corrupt a few blobs so statuses differ
    rng = np.random.default_rng(n)
    for i in rng.choice(n, size=n // 50, replace=False):
        arena[int(offs[i]) + int(rng.integers(0, 4))] ^= 0x5A
    s = CompiledSchema(cfg.chain, cfg.mode)
    got = validate_host_batch(s, arena, offs, n, chunk_blobs=chunk)
    want = ob.validate(cfg.chain, arena, offs, n, nthreads=8)
    assert np.array_equal(got, want)
    p = Pipeline(s, chunk_blobs=4096)
    assert np.array_equal(p.validate(arena, offs, n), want)
    p.close()
