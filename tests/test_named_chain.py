"""SchemaNamedChain whose FieldNames and Schemas differ in length
(schema/schema.go:943-995) — accepted, with the reference's behaviour:

* EncodeValueNamed walks FieldNames: with FEWER names only the first
  len(FieldNames) schemas are written (the bytes of the shorter plain chain);
  with MORE names every schema's field is written and then
  chain.Schemas[len(Schemas)] is indexed — a Go panic (PACKOS_STATUS_PANIC)
  unless a field failed first (its ErrEncode);
* DecodeBufferNamed fails every blob NewSeqGetAccess accepts with
  ErrConstraintViolated at position -1 (else ErrInvalidFormat at -1);
* ValidateBuffer takes the plain SchemaChain: unchanged.

No reference test exercises the mismatch (derived cases, labelled so in
tests/golden/make_golden.py); the fewer-names encode is pinned to the
reference's two-tuple vector there (derived_named_chain_fewer_names).  CPU
tests: the oracle's restatement against those properties; GPU tests: the
library against the oracle."""
import random

import numpy as np
import pytest

import oracle_bridge as ob
from packos_amd.columns import HostColumns
from packos_amd.schema import (SBool, SchemaNamedChain, SChain, SInt16, SInt32, SInt64, SStringLen,
                               SVariableString, STuple)

PANIC = 0x40000000
ERR_ENCODE, ERR_INVALID_FORMAT, ERR_CONSTRAINT = 4, 1, 3


def leaves(rng, k):
    pool = [lambda: SInt16, lambda: SInt32, lambda: SInt64, lambda: SBool, lambda: SStringLen(3),
            lambda: SVariableString(), lambda: STuple(SInt16, SVariableString())]
    return [rng.choice(pool)() for _ in range(k)]


def value(rng, node):
    if node.kind == "tuple":
        return [value(rng, c) for c in node.children]
    if node.kind == "int":
        return rng.randint(-2 ** (8 * node.width - 1), 2 ** (8 * node.width - 1) - 1)
    if node.kind == "bool":
        return rng.random() < 0.5
    return "".join(rng.choice("abcxyz") for _ in range(node.width if node.width > 0 else rng.randint(0, 40)))


def named_case(seed, more):
    """(named chain, plain chain of the encoded fields, dict rows, list rows)."""
    rng = random.Random(seed)
    m = rng.randint(1, 6) if more else rng.randint(2, 6)
    schemas = leaves(rng, m)
    k = m + rng.randint(1, 3) if more else rng.randint(1, m - 1)
    names = [f"f{j}" for j in range(k)]
    chain = SchemaNamedChain(tuple(schemas), tuple(names))
    plain = SChain(*schemas[:min(k, m)])
    n = rng.choice([1, 7, 130, 600])
    rows = [[value(rng, s) for s in schemas] for _ in range(n)]
    drows = [{names[j]: r[j] for j in range(min(k, m))} for r in rows]
    return chain, plain, drows, [r[:min(k, m)] for r in rows]


@pytest.mark.parametrize("seed", range(12))
def test_oracle_fewer_names_encode_the_named_prefix(seed):
    chain, plain, drows, prows = named_case(seed, more=False)
    for mode in (0, 1):
        a0, o0, s0 = ob.encode(chain, HostColumns.from_rows(chain, drows), mode)
        a1, o1, s1 = ob.encode(plain, HostColumns.from_rows(plain, prows), mode)
        assert np.array_equal(a0, a1) and np.array_equal(o0, o1) and np.array_equal(s0, s1)


@pytest.mark.parametrize("seed", range(8))
def test_oracle_more_names_panic_after_fields(seed):
    chain, plain, drows, prows = named_case(seed, more=True)
    a0, o0, s0 = ob.encode(chain, HostColumns.from_rows(chain, drows), 0)
    assert (s0 == PANIC).all()
    # the fields before the panic are the plain chain's (written, then discarded)
    a1, o1, _ = ob.encode(plain, HostColumns.from_rows(plain, prows), 0)
    assert np.array_equal(a0, a1) and np.array_equal(o0, o1)


def test_oracle_more_names_field_error_comes_first():
    """A field's own encode error returns before the index panic."""
    schemas = (SInt16.Range(0, 100), SVariableString())
    chain = SchemaNamedChain(schemas, ("a", "b", "c"))
    rows = [{"a": v, "b": "x"} for v in (5, 500, -1, 100)]
    _, _, st = ob.encode(chain, HostColumns.from_rows(chain, rows), 0)
    assert st[0] == PANIC and st[3] == PANIC
    assert (st[1] & 0xFF) == ERR_ENCODE and (st[2] & 0xFF) == ERR_ENCODE and not (st[1] & PANIC)


@pytest.mark.parametrize("more", [False, True])
def test_oracle_decode_named_mismatch(more):
    chain, plain, drows, prows = named_case(3, more=more)
    arena, offs, _ = ob.encode(plain, HostColumns.from_rows(plain, prows), 0)
    n = len(prows)
    _, st = ob.decode(chain, arena, offs, n)
    assert (st[:n] == ERR_CONSTRAINT).all()
    # blobs NewSeqGetAccess rejects (< 4 bytes): ErrInvalidFormat at -1
    short = np.arange(n + 1, dtype=np.uint64) * np.uint64(3)
    _, st = ob.decode(chain, np.zeros(3 * n, np.uint8), short, n)
    assert (st[:n] == ERR_INVALID_FORMAT).all()
    # ValidateBuffer takes the plain chain: the named one validates like it
    full = SChain(*chain.Schemas)
    assert np.array_equal(ob.validate(chain, arena, offs, n), ob.validate(full, arena, offs, n))


# ------------------------------------------------------------------ GPU ----
def _gpu():
    import torch
    from packos_amd.api import CompiledSchema, DeviceColumns, decode_batch, encode_batch, validate_batch
    return torch, CompiledSchema, DeviceColumns, encode_batch, decode_batch, validate_batch


@pytest.mark.gpu
@pytest.mark.parametrize("more", [False, True])
@pytest.mark.parametrize("seed", range(10))
def test_gpu_named_mismatch_vs_oracle(seed, more):
    torch, CompiledSchema, DeviceColumns, encode_batch, decode_batch, validate_batch = _gpu()
    chain, plain, drows, prows = named_case(seed, more=more)
    hc = HostColumns.from_rows(chain, drows)
    n = hc.n
    for mode in (0, 1):
        a0, o0, s0 = ob.encode(chain, hc, mode, nthreads=8)
        s = CompiledSchema(chain, mode)
        r = encode_batch(s, DeviceColumns.from_host(s, hc, "cuda:0"))
        torch.cuda.synchronize()
        assert np.array_equal(r.status.cpu().numpy().astype(np.uint32), s0), (seed, mode)
        offs = (r.offsets.cpu().numpy().astype(np.uint64) if r.offsets is not None
                else np.arange(n + 1, dtype=np.uint64) * np.uint64(r.blob_size))
        assert np.array_equal(offs, o0)
        assert np.array_equal(r.arena[: r.total].cpu().numpy(), a0)
        # DecodeBufferNamed: every blob ErrConstraintViolated at -1 (+ ErrInvalidFormat for short blobs)
        arena = r.arena[: max(r.total, 16)]
        offs_d = torch.from_numpy(offs.astype(np.int64)).to("cuda:0")
        _, st = decode_batch(s, arena, offs_d, n)
        torch.cuda.synchronize()
        g = st[:n].cpu().numpy().astype(np.uint32)
        _, ost = ob.decode(chain, a0, o0, n, mode=mode)
        assert np.array_equal(g, ost[:n]) and (g == ERR_CONSTRAINT).all()
        short = torch.arange(n + 1, dtype=torch.int64, device="cuda:0") * 3
        _, st = decode_batch(s, torch.zeros(3 * n + 16, dtype=torch.uint8, device="cuda:0"), short, n)
        torch.cuda.synchronize()
        assert (st[:n].cpu().numpy() == ERR_INVALID_FORMAT).all()
        # ValidateBuffer: the plain chain's statuses
        vst = validate_batch(s, arena, offs_d, n)
        torch.cuda.synchronize()
        assert np.array_equal(vst[:n].cpu().numpy().astype(np.uint32), ob.validate(chain, a0, o0, n, mode=mode)[:n])
