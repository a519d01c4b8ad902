"""Random schemas and rows for parity tests (seeded, reproducible)."""
import random

from packos_amd.schema import (SBool, SBytes, SFloat32, SFloat64, SInt8, SInt16, SInt32, SInt64,
                               SMap, SMapSorted, SNullBool, SNullFloat32, SNullFloat64, SNullInt8,
                               SNullInt16, SNullInt32, SNullInt64, SString, SStringLen, SUint16,
                               SUint32, SUint64, SUint8, STuple, STupleNamed, SVariableBytes,
                               SVariableString, SChain, Schema)

SCALARS = [SBool, SInt8, SInt16, SInt32, SInt64, SFloat32, SFloat64, SUint8, SUint16, SUint32, SUint64]
NULLS = [SNullBool, SNullInt8, SNullInt16, SNullInt32, SNullInt64, SNullFloat32, SNullFloat64]


def rand_leaf(rng, allow_var=True, allow_null=True):
    r = rng.random()
    if r < 0.35:
        return rng.choice(SCALARS)
    if r < 0.5 and allow_null:
        return rng.choice(NULLS)
    if r < 0.7:
        return SStringLen(rng.randint(1, 40)) if rng.random() < 0.5 else SBytes(rng.randint(1, 40))
    if allow_var:
        return rng.choice([SString, SVariableString(), SVariableBytes()])
    return SStringLen(rng.randint(1, 8))


def rand_node(rng, depth, allow_var=True, allow_null=True):
    r = rng.random()
    if depth < 3 and r < 0.15:
        k = rng.randint(0, 4)
        kids = [rand_node(rng, depth + 1, allow_var, allow_null) for _ in range(k)]
        if rng.random() < 0.3:
            return STupleNamed([f"f{j}" for j in range(k)], *kids)
        return STuple(*kids)
    if depth < 3 and r < 0.27:
        k = rng.randint(0, 3)
        keys = rng.sample(["alpha", "beta", "gamma", "delta", "eps", "a", "b", "zz"], k)
        kids = []
        for key in keys:
            kids += [SString.Match(key), rand_node(rng, depth + 1, allow_var, allow_null)]
        return SMapSorted(*kids) if rng.random() < 0.5 else SMap(*kids)
    return rand_leaf(rng, allow_var, allow_null)


def rand_chain(seed, allow_var=True, allow_null=True, max_top=10):
    rng = random.Random(seed)
    k = rng.randint(1, max_top)
    return SChain(*[rand_node(rng, 0, allow_var, allow_null) for _ in range(k)])


def rand_value(rng, node: Schema, nil_p=0.15):
    k = node.kind
    if k in ("int", "uint"):
        if node.nullable and rng.random() < nil_p:
            return None
        return rng.getrandbits(8 * node.width)
    if k == "float":
        if node.nullable and rng.random() < nil_p:
            return None
        return rng.getrandbits(8 * node.width).to_bytes(node.width, "little")
    if k == "bool":
        if node.nullable and rng.random() < nil_p:
            return None
        return rng.random() < 0.5
    if k in ("string", "bytes"):
        n = node.width if node.width > 0 else rng.choice([0, 1, 3, 7, 16, 33, 80])
        if k == "string":
            return "".join(chr(rng.randint(0x20, 0x7E)) for _ in range(n))
        return bytes(rng.getrandbits(8) for _ in range(n))
    if k == "match":
        return None
    if k == "tuple":
        if node.nullable and rng.random() < nil_p:
            return None
        return [rand_value(rng, ch, nil_p) for ch in node.children]
    if k == "map":
        if rng.random() < nil_p:
            return None
        return [rand_value(rng, ch, nil_p) for ch in node.children]
    raise ValueError(k)


def rand_rows(chain, n, seed, nil_p=0.15):
    rng = random.Random(seed)
    return [[rand_value(rng, s, nil_p) for s in chain.Schemas] for _ in range(n)]
