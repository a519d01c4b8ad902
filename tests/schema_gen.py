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
            # STupleNamed(nil) for empty tuples half the time: its arg-count
            # check has no argCount > 0 guard (schema.go:1773)
            names = None if k == 0 and rng.random() < 0.5 else [f"f{j}" for j in range(k)]
            return STupleNamed(names, *kids)
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


# ---- schemas with value checks (Range / SDateRange / Prefix / Suffix / default)
def rand_checked_leaf(rng, allow_var=True, allow_null=True):
    from packos_amd.schema import SDateRange
    r = rng.random()
    if r < 0.3:
        base = rng.choice([SInt16, SInt32, SInt64])
        bits = 8 * base.width
        lo = rng.randint(-(1 << (bits - 1)), (1 << (bits - 1)) - 1)
        hi = rng.randint(lo, (1 << (bits - 1)) - 1)
        which = rng.random()
        return base.Range(lo if which < 0.7 else None, hi if which > 0.3 else None)
    if r < 0.45:
        lo = rng.randint(-60_000_000_000, 200_000_000_000)   # RFC3339 years 68 .. 8300
        return SDateRange(allow_null and rng.random() < 0.5, lo, lo + rng.randint(0, 1 << 33))
    if r < 0.75:
        s = SString if allow_var else SStringLen(rng.randint(1, 6))
        if allow_var and rng.random() < 0.4:
            s = s.DefaultDecodeValue(rng.choice(["dflt", "x", "pre-fix", "zz-suf"]))
        k = rng.random()
        if k < 0.4:
            return s.Prefix(rng.choice(["pre", "p", "pre-f"]))
        if k < 0.8:
            return s.Suffix(rng.choice(["suf", "f", "-suf"]))
        return s
    if r < 0.85 and allow_var:
        lit = rng.choice(["key", "k"])
        return SString.DefaultDecodeValue(rng.choice([lit, "other"])).Match(lit)
    return rand_leaf(rng, allow_var, allow_null)


def rand_checked_node(rng, depth, allow_var=True, allow_null=True):
    r = rng.random()
    if depth < 2 and r < 0.15:
        kids = [rand_checked_node(rng, depth + 1, allow_var, allow_null) for _ in range(rng.randint(1, 3))]
        r2 = rng.random()
        if r2 < 0.1:
            # FieldNames shorter than Schemas: Encode of a present value and every
            # Decode fail with ErrConstraintViolated (schema.go:1756-1758, 1808-1810)
            return STupleNamed([f"f{j}" for j in range(len(kids) - 1)], *kids)
        if r2 < 0.3:
            return STupleNamed([f"f{j}" for j in range(len(kids))], *kids)
        return STuple(*kids)
    if depth < 2 and r < 0.25:
        keys = rng.sample(["alpha", "beta", "gamma", "zz"], rng.randint(1, 2))
        kids = []
        for key in keys:
            kids += [SString.Match(key), rand_checked_node(rng, depth + 1, allow_var, allow_null)]
        return SMapSorted(*kids)
    return rand_checked_leaf(rng, allow_var, allow_null)


def rand_checked_chain(seed, allow_var=True, allow_null=True, max_top=8):
    rng = random.Random(seed)
    return SChain(*[rand_checked_node(rng, 0, allow_var, allow_null) for _ in range(rng.randint(1, max_top))])


def _checked_value(rng, node, nil_p):
    """Values that mostly pass the node's check and sometimes fail it."""
    from packos_amd.schema import CHK_MAX, CHK_MIN, CHK_PREFIX, CHK_SUFFIX
    if node.kind == "int" and node.check & (CHK_MIN | CHK_MAX):
        if node.nullable and rng.random() < nil_p:
            return None
        bits = 8 * node.width
        lo = node.rmin if node.check & CHK_MIN else -(1 << (bits - 1))
        hi = node.rmax if node.check & CHK_MAX else (1 << (bits - 1)) - 1
        r = rng.random()
        if r < 0.9:
            return rng.randint(lo, hi)
        if r < 0.95 and lo > -(1 << (bits - 1)):
            return lo - 1
        if hi < (1 << (bits - 1)) - 1:
            return hi + 1
        return rng.randint(lo, hi)
    if node.kind == "string" and node.check & (CHK_PREFIX | CHK_SUFFIX):
        lit = node.check_lit.decode()
        w = node.width
        if rng.random() < 0.1:
            n = w if w > 0 else rng.choice([0, 1, 5])
            return "".join(rng.choice("abcpf-") for _ in range(n))
        if w > 0:
            if len(lit) > w:
                return "q" * w
            body = "".join(rng.choice("abcxyz") for _ in range(w - len(lit)))
        else:
            body = "".join(rng.choice("abcxyz") for _ in range(rng.choice([0, 2, 9])))
        return lit + body if node.check & CHK_PREFIX else body + lit
    if node.kind == "string" and node.width <= 0 and rng.random() < 0.3:
        return ""   # empty payload: decodes as the default when there is one
    if node.kind in ("tuple", "map"):
        if (node.kind == "map" or node.nullable) and rng.random() < nil_p:
            return None
        return [_checked_value(rng, ch, nil_p) for ch in node.children]
    return rand_value(rng, node, nil_p)


def rand_checked_rows(chain, n, seed, nil_p=0.15):
    rng = random.Random(seed)
    return [[_checked_value(rng, s, nil_p) for s in chain.Schemas] for _ in range(n)]
