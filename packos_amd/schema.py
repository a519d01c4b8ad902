"""Schema constructors mirroring the reference ``schema`` package surface.

The names follow quickwritereader/PackOS ``schema/schema.go`` so code written
against the reference reads the same here:

* ``SBool``, ``SInt8`` .. ``SInt64``, ``SFloat32``/``SFloat64`` and their
  ``SNull*`` variants — schema/schema.go:835-854
* ``SString`` (Width 0, nullable), ``SStringLen(n)`` (:1066), ``SVariableString()``
  (:872), ``SString.Match(s)`` / ``SStringExact(s)`` (:1062,1137)
* ``SBytes(n)`` / ``SVariableBytes()`` — :856, :876
* ``SMap(*schemas)`` — :858 (key, value, key, value ...)
* ``STuple``, ``STupleVal``, ``STupleNamed``, ``STupleNamedVal`` — :1551-1699
* ``SChain`` / ``SchemaNamedChain`` — :1054-1059, :943-946
* value checks: ``SInt16/32/64.Range(min, max)`` / ``.RangeValues`` (:1172-1364),
  ``SDateRange(nullable, from, to)`` (:2188-2250), ``SString.Prefix`` /
  ``.Suffix`` (:1144-1158), ``SString.DefaultDecodeValue`` (:1131)
* ``BuildSchema(json)`` — schema/schemabuilder_json.go:124

Extensions needed by the PutAccess / packable mirrors (no reference schema
constructor exists for them): ``SUint8`` .. ``SUint64`` (``AddUint*``,
access/put.go:99-118) and ``SMapSorted`` (``PackMapSorted`` /
``AddMapSortedKey*`` key order, resolved once at compile time instead of a
``utils.SortKeys`` per blob, utils/utils.go:7-14).

A schema object is pure host-side data; ``to_json()`` emits the SchemaJSON
vocabulary the C ABI's ``packos_schema_compile`` accepts.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field, replace
from typing import Any, List, Optional, Sequence

__all__ = [
    "Schema", "SchemaChain", "SchemaNamedChain", "SChain",
    "SBool", "SInt8", "SInt16", "SInt32", "SInt64", "SFloat32", "SFloat64",
    "SUint8", "SUint16", "SUint32", "SUint64",
    "SNullBool", "SNullInt8", "SNullInt16", "SNullInt32", "SNullInt64",
    "SNullFloat32", "SNullFloat64", "SNullUint8", "SNullUint16", "SNullUint32", "SNullUint64",
    "SString", "SStringLen", "SStringExact", "SVariableString", "SBytes", "SVariableBytes",
    "SMap", "SMapSorted", "SVariableMap", "STuple", "STupleVal", "STupleNamed", "STupleNamedVal",
    "STupleValFlatten", "STupleNamedValFlattened",
    "SDateRange", "BuildSchema", "TAG_OF_KIND",
    "CHK_MIN", "CHK_MAX", "CHK_DATE", "CHK_PREFIX", "CHK_SUFFIX", "CHK_DEFAULT",
]

# value-check bits (packos_amd/csrc/program.h CHK_*)
CHK_MIN, CHK_MAX, CHK_DATE, CHK_PREFIX, CHK_SUFFIX, CHK_DEFAULT = 1, 2, 4, 8, 16, 32
_GO_ZERO_TIME_UNIX = -62135596800   # time.Time{}.Unix()


def _unix(t) -> int:
    """time.Time.Unix() of a datetime (floor), or an int passed through."""
    if t is None:
        return None
    if isinstance(t, int):
        return t
    import math
    return int(math.floor(t.timestamp()))


def _rfc3339(sec: int) -> str:
    import datetime as _dt
    d = _dt.datetime(1970, 1, 1, tzinfo=_dt.timezone.utc) + _dt.timedelta(seconds=int(sec))
    return f"{d.year:04d}-{d.month:02d}-{d.day:02d}T{d.hour:02d}:{d.minute:02d}:{d.second:02d}Z"


def _parse_rfc3339(txt: str) -> int:
    """time.Parse(time.RFC3339, txt).Unix(); a parse error gives the zero
    Time, as BuildSchema discards it (schemabuilder_json.go:169-170)."""
    import datetime as _dt
    import re
    m = re.fullmatch(r"(\d{4})-(\d{2})-(\d{2})T(\d{2}):(\d{2}):(\d{2})(\.\d+)?(Z|[+-]\d{2}:\d{2})", txt or "")
    if not m:
        return _GO_ZERO_TIME_UNIX
    Y, Mo, D, h, mi, sec = (int(m.group(k)) for k in range(1, 7))
    try:
        d = _dt.datetime(Y, Mo, D, h, mi, sec, tzinfo=_dt.timezone.utc)
    except ValueError:
        return _GO_ZERO_TIME_UNIX
    tz = m.group(8)
    off = 0
    if tz != "Z":
        th, tm = int(tz[1:3]), int(tz[4:6])
        if th > 23 or tm > 59:
            return _GO_ZERO_TIME_UNIX
        off = (th * 3600 + tm * 60) * (-1 if tz[0] == "-" else 1)
    epoch = _dt.datetime(1970, 1, 1, tzinfo=_dt.timezone.utc)
    return int((d - epoch).total_seconds()) - off

# tag written in the header for each node kind (typetags/types.go:6-20)
TAG_OF_KIND = {
    "int": 1, "uint": 1, "float": 3, "bool": 5, "string": 6, "bytes": 6, "match": 6,
    "tuple": 4, "map": 7,
}


@dataclass(frozen=True)
class Schema:
    """One schema node.

    kind      : int | uint | float | bool | string | bytes | match | tuple | map
    width     : scalar byte width; SchemaString/SchemaBytes ``Width`` for
                string/bytes (>0 exact, <=0 nullable/variable)
    nullable  : scalar ``Nullable`` / TupleSchema ``Nullable``
    literal   : constant bytes of a ``match`` node (map key / SString.Match)
    children  : nested schemas (tuple fields or map key,value pairs)
    names     : TupleSchemaNamed ``FieldNames``
    variable  : TupleSchema ``VariableLength``
    sorted    : map pairs ordered by key bytes (PackMapSorted)
    check     : CHK_* value checks (Range / SDateRange / Prefix / Suffix /
                DefaultDecodeValue); rmin / rmax the int bounds, check_lit the
                prefix or suffix, default the DefaultDecodeVal
    """

    kind: str
    width: int = 0
    nullable: bool = False
    literal: bytes = b""
    children: tuple = ()
    names: Optional[tuple] = None
    variable: bool = False
    sorted: bool = False
    check: int = 0
    rmin: int = 0
    rmax: int = 0
    check_lit: bytes = b""
    default: bytes = b""
    flatten: bool = False   # STupleValFlatten / STupleNamedValFlattened (only SRepeatSchema children differ)

    # -- value checks (schema/schema.go:1131-1364, 2188-2250) ------------------
    def Range(self, min=None, max=None) -> "Schema":
        """SInt16/32/64.Range(min, max): a SchemaGeneric whose precheck is
        never nullable; out-of-range values fail with ErrOutOfRange on decode
        and encode (schema.go:1175-1364)."""
        if self.kind != "int" or self.width not in (2, 4, 8):
            raise TypeError("Range is defined on SInt16 / SInt32 / SInt64")
        chk = (CHK_MIN if min is not None else 0) | (CHK_MAX if max is not None else 0)
        return replace(self, nullable=False, check=chk, rmin=int(min or 0), rmax=int(max or 0))

    def RangeValues(self, min: int, max: int) -> "Schema":
        return self.Range(min, max)

    def _str_check(self, bit: int, lit) -> "Schema":
        if self.kind != "string":
            raise TypeError("Prefix / Suffix are defined on SchemaString")
        lb = lit.encode() if isinstance(lit, str) else bytes(lit)
        return replace(self, check=(self.check & CHK_DEFAULT) | bit, check_lit=lb)

    def Prefix(self, prefix) -> "Schema":
        """SString.Prefix: strings.HasPrefix, ErrStringPrefix (schema.go:1144-1150)."""
        return self._str_check(CHK_PREFIX, prefix)

    def Suffix(self, suffix) -> "Schema":
        """SString.Suffix: strings.HasSuffix, ErrStringSuffix (schema.go:1152-1158)."""
        return self._str_check(CHK_SUFFIX, suffix)

    def DefaultDecodeValue(self, value) -> "Schema":
        """SchemaString.DefaultDecodeValue: an empty payload decodes as `value`
        (schema.go:1131-1134, 283-285)."""
        if self.kind not in ("string", "match"):
            raise TypeError("DefaultDecodeValue is defined on SchemaString")
        vb = value.encode() if isinstance(value, str) else bytes(value)
        chk = (self.check | CHK_DEFAULT) if vb else (self.check & ~CHK_DEFAULT)
        return replace(self, check=chk, default=vb)

    # -- SchemaString helpers (schema/schema.go:1062-1171) ---------------------
    def Match(self, expected) -> "Schema":
        if self.kind != "string":
            raise TypeError("Match is defined on SchemaString")
        lit = expected.encode() if isinstance(expected, str) else bytes(expected)
        # CheckFunc keeps the receiver's Width (precheck hint) and its
        # DefaultDecodeVal (schema.go:1070-1130)
        return Schema("match", width=self.width, nullable=self.width <= 0, literal=lit,
                      check=self.check & CHK_DEFAULT, default=self.default)

    def WithWidth(self, n: int) -> "Schema":
        if self.kind != "string":
            raise TypeError("WithWidth is defined on SchemaString")
        return replace(self, width=int(n), nullable=int(n) <= 0)

    def Optional(self) -> "Schema":
        if self.kind != "string":
            raise TypeError("Optional is defined on SchemaString")
        return replace(self, width=-1, nullable=True)

    def IsNullable(self) -> bool:
        if self.kind in ("string", "bytes"):
            return self.width <= 0
        if self.kind == "map":
            return True
        if self.kind == "match":
            return True
        return self.nullable

    @property
    def is_container(self) -> bool:
        return self.kind in ("tuple", "map")

    @property
    def is_fixed_leaf(self) -> bool:
        return self.kind in ("int", "uint", "float", "bool") or (
            self.kind in ("string", "bytes") and self.width > 0)

    @property
    def tag(self) -> int:
        return TAG_OF_KIND[self.kind]

    def ordered_indices(self) -> List[int]:
        """Declaration indices of the children in emission order (sorted maps:
        key/value pairs by key bytes, utils.SortKeys = sort.Strings)."""
        idx = list(range(len(self.children)))
        if self.kind == "map" and self.sorted:
            ch = self.children
            np_ = len(ch) // 2
            if any(ch[2 * j].kind != "match" for j in range(np_)):
                raise ValueError("sorted map needs constant (exact) keys")
            order = sorted(range(np_), key=lambda j: ch[2 * j].literal)
            idx = [x for j in order for x in (2 * j, 2 * j + 1)] + idx[np_ * 2:]
        return idx

    def ordered_children(self) -> List["Schema"]:
        """Children in emission order."""
        return [self.children[i] for i in self.ordered_indices()]

    # -- SchemaJSON emission (schema/schemabuilder_json.go:8-30) --------------
    def to_json(self) -> dict:
        k = self.kind
        if k == "int" and self.check & CHK_DATE:
            d = {"type": "date"}
            if self.nullable:
                d["nullable"] = True
            rng = self.check & (CHK_MIN | CHK_MAX)
            if rng == (CHK_MIN | CHK_MAX):
                d["dateFrom"], d["dateTo"] = _rfc3339(self.rmin), _rfc3339(self.rmax)
            elif rng:
                raise ValueError("SchemaJSON 'date' takes both dateFrom and dateTo or neither")
            return d
        if k in ("int", "uint", "float"):
            d = {"type": f"{k}{self.width * 8}"}
            if self.nullable:
                d["nullable"] = True
            if self.check & CHK_MIN:
                d["min"] = self.rmin
            if self.check & CHK_MAX:
                d["max"] = self.rmax
            return d
        if k == "bool":
            return {"type": "bool", "nullable": True} if self.nullable else {"type": "bool"}
        if k in ("string", "match"):
            d = {"type": "string"}
            if self.width > 0:
                d["width"] = self.width
            elif self.width < 0:
                d["nullable"] = True
            if self.check & CHK_DEFAULT:
                d["decodeDefault"] = self.default.decode("utf-8")
            if k == "match":
                d["exact"] = self.literal.decode("utf-8")
            elif self.check & CHK_PREFIX:
                d["prefix"] = self.check_lit.decode("utf-8")
            elif self.check & CHK_SUFFIX:
                d["suffix"] = self.check_lit.decode("utf-8")
            return d
        if k == "bytes":
            return {"type": "bytes", "width": self.width} if self.width > 0 else {"type": "bytes"}
        if k == "tuple":
            d = {"type": "tuple", "schema": [c.to_json() for c in self.children]}
            if self.names:
                d["fieldNames"] = list(self.names)
            elif self.names is not None:
                # STupleNamed(nil, ...): BuildSchema routes an empty fieldNames to
                # STuple (schemabuilder_json.go:245), so the reference JSON cannot
                # say "named"; this build's compiler reads the extra key
                d["named"] = True
            if self.variable:
                d["variableLength"] = True
            if self.flatten:
                d["flatten"] = True
            return d
        if k == "map":
            d = {"type": "map", "schema": [c.to_json() for c in self.children]}
            if self.sorted:
                d["sorted"] = True
            return d
        raise ValueError(k)


def SDateRange(nullable: bool, from_=None, to=None) -> "Schema":
    """SDateRange(nullable, from, to): an int64 Unix-seconds payload checked
    against [from, to] (datetimes or ints; None = unbounded), failing with
    ErrDateOutOfRange (schema/schema.go:2188-2250)."""
    lo, hi = _unix(from_), _unix(to)
    chk = CHK_DATE | (CHK_MIN if lo is not None else 0) | (CHK_MAX if hi is not None else 0)
    return Schema("int", width=8, nullable=bool(nullable), check=chk, rmin=lo or 0, rmax=hi or 0)


def _scalar(kind, width, nullable=False):
    return Schema(kind, width=width, nullable=nullable)


SBool = _scalar("bool", 1)
SInt8 = _scalar("int", 1)
SInt16 = _scalar("int", 2)
SInt32 = _scalar("int", 4)
SInt64 = _scalar("int", 8)
SUint8 = _scalar("uint", 1)
SUint16 = _scalar("uint", 2)
SUint32 = _scalar("uint", 4)
SUint64 = _scalar("uint", 8)
SFloat32 = _scalar("float", 4)
SFloat64 = _scalar("float", 8)
SNullBool = _scalar("bool", 1, True)
SNullInt8 = _scalar("int", 1, True)
SNullInt16 = _scalar("int", 2, True)
SNullInt32 = _scalar("int", 4, True)
SNullInt64 = _scalar("int", 8, True)
SNullUint8 = _scalar("uint", 1, True)
SNullUint16 = _scalar("uint", 2, True)
SNullUint32 = _scalar("uint", 4, True)
SNullUint64 = _scalar("uint", 8, True)
SNullFloat32 = _scalar("float", 4, True)
SNullFloat64 = _scalar("float", 8, True)
# SString: SchemaString{Width: 0} — nullable, any width (schema/schema.go:853)
SString = Schema("string", width=0, nullable=True)


def SStringLen(width: int) -> Schema:
    return SString.WithWidth(width)


def SStringExact(expected) -> Schema:
    return SString.Match(expected)


def SVariableString() -> Schema:
    return Schema("string", width=-1, nullable=True)


def SBytes(width: int) -> Schema:
    return Schema("bytes", width=int(width), nullable=int(width) <= 0)


def SVariableBytes() -> Schema:
    return Schema("bytes", width=-1, nullable=True)


def SMap(*schemas: Schema) -> Schema:
    return Schema("map", width=-1, nullable=True, children=tuple(schemas))


SVariableMap = SMap


def SMapSorted(*schemas: Schema) -> Schema:
    return Schema("map", width=-1, nullable=True, children=tuple(schemas), sorted=True)


def STuple(*schemas: Schema) -> Schema:
    return Schema("tuple", nullable=True, children=tuple(schemas))


def STupleVal(*schemas: Schema) -> Schema:
    return Schema("tuple", nullable=True, children=tuple(schemas), variable=True)


def STupleValFlatten(*schemas: Schema) -> Schema:
    """STupleValFlatten (schema/schema.go:1559-1561).  Flatten changes only how
    SRepeatSchema children encode / decode (:1616-1623, :1649-1664), and repeat
    is outside the compiled subset, so the bytes are STupleVal's."""
    return Schema("tuple", nullable=True, children=tuple(schemas), variable=True, flatten=True)


def STupleNamedValFlattened(names: Sequence[str], *schemas: Schema) -> Schema:
    """STupleNamedValFlattened (schema/schema.go:1711-1719); see STupleValFlatten."""
    return Schema("tuple", nullable=True, children=tuple(schemas), names=tuple(names), variable=True,
                  flatten=True)


def STupleNamed(names: Optional[Sequence[str]], *schemas: Schema) -> Schema:
    return Schema("tuple", nullable=True, children=tuple(schemas),
                  names=tuple(names) if names is not None else tuple())


def STupleNamedVal(names: Sequence[str], *schemas: Schema) -> Schema:
    return Schema("tuple", nullable=True, children=tuple(schemas), names=tuple(names),
                  variable=True)


@dataclass(frozen=True)
class SchemaChain:
    """schema.SchemaChain (schema/schema.go:1054-1059)."""

    Schemas: tuple = field(default_factory=tuple)

    def to_json(self) -> Any:
        return [s.to_json() for s in self.Schemas]

    def json(self) -> str:
        return json.dumps(self.to_json())

    def walk(self):
        """Pre-order (node, depth, top_index, path) over the whole chain."""
        out = []

        def rec(node, depth, top, path):
            out.append((node, depth, top, path))
            names = node.names if node.kind == "tuple" else None
            for j in node.ordered_indices():
                ch = node.children[j]
                nm = names[j] if names and j < len(names) else ""
                rec(ch, depth + 1, top, f"{path}.{nm}" if nm and path else (nm or path))

        names = getattr(self, "FieldNames", None)
        for t, s in enumerate(self.Schemas):
            rec(s, 0, t, names[t] if names and t < len(names) else "")
        return out

    def columns(self):
        """Column nodes: every non-constant node in pre-order."""
        return [w for w in self.walk() if w[0].kind != "match"]


@dataclass(frozen=True)
class SchemaNamedChain(SchemaChain):
    """schema.SchemaNamedChain (schema/schema.go:943-946)."""

    FieldNames: tuple = field(default_factory=tuple)

    def to_json(self) -> Any:
        return {"type": "chain", "schema": [s.to_json() for s in self.Schemas],
                "fieldNames": list(self.FieldNames)}


def SChain(*schemas: Schema) -> SchemaChain:
    return SchemaChain(tuple(schemas))


# -- BuildSchema (schema/schemabuilder_json.go:124-300), in-scope subset ------
_INT_W = {"int8": 1, "int16": 2, "int32": 4, "int64": 8}
_UINT_W = {"uint8": 1, "uint16": 2, "uint32": 4, "uint64": 8}


def BuildSchema(js) -> Schema:
    if js is None:
        raise ValueError("nil schema")
    if isinstance(js, str):
        js = json.loads(js)
    t = js.get("type")
    nul = bool(js.get("nullable", False))
    if t == "bool":
        return SNullBool if nul else SBool
    if t in _INT_W:
        node = _scalar("int", _INT_W[t], nul)
        lo, hi = js.get("min"), js.get("max")
        if _INT_W[t] > 1 and (lo is not None or hi is not None):   # int8 ignores them
            return node.Range(lo, hi)
        return node
    if t == "date":
        if js.get("dateFrom") and js.get("dateTo"):
            return SDateRange(nul, _parse_rfc3339(js["dateFrom"]), _parse_rfc3339(js["dateTo"]))
        return SDateRange(nul)
    if t in _UINT_W:
        return _scalar("uint", _UINT_W[t], nul)
    if t in ("float32", "float64"):
        return _scalar("float", 4 if t == "float32" else 8, nul)
    if t == "string":
        s = SString
        if nul:
            s = s.Optional()
        elif int(js.get("width", 0)) > 0:
            s = s.WithWidth(int(js["width"]))
        if js.get("decodeDefault"):
            s = s.DefaultDecodeValue(js["decodeDefault"])
        if js.get("exact"):
            return s.Match(js["exact"])
        if js.get("prefix"):
            return s.Prefix(js["prefix"])
        if js.get("suffix"):
            return s.Suffix(js["suffix"])
        if js.get("pattern"):
            raise NotImplementedError("string pattern (regexp) is outside the compiled subset")
        return s
    if t == "bytes":
        w = int(js.get("width", 0))
        return SBytes(w) if w > 0 else SVariableBytes()
    if t == "tuple":
        kids = [BuildSchema(c) for c in js.get("schema", [])]
        names = js.get("fieldNames")
        var = bool(js.get("variableLength", False))
        # "flatten" counts only with variableLength (schemabuilder_json.go:247-258):
        # STupleValFlatten / STupleNamedValFlattened, byte-identical to the
        # non-flattened forms without SRepeatSchema children (rejected here)
        flat = var and bool(js.get("flatten", False))
        # every STuple* is Nullable: true; BuildSchema never reads the key
        node = Schema("tuple", nullable=True, children=tuple(kids),
                      names=tuple(names) if names else (() if js.get("named") else None),
                      variable=var, flatten=flat)
        return node
    if t == "map":
        kids = [BuildSchema(c) for c in js.get("schema", [])]
        return Schema("map", width=-1, nullable=True, children=tuple(kids),
                      sorted=bool(js.get("sorted", False)))
    raise NotImplementedError(f"schema type {t!r} is outside the compiled subset")


def BuildChain(js) -> SchemaChain:
    """A JSON array (SChain) or {"type":"chain",...} (SchemaNamedChain)."""
    if isinstance(js, str):
        js = json.loads(js)
    if isinstance(js, list):
        return SChain(*[BuildSchema(x) for x in js])
    if js.get("type") == "chain":
        kids = tuple(BuildSchema(x) for x in js.get("schema", []))
        names = js.get("fieldNames")
        if names:
            return SchemaNamedChain(kids, tuple(names))
        return SchemaChain(kids)
    return SChain(BuildSchema(js))
