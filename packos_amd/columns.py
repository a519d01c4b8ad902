"""Host-side column sets: the SoA batch layout the C ABI consumes.

One column per non-constant schema node in pre-order (include/packos.h):

* fixed-width leaf  -> ``data`` uint8[n*width]
* var-width leaf    -> ``data`` uint8 arena + ``offsets`` uint32[n+1]
* nullable leaf     -> + ``valid`` uint8[n]
* tuple / map       -> ``valid`` uint8[n] only (nil container)

``HostColumns.from_rows`` turns reference-shaped values (lists for tuples,
dicts for maps/named tuples, None for nil) into that layout; it is the batch
equivalent of feeding ``PutAccess.Add*`` one value at a time
(access/put.go:69-308).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass
from typing import Any, List, Optional

import numpy as np

from .schema import Schema, SchemaChain, SchemaNamedChain

__all__ = ["ColumnSpec", "HostColumns", "column_specs", "scalar_bytes"]


@dataclass
class ColumnSpec:
    node: Schema
    depth: int
    top: int
    path: str

    @property
    def kind(self) -> str:
        return self.node.kind

    @property
    def fixed(self) -> bool:
        return self.node.is_fixed_leaf

    @property
    def width(self) -> int:
        n = self.node
        if n.kind in ("int", "uint", "float", "bool"):
            return n.width
        if n.kind in ("string", "bytes") and n.width > 0:
            return n.width
        return 0

    @property
    def var(self) -> bool:
        return self.node.kind in ("string", "bytes") and self.node.width <= 0

    @property
    def has_valid(self) -> bool:
        n = self.node
        if n.kind in ("int", "uint", "float", "bool"):
            return n.nullable
        if n.kind == "tuple":
            return n.nullable
        return n.kind == "map"


def column_specs(chain: SchemaChain) -> List[ColumnSpec]:
    return [ColumnSpec(n, d, t, p) for (n, d, t, p) in chain.columns()]


def scalar_bytes(node: Schema, v) -> bytes:
    k, w = node.kind, node.width
    if k == "bool":
        return b"\x01" if v else b"\x00"
    if k in ("int", "uint"):
        if hasattr(v, "timestamp"):   # SDateRange encodes time.Time as Unix() seconds
            import math
            v = math.floor(v.timestamp())
        return (int(v) & ((1 << (8 * w)) - 1)).to_bytes(w, "little")
    if k == "float":
        if isinstance(v, (bytes, bytearray)):
            return bytes(v)
        return struct.pack("<f" if w == 4 else "<d", float(v))
    raise TypeError(k)


def _as_bytes(v) -> bytes:
    if isinstance(v, str):
        return v.encode("utf-8")
    return bytes(v)


class HostColumns:
    """numpy-backed column set for n blobs."""

    def __init__(self, chain: SchemaChain, n: int):
        self.chain = chain
        self.n = int(n)
        self.specs = column_specs(chain)
        self.data: List[Optional[np.ndarray]] = [None] * len(self.specs)
        self.offsets: List[Optional[np.ndarray]] = [None] * len(self.specs)
        self.valid: List[Optional[np.ndarray]] = [None] * len(self.specs)

    # ------------------------------------------------------------------ rows
    @classmethod
    def from_rows(cls, chain: SchemaChain, rows: List[Any]) -> "HostColumns":
        hc = cls(chain, len(rows))
        ncol = len(hc.specs)
        fixed = [bytearray() for _ in range(ncol)]
        arenas = [bytearray() for _ in range(ncol)]
        offs = [[0] for _ in range(ncol)]
        valid = [[] for _ in range(ncol)]
        # EncodeValueNamed reads field i under FieldNames[i]: a schema past the
        # names gets no value and is never encoded (schema.go:976)
        named = isinstance(chain, SchemaNamedChain) and len(chain.FieldNames) > 0
        nenc = min(len(chain.FieldNames), len(chain.Schemas)) if named else len(chain.Schemas)
        for row in rows:
            vals = row if isinstance(row, (list, tuple)) else [row]
            if isinstance(chain, SchemaNamedChain) and isinstance(row, dict):
                vals = [row.get(nm) for nm in chain.FieldNames[:len(chain.Schemas)]]
            vals = list(vals) + [None] * (len(chain.Schemas) - len(vals))
            col = [0]
            for j, (node, v) in enumerate(zip(chain.Schemas, vals)):
                hc._put(node, v, col, fixed, arenas, offs, valid, present=j < nenc)
        for c, sp in enumerate(hc.specs):
            if sp.fixed:
                hc.data[c] = np.frombuffer(bytes(fixed[c]), dtype=np.uint8).copy()
            elif sp.var:
                hc.data[c] = np.frombuffer(bytes(arenas[c]), dtype=np.uint8).copy()
                hc.offsets[c] = np.asarray(offs[c], dtype=np.uint32)
            if sp.has_valid:
                hc.valid[c] = np.asarray(valid[c], dtype=np.uint8)
        return hc

    def _put(self, node: Schema, v, col, fixed, arenas, offs, valid, present):
        if node.kind == "match":
            return
        c = col[0]
        col[0] += 1
        sp = self.specs[c]
        if node.kind in ("tuple", "map"):
            nil = (v is None) or not present
            if sp.has_valid:
                valid[c].append(0 if nil else 1)
            decl = list(node.children)
            vals = [None] * len(decl)
            if node.kind == "tuple":
                if isinstance(v, dict):
                    names = node.names or ()
                    vals = [v.get(nm) for nm in names] + [None] * (len(decl) - len(names))
                elif v is not None:
                    kv = list(v)
                    vals = [kv[j] if j < len(kv) else None for j in range(len(decl))]
            else:
                if isinstance(v, dict):
                    for j in range(0, len(decl) - 1, 2):
                        key = decl[j]
                        if key.kind != "match":
                            raise ValueError("map value dicts need constant keys")
                        vals[j + 1] = v.get(key.literal.decode("utf-8"))
                elif v is not None:
                    kv = list(v)
                    vals = [kv[j] if j < len(kv) else None for j in range(len(decl))]
            for j in node.ordered_indices():
                self._put(decl[j], vals[j], col, fixed, arenas, offs, valid, present and not nil)
            return
        if node.kind in ("string", "bytes"):
            b = _as_bytes(v) if (v is not None and present) else b""
            if node.width > 0:
                if present and len(b) != node.width:
                    raise ValueError(f"fixed width {node.width} field got {len(b)} bytes")
                fixed[c] += b.ljust(node.width, b"\x00")
            else:
                arenas[c] += b
                offs[c].append(len(arenas[c]))
            return
        # scalar
        nil = (v is None) or not present
        if sp.has_valid:
            valid[c].append(0 if nil else 1)
        fixed[c] += (b"\x00" * node.width) if nil else scalar_bytes(node, v)

    # ------------------------------------------------------------------ misc
    def nbytes_in(self) -> int:
        tot = 0
        for c, sp in enumerate(self.specs):
            if self.data[c] is not None:
                tot += int(self.data[c].nbytes)
            if self.offsets[c] is not None:
                tot += int(self.offsets[c].nbytes)
            if self.valid[c] is not None:
                tot += int(self.valid[c].nbytes)
        return tot

    def var_widths(self) -> np.ndarray:
        """[n, ncol] uint32 widths (var columns), used by shard planning."""
        w = np.zeros((self.n, len(self.specs)), dtype=np.uint32)
        for c, sp in enumerate(self.specs):
            if sp.var:
                w[:, c] = np.diff(self.offsets[c].astype(np.int64)).astype(np.uint32)
        return w
