"""ctypes bridge to the CPU ORACLE (oracle/liboracle.so) — test infrastructure.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this
module; the product path (packos_amd) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import List, Optional

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# PACKOS_ORACLE_LIB: the sanitizer build of tools/asan_cpu.sh (test runs only)
ORACLE_SO = os.environ.get("PACKOS_ORACLE_LIB") or os.path.join(ROOT, "oracle", "liboracle.so")

MODE_PUTACCESS = 0
MODE_PACKABLE = 1
MODE_EXTENDED = 0x100


class PackosColumn(C.Structure):
    _fields_ = [("data", C.c_void_p), ("offsets", C.c_void_p), ("valid", C.c_void_p),
                ("start", C.c_void_p), ("length", C.c_void_p), ("offsets64", C.c_void_p)]


class OrSchema(C.Structure):
    _fields_ = [("nodes", C.c_void_p), ("n_nodes", C.c_int), ("n_top", C.c_int),
                ("lit", C.c_void_p), ("lit_off", C.c_void_p), ("n_cols", C.c_int),
                ("col_of_node", C.c_int32 * 512), ("next_sibling", C.c_int32 * 512),
                ("top_nodes", C.c_int32 * 256), ("ext", C.c_void_p), ("chain_names", C.c_int)]


class OrGet(C.Structure):
    _fields_ = [("buf", C.c_void_p), ("len", C.c_int64), ("arg_count", C.c_int64),
                ("base", C.c_int64), ("xw", C.c_int), ("xmode", C.c_int)]


class OrSeq(C.Structure):
    _fields_ = [("buf", C.c_void_p), ("len", C.c_int64), ("count", C.c_int64), ("base", C.c_int64),
                ("pos", C.c_int64), ("next_off", C.c_int64), ("next_type", C.c_int),
                ("cur_off", C.c_int64), ("cur_type", C.c_int), ("xw", C.c_int)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "-s"])
        L = C.CDLL(ORACLE_SO)
        L.or_schema_prepare.argtypes = [C.POINTER(OrSchema)]
        L.or_encode_batch.argtypes = [C.POINTER(OrSchema), C.POINTER(PackosColumn), C.c_size_t,
                                      C.c_int, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p,
                                      C.c_int]
        L.or_encode_batch.restype = C.c_int64
        L.or_encoded_size_one.argtypes = [C.POINTER(OrSchema), C.POINTER(PackosColumn),
                                          C.c_size_t, C.c_int]
        L.or_encoded_size_one.restype = C.c_int64
        L.or_encoded_total.argtypes = [C.POINTER(OrSchema), C.POINTER(PackosColumn), C.c_size_t, C.c_int,
                                       C.c_void_p, C.c_int]
        L.or_encoded_total.restype = C.c_int64
        L.or_decode_batch.argtypes = [C.POINTER(OrSchema), C.c_void_p, C.c_void_p, C.c_uint64,
                                      C.c_size_t, C.POINTER(PackosColumn), C.c_void_p, C.c_int]
        L.or_decode_batch_mode.argtypes = [C.POINTER(OrSchema), C.c_void_p, C.c_void_p, C.c_uint64,
                                           C.c_size_t, C.POINTER(PackosColumn), C.c_void_p, C.c_int, C.c_int]
        L.or_validate_batch.argtypes = [C.POINTER(OrSchema), C.c_void_p, C.c_void_p, C.c_uint64,
                                        C.c_size_t, C.c_void_p, C.c_int, C.c_int]
        L.or_seq_init_ext.argtypes = [C.POINTER(OrSeq), C.c_void_p, C.c_int64, C.c_int]
        L.or_get_init.argtypes = [C.POINTER(OrGet), C.c_void_p, C.c_int64]
        L.or_get_fixed.argtypes = [C.POINTER(OrGet), C.c_int64, C.c_int, C.c_int,
                                   C.POINTER(C.c_int64)]
        L.or_get_nullable.argtypes = L.or_get_fixed.argtypes
        L.or_get_span.argtypes = [C.POINTER(OrGet), C.c_int64, C.POINTER(C.c_int64),
                                  C.POINTER(C.c_int64)]
        L.or_get_nested.argtypes = [C.POINTER(OrGet), C.c_int64, C.POINTER(OrGet),
                                    C.POINTER(C.c_int)]
        L.or_get_range.argtypes = [C.POINTER(OrGet), C.c_int64, C.POINTER(C.c_int),
                                   C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
        L.or_get_range.restype = None
        L.or_seq_init.argtypes = [C.POINTER(OrSeq), C.c_void_p, C.c_int64]
        L.or_seq_peek.argtypes = [C.POINTER(OrSeq), C.POINTER(C.c_int), C.POINTER(C.c_int64)]
        L.or_seq_advance.argtypes = [C.POINTER(OrSeq)]
        L.or_seq_next.argtypes = [C.POINTER(OrSeq), C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                  C.POINTER(C.c_int)]
        L.or_seq_peek_nested.argtypes = [C.POINTER(OrSeq), C.POINTER(OrSeq)]
        L.or_get_field_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_size_t,
                                         C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                         C.c_void_p, C.c_void_p, C.c_void_p]
        L.or_get_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_size_t, C.c_void_p,
                                   C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_uint32,
                                   C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.or_get_map_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_size_t, C.c_void_p, C.c_int,
                                       C.c_int, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_void_p, C.c_void_p, C.c_void_p]
        _lib = L
    return _lib


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data


class OracleSchema:
    """or_schema built from a packos_amd.schema chain (declaration order;
    the oracle sorts map pairs itself)."""

    def __init__(self, chain):
        nodes: List[int] = []
        lits: List[bytes] = []
        ext: List[int] = []

        def rec(n):
            k = n.kind
            li = di = 0
            if n.check & 0x18:      # prefix / suffix literal
                li = len(lits) + 1
                lits.append(n.check_lit)
            if n.check & 0x20:      # decodeDefault literal
                di = len(lits) + 1
                lits.append(n.default)
            ext.extend([n.check, n.rmin, n.rmax, li | (di << 32)])
            if k == "int":
                nodes.extend([1, n.width, int(n.nullable), 0])
            elif k == "uint":
                nodes.extend([2, n.width, int(n.nullable), 0])
            elif k == "float":
                nodes.extend([3, n.width, int(n.nullable), 0])
            elif k == "bool":
                nodes.extend([4, 1, int(n.nullable), 0])
            elif k == "string":
                nodes.extend([5, n.width, 0, 0])
            elif k == "bytes":
                nodes.extend([6, n.width, 0, 0])
            elif k == "match":
                nodes.extend([7, len(lits), n.width, 0])
                lits.append(n.literal)
            elif k == "tuple":
                named = n.names is not None
                bad = named and len(n.names) != len(n.children)
                nodes.extend([8, int(n.nullable), len(n.children), int(n.variable) | 2 * named | 4 * bad])
            elif k == "map":
                nodes.extend([9, int(n.sorted), len(n.children), 0])
            else:
                raise ValueError(k)
            for ch in n.children:
                rec(ch)

        for s in chain.Schemas:
            rec(s)
        self.nodes = np.asarray(nodes, dtype=np.int32)
        pool = b"".join(lits)
        self.lit = np.frombuffer(pool + b"\x00", dtype=np.uint8).copy()
        offs = [0]
        for l in lits:
            offs.append(offs[-1] + len(l))
        self.lit_off = np.asarray(offs, dtype=np.int32)
        self.ext = np.asarray(ext, dtype=np.int64)
        s = OrSchema()
        s.ext = _ptr(self.ext) if any(ext) else None
        s.nodes = _ptr(self.nodes)
        s.n_nodes = len(nodes) // 4
        s.n_top = len(chain.Schemas)
        s.lit = _ptr(self.lit)
        s.lit_off = _ptr(self.lit_off)
        names = getattr(chain, "FieldNames", None)   # SchemaNamedChain
        s.chain_names = len(names) if names and len(names) != len(chain.Schemas) else 0
        if lib().or_schema_prepare(C.byref(s)) != 0:
            raise ValueError("oracle rejected schema")
        self.s = s
        self.n_cols = s.n_cols


def make_cols(hc, keep):
    arr = (PackosColumn * max(1, len(hc.specs)))()
    for c in range(len(hc.specs)):
        for a in (hc.data[c], hc.offsets[c], hc.valid[c]):
            if a is not None:
                keep.append(a)
        arr[c].data = _ptr(hc.data[c])
        if hc.data[c] is not None and hc.data[c].size == 0:
            z = np.zeros(16, np.uint8)
            keep.append(z)
            arr[c].data = _ptr(z)
        arr[c].offsets = _ptr(hc.offsets[c])
        arr[c].valid = _ptr(hc.valid[c])
    return arr


def encode(chain, hc, mode=MODE_PUTACCESS, nthreads=1):
    """Oracle encode of a HostColumns batch -> (arena, offsets[n+1], status)."""
    os_ = OracleSchema(chain)
    keep = []
    cols = make_cols(hc, keep)
    n = hc.n
    offs = np.zeros(n + 1, dtype=np.uint64)
    total = lib().or_encoded_total(C.byref(os_.s), cols, n, mode, _ptr(offs), max(nthreads, 8))
    arena = np.zeros(max(total, 1), dtype=np.uint8)
    st = np.zeros(max(n, 1), dtype=np.uint32)
    r = lib().or_encode_batch(C.byref(os_.s), cols, n, mode, _ptr(arena), arena.size, _ptr(offs),
                              _ptr(st), nthreads)
    assert r == total, (r, total)
    return arena[:total], offs, st[:n]


class DecodeOut:
    def __init__(self, specs, n):
        self.specs = specs
        self.n = n
        self.data, self.valid, self.start, self.length = [], [], [], []
        for sp in specs:
            self.data.append(np.zeros(max(n * sp.width, 1), np.uint8) if sp.fixed else None)
            self.valid.append(np.full(max(n, 1), 255, np.uint8) if sp.has_valid else None)
            self.start.append(np.zeros(max(n, 1), np.uint64) if sp.var else None)
            self.length.append(np.zeros(max(n, 1), np.uint32) if sp.var else None)

    def cols(self):
        arr = (PackosColumn * max(1, len(self.specs)))()
        for c in range(len(self.specs)):
            arr[c].data = _ptr(self.data[c])
            arr[c].valid = _ptr(self.valid[c])
            arr[c].start = _ptr(self.start[c])
            arr[c].length = _ptr(self.length[c])
        return arr


def decode(chain, arena: np.ndarray, offsets: Optional[np.ndarray], n: int, stride: int = 0,
           nthreads=1, mode=0):
    from packos_amd.columns import column_specs
    os_ = OracleSchema(chain)
    out = DecodeOut(column_specs(chain), n)
    st = np.zeros(max(n, 1), np.uint32)
    a = np.ascontiguousarray(arena, dtype=np.uint8)
    if a.size == 0:
        a = np.zeros(1, np.uint8)
    o = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
    lib().or_decode_batch_mode(C.byref(os_.s), _ptr(a), _ptr(o), stride, n, out.cols(), _ptr(st),
                               nthreads, mode)
    return out, st[:n]


def validate(chain, arena: np.ndarray, offsets: Optional[np.ndarray], n: int, stride: int = 0,
             nthreads=1, mode=0):
    """or_validate_batch: ValidateBuffer's status word per blob."""
    os_ = OracleSchema(chain)
    st = np.zeros(max(n, 1), np.uint32)
    a = np.ascontiguousarray(arena, dtype=np.uint8)
    if a.size == 0:
        a = np.zeros(1, np.uint8)
    o = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
    lib().or_validate_batch(C.byref(os_.s), _ptr(a), _ptr(o), stride, n, _ptr(st), nthreads, mode)
    return st[:n]


def get_field_batch(arena, offsets, n, path, want_tag, want_width, stride=0):
    a = np.ascontiguousarray(arena, dtype=np.uint8)
    if a.size == 0:
        a = np.zeros(1, np.uint8)
    o = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
    p = np.asarray(path, dtype=np.int32)
    s0 = np.zeros(max(n, 1), np.uint64)
    ln = np.zeros(max(n, 1), np.uint32)
    tg = np.zeros(max(n, 1), np.uint8)
    st = np.zeros(max(n, 1), np.uint8)
    lib().or_get_field_batch(_ptr(a), _ptr(o), stride, n, _ptr(p), len(path), want_tag,
                             want_width, _ptr(s0), _ptr(ln), _ptr(tg), _ptr(st))
    return s0[:n], ln[:n], tg[:n], st[:n]


def get_batch(arena, offsets, n, path, getter, want_tag=0, want_width=0, stride=0, values=True):
    """or_get_batch: (values, start, length, tag, status), same contract as
    packos_amd.api.get_batch."""
    a = np.ascontiguousarray(arena, dtype=np.uint8)
    if a.size == 0:
        a = np.zeros(1, np.uint8)
    o = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
    p = np.asarray(path, dtype=np.int32)
    fam = getter & 0xFF
    vw = 8 if fam in (3, 4) else max(want_width, 0)
    gather = values and fam not in (2, 5) and vw > 0
    vals = np.zeros((max(n, 1), vw), np.uint8) if gather else None
    s0 = np.zeros(max(n, 1), np.uint64)
    ln = np.zeros(max(n, 1), np.uint32)
    tg = np.zeros(max(n, 1), np.uint8)
    st = np.zeros(max(n, 1), np.uint8)
    lib().or_get_batch(_ptr(a), _ptr(o), stride, n, _ptr(p), len(path), getter, want_tag, want_width,
                       _ptr(vals), vw if gather else 0, _ptr(s0), _ptr(ln), _ptr(tg), _ptr(st))
    return (None if vals is None else vals[:n]), s0[:n], ln[:n], tg[:n], st[:n]


def get_map_batch(arena, offsets, n, path, flags, max_pairs, stride=0):
    """or_get_map_batch: (pairs, key_start, key_len, val_start, val_len,
    val_tag, status) with (n, max_pairs) span arrays, the contract of
    packos_amd.api.get_map_batch."""
    a = np.ascontiguousarray(arena, dtype=np.uint8)
    if a.size == 0:
        a = np.zeros(1, np.uint8)
    o = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
    p = np.asarray(path, dtype=np.int32)
    m = max(max_pairs, 1)
    pr = np.zeros(max(n, 1), np.uint32)
    ks, kl = np.zeros((max(n, 1), m), np.uint64), np.zeros((max(n, 1), m), np.uint32)
    vs, vl = np.zeros((max(n, 1), m), np.uint64), np.zeros((max(n, 1), m), np.uint32)
    vt = np.zeros((max(n, 1), m), np.uint8)
    st = np.zeros(max(n, 1), np.uint8)
    lib().or_get_map_batch(_ptr(a), _ptr(o), stride, n, _ptr(p), len(path), flags, max_pairs, _ptr(pr), _ptr(ks),
                           _ptr(kl), _ptr(vs), _ptr(vl), _ptr(vt), _ptr(st))
    mp = max_pairs
    return pr[:n], ks[:n, :mp], kl[:n, :mp], vs[:n, :mp], vl[:n, :mp], vt[:n, :mp], st[:n]


# ---- single-buffer GetAccess / SeqGetAccess wrappers (golden decode tests) ----
class Get:
    def __init__(self, buf: bytes):
        self.arr = np.frombuffer(bytes(buf) + b"\x00\x00", dtype=np.uint8).copy()
        self.g = OrGet()
        self.ok = bool(lib().or_get_init(C.byref(self.g), _ptr(self.arr), len(buf)))

    def fixed(self, pos, tag, width):
        st = C.c_int64()
        r = lib().or_get_fixed(C.byref(self.g), pos, tag, width, C.byref(st))
        if r:
            return None
        return bytes(self.arr[st.value: st.value + width])

    def span(self, pos):
        a, b = C.c_int64(), C.c_int64()
        if lib().or_get_span(C.byref(self.g), pos, C.byref(a), C.byref(b)):
            return None
        return bytes(self.arr[a.value:b.value])

    def nested(self, pos):
        nx = Get(b"")
        tp = C.c_int()
        r = lib().or_get_nested(C.byref(self.g), pos, C.byref(nx.g), C.byref(tp))
        if r:
            return None
        nx.arr = self.arr  # nested buf points into parent array
        off = nx.g.buf - self.g.buf
        sub = Get(bytes(self.arr[off: off + nx.g.len]))
        return sub

    @property
    def arg_count(self):
        return self.g.arg_count


class Seq:
    def __init__(self, buf: bytes, _arr=None):
        self.arr = _arr if _arr is not None else np.frombuffer(bytes(buf) + b"\x00\x00",
                                                               dtype=np.uint8).copy()
        self.q = OrSeq()
        if _arr is None:
            self.err = lib().or_seq_init(C.byref(self.q), _ptr(self.arr), len(buf))

    def next(self):
        s, w, t = C.c_int64(), C.c_int64(), C.c_int()
        r = lib().or_seq_next(C.byref(self.q), C.byref(s), C.byref(w), C.byref(t))
        base = self.q.buf - _ptr(self.arr)
        if r:
            return None, t.value, True
        return bytes(self.arr[base + s.value: base + s.value + w.value]), t.value, False

    def peek(self):
        t, w = C.c_int(), C.c_int64()
        r = lib().or_seq_peek(C.byref(self.q), C.byref(t), C.byref(w))
        return t.value, w.value, bool(r)

    def advance(self):
        return lib().or_seq_advance(C.byref(self.q)) == 0

    def nested(self):
        sub = Seq(b"", _arr=self.arr)
        r = lib().or_seq_peek_nested(C.byref(self.q), C.byref(sub.q))
        if r:
            return None
        sub.err = 0
        return sub
