"""Batch API over the C ABI: compile a schema once, then encode / decode whole
batches of blobs resident in MI355X HBM.

Reference correspondence (quickwritereader/PackOS):

* ``CompiledSchema``      <- schema.BuildSchema + the Schema tree (schema/schema.go:177-182)
* ``encode_batch``        <- PutAccess Add*/Pack() (access/put.go:69-308,619) per blob, or
                             packable.Pack(args...) (packable/pack.go:59) with mode=MODE_PACKABLE
* ``decode_batch``        <- schema.DecodeBuffer (schema/schema.go:893) per blob
* ``get_field_batch``     <- GetAccess.Get*(pos) (access/get.go:60-375)

Device memory is torch CUDA tensors (plumbing only); every byte of PackOS
work happens in libpackos.so's HIP kernels.
"""
from __future__ import annotations

import ctypes as C
import json
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from . import _lib
from ._lib import MODE_EXTENDED, MODE_PACKABLE, MODE_PUTACCESS, PackosColumn, PackosColumnInfo, check, lib
from .columns import HostColumns, column_specs
from .schema import SchemaChain

__all__ = ["CompiledSchema", "DeviceColumns", "DecodedColumns", "HostDecoded", "encode_batch", "decode_batch",
           "encode_host_batch", "decode_host_batch", "Pipeline",
           "get_field_batch", "get_batch", "get_map_batch", "GET_FIXED", "GET_NULLABLE", "GET_SPAN", "GET_INT",
           "GET_FLOAT", "GET_ANY", "GET_EXTENDED", "MAP_STR", "MAP_ANY", "MODE_PUTACCESS", "MODE_PACKABLE", "MODE_EXTENDED"]


def _torch():
    import torch
    return torch


class CompiledSchema:
    """A compiled, immutable schema handle (packos_schema*)."""

    def __init__(self, chain, mode: int = MODE_PUTACCESS):
        if isinstance(chain, SchemaChain):
            self.chain = chain
            js = json.dumps(chain.to_json())
        else:
            from .schema import BuildChain
            js = chain if isinstance(chain, str) else json.dumps(chain)
            self.chain = BuildChain(js)
        self.mode = mode
        self.json = js
        h = C.c_void_p()
        check(lib().packos_schema_compile(js.encode(), mode, C.byref(h)), "packos_schema_compile")
        self._h = h
        self.specs = column_specs(self.chain)
        n = lib().packos_schema_num_columns(h)
        assert n == len(self.specs), (n, len(self.specs))

    @property
    def handle(self):
        return self._h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().packos_schema_free(h)
            except Exception:
                pass
            self._h = None

    @property
    def n_columns(self) -> int:
        return lib().packos_schema_num_columns(self._h)

    def column_info(self, c: int) -> dict:
        ci = PackosColumnInfo()
        check(lib().packos_schema_column_info(self._h, c, C.byref(ci)), "column_info")
        return {"kind": _lib.KIND_NAMES.get(ci.kind, "?"), "width": ci.width,
                "nullable": bool(ci.nullable), "tag": ci.tag, "top_index": ci.top_index,
                "depth": ci.depth, "name": ci.name.decode()}

    @property
    def fixed_blob_size(self) -> int:
        return int(lib().packos_schema_fixed_blob_size(self._h))

    @property
    def ext_overhead(self) -> int:
        """MODE_EXTENDED: most bytes extended header blocks add to one blob (0 otherwise)."""
        return int(lib().packos_schema_ext_overhead(self._h))

    @property
    def decode_fast(self) -> bool:
        """True when decode_batch uses the tiled fixed-layout decoder."""
        return bool(lib().packos_schema_decode_fast(self._h))

    @property
    def has_checks(self) -> bool:
        """True when encode needs a status array (value checks, include/packos.h)."""
        return bool(lib().packos_schema_has_checks(self._h))

    def all_present_size(self) -> int:
        return int(lib().packos_schema_blob_size_host(self._h, None, None))

    def blob_size_host(self, widths: Optional[np.ndarray] = None,
                       valid: Optional[np.ndarray] = None) -> int:
        w = None if widths is None else np.ascontiguousarray(widths, np.uint32)
        v = None if valid is None else np.ascontiguousarray(valid, np.uint8)
        return int(lib().packos_schema_blob_size_host(
            self._h, None if w is None else w.ctypes.data, None if v is None else v.ctypes.data))

    def column_default(self, c: int) -> bytes:
        """decodeDefault literal of column c (b"" when it has none)."""
        n = int(lib().packos_schema_column_default(self._h, c, None, 0))
        if n <= 0:
            return b""
        buf = C.create_string_buffer(n)
        lib().packos_schema_column_default(self._h, c, buf, n)
        return buf.raw[:n]

    def describe(self) -> str:
        n = lib().packos_schema_describe(self._h, None, 0)
        buf = C.create_string_buffer(n)
        lib().packos_schema_describe(self._h, buf, n)
        return buf.value.decode()


class DeviceColumns:
    """Input column set resident on a GPU (one entry per schema column)."""

    def __init__(self, schema: CompiledSchema, n: int, data, offsets, valid):
        self.schema = schema
        self.n = int(n)
        self.data: List = data
        self.offsets: List = offsets
        self.valid: List = valid

    @classmethod
    def from_host(cls, schema: CompiledSchema, hc: HostColumns, device="cuda"):
        torch = _torch()
        data, offs, valid = [], [], []
        for c, sp in enumerate(schema.specs):
            d = hc.data[c]
            if d is not None:
                t = torch.from_numpy(d if d.size else np.zeros(16, np.uint8)).to(device)
                data.append(t)
            else:
                data.append(None)
            o = hc.offsets[c]
            offs.append(None if o is None else torch.from_numpy(o.view(np.int32)).to(device))
            v = hc.valid[c]
            valid.append(None if v is None else torch.from_numpy(v).to(device))
        return cls(schema, hc.n, data, offs, valid)

    def any_valid(self) -> bool:
        return any(v is not None for v in self.valid)

    def has_var(self) -> bool:
        return any(sp.var for sp in self.schema.specs)

    def ctypes_array(self):
        arr = (PackosColumn * max(1, len(self.schema.specs)))()
        for c in range(len(self.schema.specs)):
            arr[c].data = self.data[c].data_ptr() if self.data[c] is not None else None
            arr[c].offsets = self.offsets[c].data_ptr() if self.offsets[c] is not None else None
            arr[c].valid = self.valid[c].data_ptr() if self.valid[c] is not None else None
        return arr

    def nbytes(self) -> int:
        t = 0
        for lst in (self.data, self.offsets, self.valid):
            for x in lst:
                if x is not None:
                    t += x.numel() * x.element_size()
        return t


def _stream_ptr(stream):
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)


@dataclass
class EncodeResult:
    arena: object      # torch.uint8 [total]
    offsets: object    # torch.int64 [n+1] or None (fixed size: blob i at i*B)
    status: object     # torch.int32 [n] or None
    total: int
    blob_size: int     # B for fixed-size batches, -1 otherwise


def encode_batch(schema: CompiledSchema, cols: DeviceColumns, want_offsets: bool = True,
                 want_status: bool = True, out=None, stream=None, flags: int = 0) -> EncodeResult:
    """Encode every blob of the batch (async on `stream`; one host sync for
    variable-size batches to size the arena)."""
    torch = _torch()
    L = lib()
    n = cols.n
    dev = cols.data[0].device if cols.data and cols.data[0] is not None else torch.device("cuda")
    st = _stream_ptr(stream)
    arr = cols.ctypes_array()
    want_status = want_status or schema.has_checks   # checks report through the status only
    status = torch.empty(max(n, 1), dtype=torch.int32, device=dev) if want_status else None
    fixed = (not cols.has_var()) and not cols.any_valid() and schema.fixed_blob_size >= 0
    if fixed:
        B = schema.all_present_size()
        total = B * n
        if out is None:
            out = torch.empty(max(total, 16), dtype=torch.uint8, device=dev)
        offs = torch.empty(n + 1, dtype=torch.int64, device=dev) if want_offsets else None
        check(L.packos_encode_batch(schema.handle, arr, n, out.data_ptr(), out.numel(),
                                    None if offs is None else offs.data_ptr(),
                                    None if status is None else status.data_ptr(), None, 0, flags, st),
              "packos_encode_batch")
        return EncodeResult(out, offs, status[:n] if status is not None else None, total, B)
    offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    wsb = L.packos_encode_workspace_size(schema.handle, n)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    check(L.packos_encoded_size_batch(schema.handle, arr, n, offs.data_ptr(), ws.data_ptr(), wsb, st),
          "packos_encoded_size_batch")
    total = int(offs[n].item()) if n else 0
    if out is None or out.numel() < total:
        out = torch.empty(max(total, 16), dtype=torch.uint8, device=dev)
    # the size pass above gave the layout and the exact size: no second size
    # pass (a closed-form layout is rewritten identically by the encoder), and
    # the kernel choice from the exact size (no read-back, no device pick)
    flags |= _lib.ENC_SIZED | _lib.ENC_CAP_EXACT
    check(L.packos_encode_batch(schema.handle, arr, n, out.data_ptr(), total, offs.data_ptr(),
                                None if status is None else status.data_ptr(), ws.data_ptr(), wsb,
                                flags, st), "packos_encode_batch")
    return EncodeResult(out, offs, status[:n] if status is not None else None, total, -1)


def host_batch_bound(schema: CompiledSchema, hc: HostColumns) -> int:
    """Output bytes that always suffice: every non-var item present in every
    blob + all var bytes."""
    L = lib()
    ncol = len(schema.specs)
    widths = np.zeros(max(1, ncol), dtype=np.uint32)
    valid = np.ones(max(1, ncol), dtype=np.uint8)
    stat = int(L.packos_schema_blob_size_host(schema.handle, widths.ctypes.data, valid.ctypes.data))
    stat += int(L.packos_schema_ext_overhead(schema.handle))   # extended header blocks (MODE_EXTENDED)
    var_bytes = sum(int(o[hc.n]) - int(o[0]) for o in hc.offsets if o is not None)
    return max(16, hc.n * max(stat, 0) + var_bytes)


def _host_encode_args(schema: CompiledSchema, hc: HostColumns, want_status, out, offsets, status):
    """ctypes column array (+ the arrays it points into) and the output
    buffers of a host-resident encode.  A uint64 offsets array binds as
    offsets64 (arenas past 4 GiB)."""
    n = hc.n
    keep = []
    arr = (PackosColumn * max(1, len(schema.specs)))()
    for c in range(len(schema.specs)):
        for name, attr in (("data", "data"), ("offsets", "offsets"), ("valid", "valid")):
            a = getattr(hc, attr)[c]
            if a is None:
                continue
            a = np.ascontiguousarray(a)
            keep.append(a)
            if name == "offsets" and a.dtype == np.uint64:
                name = "offsets64"
            setattr(arr[c], name, a.ctypes.data)
    if out is None:
        out = np.empty(host_batch_bound(schema, hc), dtype=np.uint8)
    offs = offsets if offsets is not None else np.empty(n + 1, dtype=np.uint64)
    want_status = want_status or schema.has_checks
    st = status if status is not None else (np.empty(max(n, 1), dtype=np.uint32) if want_status else None)
    return arr, keep, out, offs, st


def encode_host_batch(schema: CompiledSchema, hc: HostColumns, chunk_blobs: int = 0,
                      want_status: bool = True, out=None, offsets=None, status=None):
    """Host-resident batch -> host arena through packos_encode_host_batch
    (the schema's cached pipeline on the current device: H2D, kernels and D2H
    of consecutive chunks overlap; the entry point a cgo shim binds).  `out` /
    `offsets` / `status` may be preallocated numpy arrays (e.g. views of
    pinned memory).  Returns (arena, offsets, status); arena is trimmed to the
    encoded bytes."""
    n = hc.n
    arr, keep, out, offs, st = _host_encode_args(schema, hc, want_status, out, offsets, status)
    check(lib().packos_encode_host_batch(schema.handle, arr, n, out.ctypes.data, out.size, offs.ctypes.data,
                                         None if st is None else st.ctypes.data, chunk_blobs),
          "packos_encode_host_batch")
    del keep
    return out[: int(offs[n])], offs, (st[:n] if st is not None else None)


class Pipeline:
    """An explicit host pipeline (packos_pipeline_create): device buffers,
    streams and events kept across calls, bound to the current device.  The
    schema must outlive it."""

    def __init__(self, schema: CompiledSchema, chunk_blobs: int = 0, slots: int = 0):
        self.schema = schema
        h = C.c_void_p()
        check(lib().packos_pipeline_create(schema.handle, chunk_blobs, slots, C.byref(h)), "packos_pipeline_create")
        self._h = h

    def close(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib().packos_pipeline_free(h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def encode(self, hc: HostColumns, want_status: bool = True, out=None, offsets=None, status=None):
        """packos_pipeline_encode: (arena, offsets, status) like encode_host_batch."""
        n = hc.n
        arr, keep, out, offs, st = _host_encode_args(self.schema, hc, want_status, out, offsets, status)
        check(lib().packos_pipeline_encode(self._h, arr, n, out.ctypes.data, out.size, offs.ctypes.data,
                                           None if st is None else st.ctypes.data), "packos_pipeline_encode")
        del keep
        return out[: int(offs[n])], offs, (st[:n] if st is not None else None)

    def decode(self, arena: np.ndarray, offsets: Optional[np.ndarray], n: int, stride: int = 0,
               out: Optional["HostDecoded"] = None, status: Optional[np.ndarray] = None):
        """packos_pipeline_decode: (HostDecoded, status) like decode_host_batch."""
        a = np.ascontiguousarray(arena, dtype=np.uint8)
        o = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
        out = out if out is not None else HostDecoded(self.schema, n)
        st = status if status is not None else np.empty(max(n, 1), np.uint32)
        check(lib().packos_pipeline_decode(self._h, a.ctypes.data if a.size else None,
                                           None if o is None else o.ctypes.data, stride, n, out.ctypes_array(),
                                           st.ctypes.data), "packos_pipeline_decode")
        return out, st[:n]

    def validate(self, arena: np.ndarray, offsets: Optional[np.ndarray], n: int, stride: int = 0,
                 status: Optional[np.ndarray] = None):
        """packos_pipeline_validate: the status like validate_host_batch."""
        a = np.ascontiguousarray(arena, dtype=np.uint8)
        o = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
        st = status if status is not None else np.empty(max(n, 1), np.uint32)
        check(lib().packos_pipeline_validate(self._h, a.ctypes.data if a.size else None,
                                             None if o is None else o.ctypes.data, stride, n, st.ctypes.data),
              "packos_pipeline_validate")
        return st[:n]


class HostDecoded:
    """Host (numpy) decode output of decode_host_batch, the layout of
    DecodedColumns: fixed rows, validity, absolute (start, length) views into
    the host arena."""

    def __init__(self, schema: CompiledSchema, n: int, alloc=np.zeros):
        self.schema, self.n = schema, n
        self.data, self.valid, self.start, self.length = [], [], [], []
        for sp in schema.specs:
            self.data.append(alloc(max(n * sp.width, 16), np.uint8) if sp.fixed else None)
            self.valid.append(alloc(max(n, 1), np.uint8) if sp.has_valid else None)
            self.start.append(alloc(max(n, 1), np.uint64) if sp.var else None)
            self.length.append(alloc(max(n, 1), np.uint32) if sp.var else None)

    def ctypes_array(self):
        arr = (PackosColumn * max(1, len(self.schema.specs)))()
        for c in range(len(self.schema.specs)):
            for name in ("data", "valid", "start", "length"):
                a = getattr(self, name)[c]
                if a is not None:
                    setattr(arr[c], name, a.ctypes.data)
        return arr


def decode_host_batch(schema: CompiledSchema, arena: np.ndarray, offsets: Optional[np.ndarray], n: int,
                      stride: int = 0, chunk_blobs: int = 0, out: Optional[HostDecoded] = None,
                      status: Optional[np.ndarray] = None):
    """DecodeBuffer over a HOST-resident batch through packos_decode_host_batch
    (the schema's cached pipeline: chunked H2D / decode / D2H overlapped; the
    cgo shim's read entry point).  Returns (HostDecoded, status)."""
    a = np.ascontiguousarray(arena, dtype=np.uint8)
    o = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
    out = out if out is not None else HostDecoded(schema, n)
    st = status if status is not None else np.empty(max(n, 1), np.uint32)
    check(lib().packos_decode_host_batch(schema.handle, a.ctypes.data if a.size else None,
                                         None if o is None else o.ctypes.data, stride, n, out.ctypes_array(),
                                         st.ctypes.data, chunk_blobs), "packos_decode_host_batch")
    return out, st[:n]


class EncodePlan:
    """Pre-bound encode of one batch into a preallocated arena: run() issues
    only C-ABI calls on `stream` (no host sync, no allocation) — what a serving
    loop or a graph capture replays.  Fixed-size batches: one encode call.
    Variable-size batches: one packos_encode_batch call (size kernel with a
    look-back scan, then the encode kernel); the arena is sized once at construction
    (one host sync there) and `offsets` / `status` are refreshed by every
    run()."""

    def __init__(self, schema: CompiledSchema, cols: DeviceColumns, out=None, stream=None, flags: int = 0,
                 want_status: bool = False):
        torch = _torch()
        L = lib()
        self.flags = flags
        self.schema, self.cols = schema, cols
        n = cols.n
        dev = cols.data[0].device if cols.data and cols.data[0] is not None else torch.device("cuda")
        self.fixed = (not cols.has_var()) and not cols.any_valid() and schema.fixed_blob_size >= 0
        self._arr = cols.ctypes_array()
        self._stream = stream
        want_status = want_status or schema.has_checks
        self.status = torch.empty(max(n, 1), dtype=torch.int32, device=dev) if want_status else None
        if self.fixed:
            self.B = schema.all_present_size()
            self.total = self.B * n
            self.offsets = None
            self.ws, self.wsb = None, 0
        else:
            self.B = -1
            self.offsets = torch.empty(n + 1, dtype=torch.int64, device=dev)
            self.wsb = L.packos_encode_workspace_size(schema.handle, n)
            self.ws = torch.empty(max(self.wsb, 16), dtype=torch.uint8, device=dev)
            check(L.packos_encoded_size_batch(schema.handle, self._arr, n, self.offsets.data_ptr(),
                                              self.ws.data_ptr(), self.wsb, _stream_ptr(stream)),
                  "packos_encoded_size_batch")
            if stream is not None:
                stream.synchronize()
            self.total = int(self.offsets[n].item()) if n else 0
        self.out = out if out is not None else torch.empty(max(self.total, 16), dtype=torch.uint8, device=dev)
        if self.out.numel() < self.total:
            raise ValueError("EncodePlan: `out` is smaller than the batch's encoded size")
        # the capacity passed is the batch's exact size (known from the size
        # pass above, whatever `out` holds beyond it): the kernel choice is made
        # on the host and run() never reads anything back
        self.cap = self.out.numel() if self.fixed else self.total
        if not self.fixed:
            self.flags |= _lib.ENC_CAP_EXACT

    def run(self):
        L = lib()
        st = _stream_ptr(self._stream)
        n = self.cols.n
        stp = None if self.status is None else self.status.data_ptr()
        if self.fixed:
            check(L.packos_encode_batch(self.schema.handle, self._arr, n, self.out.data_ptr(), self.out.numel(),
                                        None, stp, None, 0, self.flags, st), "packos_encode_batch")
            return self.out
        # one call: the size kernel (sizes + look-back scan -> offsets) and the
        # encode kernel; `offsets` is rewritten by every run
        check(L.packos_encode_batch(self.schema.handle, self._arr, n, self.out.data_ptr(), self.cap,
                                    self.offsets.data_ptr(), stp, self.ws.data_ptr(), self.wsb,
                                    self.flags, st), "packos_encode_batch")
        return self.out


class DecodedColumns:
    """Decode output: fixed columns, validity, (start, length) views of var
    columns into the input arena."""

    def __init__(self, schema: CompiledSchema, n: int, device):
        torch = _torch()
        self.schema, self.n = schema, n
        self.data, self.valid, self.start, self.length = [], [], [], []
        for sp in schema.specs:
            self.data.append(torch.zeros(max(n * sp.width, 16), dtype=torch.uint8, device=device)
                             if sp.fixed else None)
            self.valid.append(torch.full((max(n, 1),), 255, dtype=torch.uint8, device=device)
                              if sp.has_valid else None)
            self.start.append(torch.zeros(max(n, 1), dtype=torch.int64, device=device) if sp.var else None)
            self.length.append(torch.zeros(max(n, 1), dtype=torch.int32, device=device) if sp.var else None)

    def var_values(self, c: int, arena) -> List[bytes]:
        """Bytes of var column c per blob (host copy): the arena slice each view
        aliases, or the schema's decodeDefault literal for PACKOS_VIEW_DEFAULT
        views (what DecodeBuffer returns, schema/schema.go:279-286)."""
        a = arena.cpu().numpy() if hasattr(arena, "cpu") else np.asarray(arena)
        st = self.start[c][: self.n].cpu().numpy().view(np.uint64)
        ln = self.length[c][: self.n].cpu().numpy().view(np.uint32)
        dflt = self.schema.column_default(c)
        return [dflt if int(s0) == VIEW_DEFAULT else bytes(a[int(s0): int(s0) + int(l0)])
                for s0, l0 in zip(st, ln)]

    def ctypes_array(self):
        arr = (PackosColumn * max(1, len(self.schema.specs)))()
        for c in range(len(self.schema.specs)):
            arr[c].data = self.data[c].data_ptr() if self.data[c] is not None else None
            arr[c].valid = self.valid[c].data_ptr() if self.valid[c] is not None else None
            arr[c].start = self.start[c].data_ptr() if self.start[c] is not None else None
            arr[c].length = self.length[c].data_ptr() if self.length[c] is not None else None
        return arr


def decode_batch(schema: CompiledSchema, arena, offsets=None, n: Optional[int] = None, stride: int = 0,
                 stream=None, out: Optional[DecodedColumns] = None, status=None):
    """schema.DecodeBuffer over every blob; returns (DecodedColumns, status).
    `out` / `status` reuse buffers from an earlier call (no allocation)."""
    torch = _torch()
    if n is None:
        n = offsets.numel() - 1
    if out is None:
        out = DecodedColumns(schema, n, arena.device)
    elif out.n < n or out.schema is not schema:
        raise ValueError("decode_batch: `out` was allocated for another schema or a smaller batch")
    if status is None:
        status = torch.empty(max(n, 1), dtype=torch.int32, device=arena.device)
    elif status.numel() < n or status.dtype != torch.int32:
        raise ValueError("decode_batch: `status` needs n int32 entries")
    check(lib().packos_decode_batch(schema.handle, arena.data_ptr(),
                                    None if offsets is None else offsets.data_ptr(), stride, n,
                                    out.ctypes_array(), status.data_ptr(), _stream_ptr(stream)),
          "packos_decode_batch")
    return out, status[:n]


def validate_batch(schema: CompiledSchema, arena, offsets=None, n: Optional[int] = None, stride: int = 0,
                   stream=None, status=None):
    """schema.ValidateBuffer over every blob (packos_validate_batch): the int32
    status word per blob, under the Validate methods' rules
    (schema/schema.go:880-891; include/packos.h lists where they differ from
    DecodeBuffer's).  No columns."""
    torch = _torch()
    if n is None:
        n = offsets.numel() - 1
    if status is None:
        status = torch.empty(max(n, 1), dtype=torch.int32, device=arena.device)
    elif status.numel() < n or status.dtype != torch.int32:
        raise ValueError("validate_batch: `status` needs n int32 entries")
    check(lib().packos_validate_batch(schema.handle, arena.data_ptr(),
                                      None if offsets is None else offsets.data_ptr(), stride, n,
                                      status.data_ptr(), _stream_ptr(stream)), "packos_validate_batch")
    return status[:n]


def validate_host_batch(schema: CompiledSchema, arena: np.ndarray, offsets: Optional[np.ndarray], n: int,
                        stride: int = 0, chunk_blobs: int = 0, status: Optional[np.ndarray] = None):
    """ValidateBuffer over a HOST-resident batch (packos_validate_host_batch):
    the uint32 status per blob."""
    a = np.ascontiguousarray(arena, dtype=np.uint8)
    o = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
    st = status if status is not None else np.empty(max(n, 1), np.uint32)
    check(lib().packos_validate_host_batch(schema.handle, a.ctypes.data if a.size else None,
                                           None if o is None else o.ctypes.data, stride, n, st.ctypes.data,
                                           chunk_blobs), "packos_validate_host_batch")
    return st[:n]


def get_field_batch(arena, offsets, n: int, path, want_tag: int, want_width: int, stride: int = 0,
                    stream=None):
    """GetAccess.Get*(path) over every blob: (start, length, tag, status)."""
    torch = _torch()
    dev = arena.device
    s0 = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    ln = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    tg = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    st = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    p = (C.c_int32 * len(path))(*path)
    check(lib().packos_get_field_batch(arena.data_ptr(), None if offsets is None else offsets.data_ptr(),
                                       stride, n, p, len(path), want_tag, want_width, s0.data_ptr(),
                                       ln.data_ptr(), tg.data_ptr(), st.data_ptr(), _stream_ptr(stream)),
          "packos_get_field_batch")
    return s0[:n], ln[:n], tg[:n], st[:n]


# decode view of an empty string payload replaced by its decodeDefault (include/packos.h)
VIEW_DEFAULT = 0x8000000000000000

# getter families of packos_get_batch (include/packos.h)
GET_FIXED, GET_NULLABLE, GET_SPAN, GET_INT, GET_FLOAT, GET_ANY = range(6)
MAP_STR, MAP_ANY = 0, 1   # packos_get_map_batch: GetMapStr / GetMapAny (include/packos.h)
GET_EXTENDED = 0x100   # OR-ed into a getter: read ADR-001 extended containers (include/packos.h)


def get_batch(arena, offsets, n: int, path, getter: int, want_tag: int = 0, want_width: int = 0,
              stride: int = 0, values: bool = True, spans: bool = True, stream=None):
    """One GetAccess getter over every blob (access/get.go:60-375):
    (values, start, length, tag, status).

    `getter` picks the Get* family: GET_FIXED (Get{Bool,IntN,UintN,FloatN}),
    GET_NULLABLE (GetNullable*: width 0 -> status 4 before the tag check),
    GET_SPAN (GetBytes/GetString), GET_INT (GetInt: any of 1/2/4/8 bytes,
    sign-extended to int64), GET_FLOAT (GetFloating: 4/8 bytes, raw bits),
    GET_ANY (GetTypeAndValue: any tag, end >= start; span + tag only).
    OR GET_EXTENDED into `getter` to read ADR-001 extended containers.
    `values` is an (n, value_width) uint8 tensor of the gathered typed values
    (None for GET_SPAN or values=False); view it with .view(torch.int64) etc.
    spans=False (typed gathers only) skips start / length / tag, returned as
    None: GetInt / GetFloating / Get<T> return just (value, error)."""
    torch = _torch()
    dev = arena.device
    fam = getter & ~GET_EXTENDED   # GET_EXTENDED: read MODE_EXTENDED blobs
    vw = 8 if fam in (GET_INT, GET_FLOAT) else max(want_width, 0)
    gather = values and fam not in (GET_SPAN, GET_ANY) and vw > 0
    if not spans and not gather:
        raise ValueError("spans=False needs a typed gather (values=True, a FIXED/NULLABLE/INT/FLOAT getter)")
    vals = torch.empty((max(n, 1), vw), dtype=torch.uint8, device=dev) if gather else None
    s0 = torch.empty(max(n, 1), dtype=torch.int64, device=dev) if spans else None
    ln = torch.empty(max(n, 1), dtype=torch.int32, device=dev) if spans else None
    tg = torch.empty(max(n, 1), dtype=torch.uint8, device=dev) if spans else None
    st = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    p = (C.c_int32 * len(path))(*path)
    ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    check(lib().packos_get_batch(arena.data_ptr(), None if offsets is None else offsets.data_ptr(), stride, n,
                                 p, len(path), getter, want_tag, want_width,
                                 ptr(vals), vw if gather else 0,
                                 ptr(s0), ptr(ln), ptr(tg), st.data_ptr(), _stream_ptr(stream)),
          "packos_get_batch")
    cut = lambda t: None if t is None else t[:n]  # noqa: E731
    return cut(vals), cut(s0), cut(ln), cut(tg), st[:n]


def get_map_batch(arena, offsets, n: int, path, flags: int = MAP_STR, max_pairs: int = 8, stride: int = 0,
                  stream=None):
    """GetMapStr (flags=MAP_STR) / GetMapAny (MAP_ANY) of the map at `path`
    over every blob (access/get.go:412-490): (pairs, key_start, key_len,
    val_start, val_len, val_tag, status); the span tensors are (n, max_pairs),
    pair j of blob i in wire order (GetMapOrderedAny's order).  status: 0 ok,
    1 decode error, 2 nil nested accessor, 3 nil accessor (panic), 4 nil map,
    5 more pairs than max_pairs, 6 nested deeper than 32 maps."""
    torch = _torch()
    dev = arena.device
    m = max(max_pairs, 1)
    pr = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    ks = torch.empty((max(n, 1), m), dtype=torch.int64, device=dev)
    kl = torch.empty((max(n, 1), m), dtype=torch.int32, device=dev)
    vs = torch.empty((max(n, 1), m), dtype=torch.int64, device=dev)
    vl = torch.empty((max(n, 1), m), dtype=torch.int32, device=dev)
    vt = torch.empty((max(n, 1), m), dtype=torch.uint8, device=dev)
    st = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
    p = (C.c_int32 * len(path))(*path)
    check(lib().packos_get_map_batch(arena.data_ptr(), None if offsets is None else offsets.data_ptr(), stride, n,
                                     p, len(path), flags, max_pairs, pr.data_ptr(), ks.data_ptr(), kl.data_ptr(),
                                     vs.data_ptr(), vl.data_ptr(), vt.data_ptr(), st.data_ptr(), _stream_ptr(stream)),
          "packos_get_map_batch")
    mp = max_pairs
    return pr[:n], ks[:n, :mp], kl[:n, :mp], vs[:n, :mp], vl[:n, :mp], vt[:n, :mp], st[:n]
