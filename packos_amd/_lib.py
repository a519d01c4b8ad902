"""ctypes binding of libpackos.so (the C ABI in include/packos.h).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc, gfx950).
There is no fallback: if the shared object is missing every batch call
raises, so a GPU run can never silently route around the HIP kernels.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PACKOS_LIB") or os.path.join(HERE, "libpackos.so")  # override: experiments only

ABI_VERSION = 4        # PACKOS_ABI_VERSION this binding's structs and signatures follow
MODE_PUTACCESS = 0
MODE_PACKABLE = 1
MODE_EXTENDED = 0x100   # ADR-001 extended containers (include/packos.h), OR-ed into a mode
ENC_OFFSETS_READY = 1
ENC_FORCE_GENERIC = 2
ENC_CAP_EXACT = 4       # out_capacity is the batch's exact encoded size (the kernel choice is made on the host)
ENC_SIZED = 8           # out_offsets hold packos_encoded_size_batch's result (no second size pass)


def ENC_FIXED_VARIANT(v: int) -> int:
    """PACKOS_ENC_FIXED_VARIANT(v): testing/benchmark knob (include/packos.h)."""
    return (v & 0xF) << 4

STATUS_PANIC = 0x40000000
STATUS_OVERFLOW13 = 0x80000000

KIND_NAMES = {1: "int", 2: "uint", 3: "float", 4: "bool", 5: "string", 6: "bytes", 7: "tuple",
              8: "map"}

EXPORTED = [
    "packos_schema_compile", "packos_schema_free", "packos_schema_num_columns",
    "packos_schema_num_top_fields", "packos_schema_column_info", "packos_schema_fixed_blob_size",
    "packos_schema_ext_overhead",
    "packos_schema_decode_fast", "packos_schema_has_checks", "packos_schema_column_default",
    "packos_schema_describe", "packos_schema_blob_size_host", "packos_encode_workspace_size",
    "packos_encoded_size_batch", "packos_encode_batch", "packos_encode_host_batch", "packos_decode_host_batch", "packos_decode_batch",
    "packos_pipeline_create", "packos_pipeline_free", "packos_pipeline_encode", "packos_pipeline_decode",
    "packos_pipeline_validate", "packos_validate_batch", "packos_validate_host_batch",
    "packos_get_field_batch", "packos_get_batch", "packos_get_map_batch", "packos_strerror", "packos_last_error", "packos_abi_version",
    "packos_last_encoder",
]


class PackosColumn(C.Structure):
    _fields_ = [("data", C.c_void_p), ("offsets", C.c_void_p), ("valid", C.c_void_p),
                ("start", C.c_void_p), ("length", C.c_void_p), ("offsets64", C.c_void_p)]


class PackosColumnInfo(C.Structure):
    _fields_ = [("kind", C.c_int32), ("width", C.c_int32), ("nullable", C.c_int32),
                ("tag", C.c_int32), ("top_index", C.c_int32), ("depth", C.c_int32),
                ("name", C.c_char * 96)]


class PackosError(RuntimeError):
    def __init__(self, code: int, where: str):
        L = lib()
        msg = L.packos_strerror(code).decode()
        detail = L.packos_last_error().decode()
        super().__init__(f"{where}: {msg} ({code}){': ' + detail if detail else ''}")
        self.code = code


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
    L = C.CDLL(LIB_PATH)
    vp, sz, i32, u32, u64, i64 = C.c_void_p, C.c_size_t, C.c_int, C.c_uint32, C.c_uint64, C.c_int64
    L.packos_schema_compile.argtypes = [C.c_char_p, i32, C.POINTER(vp)]
    L.packos_schema_free.argtypes = [vp]
    L.packos_schema_free.restype = None
    L.packos_schema_num_columns.argtypes = [vp]
    L.packos_schema_num_top_fields.argtypes = [vp]
    L.packos_schema_column_info.argtypes = [vp, i32, C.POINTER(PackosColumnInfo)]
    L.packos_schema_fixed_blob_size.argtypes = [vp]
    L.packos_schema_fixed_blob_size.restype = i64
    L.packos_schema_ext_overhead.argtypes = [vp]
    L.packos_schema_ext_overhead.restype = i64
    L.packos_schema_decode_fast.argtypes = [vp]
    L.packos_schema_decode_fast.restype = C.c_int
    L.packos_schema_has_checks.argtypes = [vp]
    L.packos_schema_has_checks.restype = C.c_int
    L.packos_schema_column_default.argtypes = [vp, i32, C.c_char_p, sz]
    L.packos_schema_column_default.restype = i64
    L.packos_schema_describe.argtypes = [vp, C.c_char_p, sz]
    L.packos_schema_describe.restype = sz
    L.packos_schema_blob_size_host.argtypes = [vp, vp, vp]
    L.packos_schema_blob_size_host.restype = i64
    L.packos_encode_workspace_size.argtypes = [vp, sz]
    L.packos_encode_workspace_size.restype = sz
    L.packos_encoded_size_batch.argtypes = [vp, C.POINTER(PackosColumn), sz, vp, vp, sz, vp]
    L.packos_encode_batch.argtypes = [vp, C.POINTER(PackosColumn), sz, vp, u64, vp, vp, vp, sz,
                                      u32, vp]
    L.packos_encode_host_batch.argtypes = [vp, C.POINTER(PackosColumn), sz, vp, u64, vp, vp, sz]
    L.packos_decode_host_batch.argtypes = [vp, vp, vp, u64, sz, C.POINTER(PackosColumn), vp, sz]
    L.packos_pipeline_create.argtypes = [vp, sz, i32, C.POINTER(vp)]
    L.packos_pipeline_free.argtypes = [vp]
    L.packos_pipeline_free.restype = None
    L.packos_pipeline_encode.argtypes = [vp, C.POINTER(PackosColumn), sz, vp, u64, vp, vp]
    L.packos_pipeline_decode.argtypes = [vp, vp, vp, u64, sz, C.POINTER(PackosColumn), vp]
    L.packos_decode_batch.argtypes = [vp, vp, vp, u64, sz, C.POINTER(PackosColumn), vp, vp]
    L.packos_validate_batch.argtypes = [vp, vp, vp, u64, sz, vp, vp]
    L.packos_validate_host_batch.argtypes = [vp, vp, vp, u64, sz, vp, sz]
    L.packos_pipeline_validate.argtypes = [vp, vp, vp, u64, sz, vp]
    L.packos_get_field_batch.argtypes = [vp, vp, u64, sz, C.POINTER(C.c_int32), i32, i32, i32,
                                         vp, vp, vp, vp, vp]
    L.packos_get_batch.argtypes = [vp, vp, u64, sz, C.POINTER(C.c_int32), i32, i32, i32, i32,
                                   vp, u32, vp, vp, vp, vp, vp]
    L.packos_get_map_batch.argtypes = [vp, vp, u64, sz, C.POINTER(C.c_int32), i32, i32, u32, vp, vp, vp, vp, vp,
                                       vp, vp, vp]
    L.packos_strerror.argtypes = [i32]
    L.packos_strerror.restype = C.c_char_p
    L.packos_last_error.restype = C.c_char_p
    if os.environ.get("PACKOS_LIB") is None or hasattr(L, "packos_last_encoder"):   # older builds in A/Bs lack it
        L.packos_last_encoder.restype = C.c_char_p
    L.packos_abi_version.restype = i32
    got = L.packos_abi_version()
    if got != ABI_VERSION:   # a stale or foreign .so would read packos_column with the wrong stride
        raise RuntimeError(f"{LIB_PATH}: packos_abi_version() = {got}, this binding needs {ABI_VERSION}; "
                           "rebuild it with __graft_entry__.build()")
    _lib = L
    return L


def check(code: int, where: str):
    if code != 0:
        raise PackosError(code, where)
