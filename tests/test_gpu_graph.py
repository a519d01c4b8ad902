"""Every device-resident entry point is asynchronous on its stream and
capturable in a HIP graph (what a serving loop replays): encode (fixed and
variable layouts, EncodePlan), decode, validate and the GetAccess gather,
captured once, replayed, and bit-exact against the CPU oracle."""
import ctypes as C

import numpy as np
import pytest

import oracle_bridge as ob
from packos_amd import _lib
from packos_amd.api import (CompiledSchema, DecodedColumns, DeviceColumns, EncodePlan, decode_batch,
                            validate_batch)
from packos_amd.configs import CONFIGS, make_columns

pytestmark = pytest.mark.gpu


def torch():
    import torch as t
    return t


def replay(T, fn, times=2):
    s = T.cuda.Stream()
    s.wait_stream(T.cuda.current_stream())
    with T.cuda.stream(s):
        fn()   # warm-up outside the capture (device tables uploaded once)
    T.cuda.current_stream().wait_stream(s)
    T.cuda.synchronize()
    g = T.cuda.CUDAGraph()
    with T.cuda.graph(g):
        fn()
    for _ in range(times):
        g.replay()
    T.cuda.synchronize()


@pytest.mark.parametrize("name", ["M", "C2", "C3", "C4", "C5"])
def test_capture_encode_decode_validate_get(name):
    T = torch()
    cfg = CONFIGS[name]
    hc = make_columns(cfg, n=3000)
    schema = CompiledSchema(cfg.chain, cfg.mode)
    a0, o0, _ = ob.encode(cfg.chain, hc, cfg.mode, nthreads=8)
    n = hc.n
    plan = EncodePlan(schema, DeviceColumns.from_host(schema, hc, "cuda:0"))
    fixed = plan.offsets is None
    stride = plan.B if fixed else 0
    dcols = DecodedColumns(schema, n, "cuda:0")
    dst = T.empty(n, dtype=T.int32, device="cuda:0")
    vst = T.empty(n, dtype=T.int32, device="cuda:0")
    L = _lib.lib()
    path = (C.c_int32 * 1)(0)
    gv = T.empty((n, 8), dtype=T.uint8, device="cuda:0")
    gst = T.empty(n, dtype=T.uint8, device="cuda:0")

    def step():
        st = T.cuda.current_stream()
        plan.run()
        offs = None if fixed else plan.offsets
        decode_batch(schema, plan.out, offs, n, stride=stride, stream=st, out=dcols, status=dst)
        validate_batch(schema, plan.out, offs, n, stride=stride, stream=st, status=vst)
        rc = L.packos_get_batch(plan.out.data_ptr(), None if fixed else plan.offsets.data_ptr(), stride, n, path, 1,
                                3, 0, 0, gv.data_ptr(), 8, None, None, None, gst.data_ptr(),
                                C.c_void_p(st.cuda_stream))
        assert rc == 0, L.packos_last_error()
    replay(T, step)
    total = int(o0[n])
    assert np.array_equal(plan.out[:total].cpu().numpy(), a0)
    if not fixed:
        assert np.array_equal(plan.offsets.cpu().numpy().astype(np.uint64), o0)
    _, ost = ob.decode(cfg.chain, a0, o0, n, mode=cfg.mode)
    assert np.array_equal(dst.cpu().numpy().astype(np.uint32), ost[:n])
    assert np.array_equal(vst.cpu().numpy().astype(np.uint32), ob.validate(cfg.chain, a0, o0, n, mode=cfg.mode)[:n])
    ov, _, _, _, ogs = ob.get_batch(a0, o0, n, [0], 3)
    assert np.array_equal(gst.cpu().numpy(), ogs[:n])
    ok = ogs[:n] == 0
    assert np.array_equal(gv.cpu().numpy()[ok], ov[:n][ok])
