"""k_encode_tiles with a staging pool sized from the exact capacity (closed-form
chains whose var bytes per blob overflow the default 40-B pool; kernels.hip,
the dispatch after the six-workgroup choice) vs the CPU oracle, bit-exact:
C3's chain with longer labels, heavy-tailed labels (most tiles fit the sized
pool, some overflow it and take the hole path), two var columns, and the
same batches through `encode_batch` (exact capacity) and an oversized
`EncodePlan` arena (no exact capacity: the default pool)."""
import numpy as np
import pytest

import oracle_bridge as ob
from packos_amd import _lib
from packos_amd.api import CompiledSchema, DeviceColumns, EncodePlan, encode_batch
from packos_amd.configs import CHAIN_C3, fixed_columns, splitmix64
from packos_amd.schema import SChain, SInt32, SInt64, SVariableBytes, SVariableString

pytestmark = pytest.mark.gpu


def torch():
    import torch as t
    return t


def check(chain, hc, out, offsets):
    a0, o0, _ = ob.encode(chain, hc, 0, nthreads=8)
    tot = int(o0[hc.n])
    assert np.array_equal(offsets.cpu().numpy().astype(np.uint64), o0)
    assert np.array_equal(out[:tot].cpu().numpy(), a0)


def label_lengths(n, span, tail):
    r = splitmix64(0xC3C3 ^ span, n)
    ln = (8 + (r % np.uint64(span))).astype(np.uint32)
    if tail:   # every 37th label 600-1100 B: a few tiles overflow any pool
        ln[::37] = (600 + (r[::37] % np.uint64(500))).astype(np.uint32)
    return ln


@pytest.mark.parametrize("span,tail", [(40, False), (70, False), (110, False), (160, False), (220, False),
                                       (110, True), (30, True)])
def test_sized_pool_c3_labels(span, tail):
    T = torch()
    n = 20000 + 37
    hc = fixed_columns(CHAIN_C3, n, 0x5EED0003, {4: label_lengths(n, span, tail)})
    s = CompiledSchema(CHAIN_C3)
    dc = DeviceColumns.from_host(s, hc, "cuda:0")
    plan = EncodePlan(s, dc)
    plan.run()
    T.cuda.synchronize()
    assert _lib.lib().packos_last_encoder().decode() in ("tiles", "tiles6", "flat")
    check(CHAIN_C3, hc, plan.out, plan.offsets)
    r = encode_batch(s, dc)
    T.cuda.synchronize()
    check(CHAIN_C3, hc, r.arena, r.offsets)
    # no exact capacity (an oversized arena): the default pool, holes
    big = T.empty(int(plan.out.numel()) * 2 + 4096, dtype=T.uint8, device="cuda:0")
    p2 = EncodePlan(s, dc, out=big)
    p2.run()
    T.cuda.synchronize()
    check(CHAIN_C3, hc, p2.out, p2.offsets)


@pytest.mark.parametrize("span", [50, 90])
def test_sized_pool_two_var_columns(span):
    T = torch()
    chain = SChain(SInt32, SVariableString(), SInt64, SVariableBytes())
    n = 9000
    r = splitmix64(0xBEEF ^ span, 2 * n)
    lens = {1: (r[:n] % np.uint64(span)).astype(np.uint32), 3: (r[n:] % np.uint64(span // 2 + 1)).astype(np.uint32)}
    hc = fixed_columns(chain, n, 0x5EED0099, lens)
    s = CompiledSchema(chain)
    plan = EncodePlan(s, DeviceColumns.from_host(s, hc, "cuda:0"))
    plan.run()
    T.cuda.synchronize()
    check(chain, hc, plan.out, plan.offsets)
