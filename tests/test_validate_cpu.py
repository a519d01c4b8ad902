"""ValidateBuffer's oracle on CPU: the mutation sweep of test_gpu_validate.py
reaches all three places where the Validate methods' rules differ from
Decode's (schema/schema.go:596-715 payload reads, :1085-1087 nullable-empty
checks, :336-359 odd SMap), so the GPU sweep over the same batches covers them."""
import numpy as np

import oracle_bridge as ob
from test_gpu_validate import _divergence_batch


def test_validate_mutations_reach_every_divergence():
    seen = set()
    for seed in range(40):
        mchain, arena, offs, n = _divergence_batch(seed)
        v = ob.validate(mchain, arena, offs, n, nthreads=8)
        d = ob.decode(mchain, arena, offs, n, nthreads=8)[1]
        diff = (v != d)
        for dv in d[diff]:
            code = int(dv) & 0xFF
            if int(dv) & 0x40000000:
                seen.add("panic")
            elif code in (6, 7, 9):
                seen.add("check")
            elif code in (1, 3):
                seen.add("struct")
    assert {"panic", "check", "struct"} <= seen, seen
