#!/usr/bin/env python3
"""Debug: first mismatching ranges of the stream encoder vs the oracle for one
random schema seed (tests/schema_gen.py)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_bridge as ob  # noqa: E402
from packos_amd.api import CompiledSchema, DeviceColumns, encode_batch  # noqa: E402
from packos_amd.columns import HostColumns  # noqa: E402
from schema_gen import rand_chain, rand_rows  # noqa: E402
import torch  # noqa: E402

seed, mode = int(sys.argv[1]), int(sys.argv[2])
chain = rand_chain(seed)
hc = HostColumns.from_rows(chain, rand_rows(chain, 257 + 300 * (seed % 3), seed * 7 + 1))
a0, o0, s0 = ob.encode(chain, hc, mode, nthreads=8)
s = CompiledSchema(chain, mode)
dc = DeviceColumns.from_host(s, hc, "cuda:0")
r = encode_batch(s, dc)
torch.cuda.synchronize()
a1 = r.arena[: r.total].cpu().numpy()
bad = np.nonzero(a0 != a1)[0]
print("n", hc.n, "total", a0.size, "mismatches", bad.size)
if bad.size:
    runs = np.split(bad, np.nonzero(np.diff(bad) != 1)[0] + 1)
    for rr in runs[:12]:
        b = int(rr[0])
        blob = int(np.searchsorted(o0, b, side="right") - 1)
        print(f"bytes {b}..{int(rr[-1])} ({rr.size}) blob {blob} +{b - int(o0[blob])} blob size {int(o0[blob+1]-o0[blob])}"
              f" exp {a0[b:b+8].tobytes().hex()} got {a1[b:b+8].tobytes().hex()}")
