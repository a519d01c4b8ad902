#!/usr/bin/env python3
"""C3-shaped var encode whose label values overflow the tile encoder's
staging pool (every value past 16 B becomes a hole chunk): times the
library PACKOS_LIB points at (warm, median of reps, HIP events on the launch
stream) and checks the whole batch against the CPU oracle.  A/B tool for the
hole path of k_encode_tiles (VERDICT r5 Weak #11: the W = 6 build spills on
it).  Diagnostic only.
    PACKOS_LIB=abl/libpackos_x.so python tools/holes_bench.py [maxlen ...]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import oracle_bridge as ob  # noqa: E402
from packos_amd import _lib  # noqa: E402
from packos_amd.api import CompiledSchema, DeviceColumns, EncodePlan  # noqa: E402
from packos_amd.configs import CHAIN_C3, algorithmic_bytes, fixed_columns, splitmix64  # noqa: E402


def main():
    import torch
    torch.cuda.init()
    n = 1 << 20
    L = _lib.lib()
    for span in [int(x) for x in sys.argv[1:]] or [33, 96, 200]:
        r = splitmix64(0xC3C3 ^ span, n)
        hc = fixed_columns(CHAIN_C3, n, 0x5EED0003, {4: (8 + (r % np.uint64(span))).astype(np.uint32)})
        s = CompiledSchema(CHAIN_C3)
        plan = EncodePlan(s, DeviceColumns.from_host(s, hc, "cuda:0"))
        st = torch.cuda.current_stream()
        plan.run()
        torch.cuda.synchronize()
        enc = L.packos_last_encoder().decode()
        ts = []
        for _ in range(20):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            plan.run()
            b.record(st)
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        ms = float(np.median(ts))
        a0, o0, _ = ob.encode(CHAIN_C3, hc, 0, nthreads=16)
        tot = int(o0[n])
        same = np.array_equal(plan.out[:tot].cpu().numpy(), a0) and np.array_equal(
            plan.offsets.cpu().numpy().astype(np.uint64), o0)
        alg = algorithmic_bytes(hc, tot, True)
        print(f"labels 8..{7 + span} B: mean blob {tot / n:.1f} B, kernel {enc}, {ms:.4f} ms, "
              f"{alg / ms / 1e9:.3f} TB/s = {alg / ms / 8e9:.3f} of 8 TB/s, parity {'bit-exact' if same else 'DIFF'}",
              flush=True)


if __name__ == "__main__":
    main()
