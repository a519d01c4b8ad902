#!/usr/bin/env python3
"""Encode (var path) and decode timings for the BASELINE configs (one process)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from packos_amd.api import CompiledSchema, DeviceColumns, decode_batch, encode_batch  # noqa: E402
from packos_amd.configs import CONFIGS, algorithmic_bytes, make_columns  # noqa: E402


def tmed(fn, reps=10):
    st = torch.cuda.current_stream()
    ts = []
    fn()
    torch.cuda.synchronize()
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        fn()
        b.record(st)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts))


def main():
    sizes = {"C3": 1 << 20, "C5": 1 << 21, "M": 1 << 20, "C4": 1 << 22, "C2": 1 << 20}
    names = sys.argv[1:] or ["C3", "C5", "M", "C4"]
    for name in names:
        cfg = CONFIGS[name]
        n = sizes[name]
        hc = make_columns(cfg, n=n)
        s = CompiledSchema(cfg.chain, cfg.mode)
        dc = DeviceColumns.from_host(s, hc, "cuda:0")
        r = encode_batch(s, dc, want_status=True)
        torch.cuda.synchronize()
        res = {"n": n, "total_out": r.total}
        fixed = s.fixed_blob_size > 0
        if not fixed:
            ms = tmed(lambda: encode_batch(s, dc, want_status=True, out=r.arena))
            alg = algorithmic_bytes(hc, r.total, True)
            res["encode_ms_incl_size_pass_and_sync"] = round(ms, 4)
            res["encode_GBs"] = round(alg / ms / 1e6, 1)
        offs = r.offsets if r.offsets is not None else torch.arange(n + 1, device="cuda:0", dtype=torch.int64) * s.fixed_blob_size
        out, st = decode_batch(s, r.arena, offs, n)
        torch.cuda.synchronize()
        res["decode_status_nonzero"] = int((st != 0).sum().item())
        res["decode_fast"] = s.decode_fast
        ms = tmed(lambda: decode_batch(s, r.arena, offs, n, out=out, status=st))
        vals = sum(n * sp.width for sp in s.specs if sp.fixed) + sum(12 * n for sp in s.specs if sp.var)
        alg = r.total + 8 * n + vals + 4 * n
        res["decode_ms"] = round(ms, 4)
        res["decode_GBs"] = round(alg / ms / 1e6, 1)
        if s.decode_fast:
            os.environ["PACKOS_DECODE_GENERIC"] = "1"
            ms_g = tmed(lambda: decode_batch(s, r.arena, offs, n, out=out, status=st))
            del os.environ["PACKOS_DECODE_GENERIC"]
            res["decode_generic_ms"] = round(ms_g, 4)
        print(json.dumps({name: res}), flush=True)


if __name__ == "__main__":
    main()
