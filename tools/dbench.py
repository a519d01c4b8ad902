#!/usr/bin/env python3
"""Decode timings (DecodeBuffer semantics) per config, HIP-event median."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from packos_amd.api import CompiledSchema, DeviceColumns, decode_batch, encode_batch  # noqa: E402
from packos_amd.configs import CONFIGS, make_columns  # noqa: E402

SIZES = {"C2": 1 << 20, "C3": 1 << 20, "C4": 1 << 22, "C5": 1 << 21, "M": 1 << 20}


def tmed(fn, reps=20):
    st = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        fn()
        b.record(st)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts))


for name in sys.argv[1:] or ["M", "C2", "C4", "C3"]:
    cfg = CONFIGS[name]
    n = SIZES[name]
    hc = make_columns(cfg, n=n)
    s = CompiledSchema(cfg.chain, cfg.mode)
    dc = DeviceColumns.from_host(s, hc, "cuda:0")
    r = encode_batch(s, dc)
    torch.cuda.synchronize()
    offs = r.offsets if r.offsets is not None else torch.arange(n + 1, device="cuda:0", dtype=torch.int64) * s.fixed_blob_size
    out, st = decode_batch(s, r.arena, offs, n)
    torch.cuda.synchronize()
    bad = int((st != 0).sum().item())
    ms = tmed(lambda: decode_batch(s, r.arena, offs, n, out=out, status=st))
    vals = sum(n * sp.width for sp in s.specs if sp.fixed) + sum(12 * n for sp in s.specs if sp.var)
    # var values come back as views into the arena: their bytes are not read
    var_bytes = sum(int(hc.offsets[c][-1]) for c, sp in enumerate(hc.specs) if sp.var)
    alg = r.total - var_bytes + 8 * n + vals + 4 * n
    extra = {}
    if r.offsets is None:   # fixed-size batch: also by stride (no offsets array)
        extra["decode_stride_ms"] = round(tmed(lambda: decode_batch(s, r.arena, None, n, out=out, status=st,
                                                                    stride=s.fixed_blob_size)), 4)
    print(json.dumps({"config": name, "n": n, **extra, "decode_ms": round(ms, 4), "GBs": round(alg / ms / 1e6, 1),
                      "frac": round(alg / ms / 1e6 / 8000, 4), "fast": s.decode_fast, "bad_status": bad}), flush=True)
