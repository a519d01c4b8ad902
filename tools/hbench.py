#!/usr/bin/env python3
"""Host -> host encode rate through packos_encode_host_batch (pinned inputs and
outputs, chunked H2D / encode / D2H on two streams), per config.
    python tools/hbench.py [M C3 C5] [--chunk N]"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from packos_amd.api import CompiledSchema, encode_host_batch, host_batch_bound  # noqa: E402
from packos_amd.configs import CONFIGS, make_columns  # noqa: E402

SIZES = {"M": 1 << 20, "C3": 1 << 20, "C5": 1 << 20, "C2": 1 << 20, "C4": 1 << 21}


def pinned(a):
    return torch.from_numpy(np.ascontiguousarray(a)).pin_memory().numpy()


args = [a for a in sys.argv[1:] if not a.startswith("--")]
chunk = int(sys.argv[sys.argv.index("--chunk") + 1]) if "--chunk" in sys.argv else 0
torch.cuda.set_device(0)
for name in args or ["M", "C3", "C5"]:
    cfg = CONFIGS[name]
    n = SIZES[name]
    hc = make_columns(cfg, n=n)
    for lst in (hc.data, hc.offsets, hc.valid):
        for c, a in enumerate(lst):
            if a is not None:
                lst[c] = pinned(a)
    s = CompiledSchema(cfg.chain, cfg.mode)
    out = pinned(np.empty(host_batch_bound(s, hc), dtype=np.uint8))
    offs = pinned(np.empty(n + 1, dtype=np.uint64))
    st = pinned(np.empty(n, dtype=np.uint32))
    for c in ([chunk] if chunk else [1 << 17, 1 << 18, 1 << 19]):
        encode_host_batch(s, hc, chunk_blobs=c, out=out, offsets=offs, status=st)   # warm-up
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            a, o, _ = encode_host_batch(s, hc, chunk_blobs=c, out=out, offsets=offs, status=st)
            ts.append(time.perf_counter() - t0)
        el = float(np.median(ts))
        inb = sum(x.nbytes for lst in (hc.data, hc.offsets, hc.valid) for x in lst if x is not None)
        print(json.dumps({"config": name, "n": n, "chunk": c, "ms": round(el * 1e3, 3),
                          "million_blobs_per_s": round(n / el / 1e6, 2),
                          "gib_per_s_out": round(int(o[n]) / el / 2 ** 30, 2),
                          "gib_per_s_in_plus_out": round((inb + int(o[n])) / el / 2 ** 30, 2),
                          "note": "pinned host columns -> packos_encode_host_batch -> pinned host arena"}),
              flush=True)
