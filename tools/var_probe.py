#!/usr/bin/env python3
"""Phase timing of the tiled var encode (debug: PACKOS_VAR_PROF prints
per-block s_memtime cycles per phase to stderr)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from packos_amd.api import CompiledSchema, DeviceColumns, encode_batch  # noqa: E402
from packos_amd.configs import CONFIGS, make_columns  # noqa: E402

for name, n in (("C3", 1 << 20), ("C5", 1 << 20)):
    cfg = CONFIGS[name]
    hc = make_columns(cfg, n=n)
    s = CompiledSchema(cfg.chain, cfg.mode)
    dc = DeviceColumns.from_host(s, hc, "cuda:0")
    r = encode_batch(s, dc)
    torch.cuda.synchronize()
    for vt in ("64", "128", "256"):
        os.environ["PACKOS_VAR_TILE"] = vt
        os.environ["PACKOS_VAR_PROF"] = "1"
        print(name, "VT", vt, file=sys.stderr, flush=True)
        encode_batch(s, dc, out=r.arena)
        torch.cuda.synchronize()
        del os.environ["PACKOS_VAR_PROF"]
