#!/usr/bin/env python3
"""Var-size encode A/B: k_stream_sizes + k_encode_stream (EncodePlan.run, one call)
vs the two-kernel tiled encoder (PACKOS_VAR_KERNEL=tile: size pass + scan +
tile kernel), same process, interleaved; outputs must be byte-equal.

    python tools/sbench.py [C3 C5 ...]     env knobs pass through (PACKOS_STREAM_*)
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from packos_amd.api import CompiledSchema, DeviceColumns, EncodePlan  # noqa: E402
from packos_amd.configs import CONFIGS, algorithmic_bytes, make_columns  # noqa: E402

SIZES = {"C3": 1 << 20, "C5": 1 << 21}


def tone(fn):
    st = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    fn()
    b.record(st)
    torch.cuda.synchronize()
    return a.elapsed_time(b)


def main():
    names = sys.argv[1:] or ["C3", "C5"]
    reps = int(os.environ.get("SB_REPS", "20"))
    for name in names:
        cfg = CONFIGS[name]
        n = SIZES.get(name, 1 << 20)
        hc = make_columns(cfg, n=n)
        s = CompiledSchema(cfg.chain, cfg.mode)
        dc = DeviceColumns.from_host(s, hc, "cuda:0")
        p = EncodePlan(s, dc, want_status=True)
        p.run()
        torch.cuda.synchronize()
        a_stream = p.out[: p.total].clone()
        o_stream = p.offsets.clone()

        def run_tile():
            os.environ["PACKOS_VAR_KERNEL"] = "tile"
            from packos_amd import _lib
            L = _lib.lib()
            st = torch.cuda.current_stream().cuda_stream
            L.packos_encoded_size_batch(s.handle, p._arr, n, p.offsets.data_ptr(), p.ws.data_ptr(), p.wsb, st)
            L.packos_encode_batch(s.handle, p._arr, n, p.out.data_ptr(), p.out.numel(), p.offsets.data_ptr(),
                                  p.status.data_ptr(), p.ws.data_ptr(), p.wsb, _lib.ENC_OFFSETS_READY, st)
            del os.environ["PACKOS_VAR_KERNEL"]

        run_tile()
        torch.cuda.synchronize()
        same = bool(torch.equal(p.out[: p.total], a_stream)) and bool(torch.equal(p.offsets, o_stream))
        ts, tt = [], []
        for _ in range(reps):
            ts.append(tone(p.run))
            tt.append(tone(run_tile))
        alg = algorithmic_bytes(hc, p.total, True)
        ms_s, ms_t = float(np.median(ts)), float(np.median(tt))
        from packos_amd import _lib

        def run_ready():
            _lib.lib().packos_encode_batch(s.handle, p._arr, n, p.out.data_ptr(), p.out.numel(),
                                           p.offsets.data_ptr(), p.status.data_ptr(), p.ws.data_ptr(), p.wsb,
                                           _lib.ENC_OFFSETS_READY, torch.cuda.current_stream().cuda_stream)
        tr = [tone(run_ready) for _ in range(reps)]
        extra = {"stream_ready_ms": round(float(np.median(tr)), 4)}
        for k in os.environ.get("SB_VARY", "").split(";"):
            if not k:
                continue
            kv = [x.split("=") for x in k.split(",")]
            saved = {var: os.environ.get(var) for var, _ in kv}
            for var, val in kv:
                os.environ[var] = val
            extra[k + "_ms"] = round(float(np.median([tone(p.run) for _ in range(reps)])), 4)
            for var, old in saved.items():
                if old is None:
                    del os.environ[var]
                else:
                    os.environ[var] = old
        if os.environ.get("SB_PROF"):
            os.environ["PACKOS_STREAM_PROF"] = "1"
            p.run()
            torch.cuda.synchronize()
            del os.environ["PACKOS_STREAM_PROF"]
        print(json.dumps({"config": name, "n": n, "total_out": p.total, "same_bytes": same, **extra,
                          "stream_ms": round(ms_s, 4), "tile_ms": round(ms_t, 4),
                          "stream_GBs": round(alg / ms_s / 1e6, 1), "tile_GBs": round(alg / ms_t / 1e6, 1),
                          "stream_frac": round(alg / ms_s / 1e6 / 8000, 4)}), flush=True)


if __name__ == "__main__":
    main()
