#!/usr/bin/env python3
"""Interleaved A/B timing of encode kernel variants in ONE process
(cdna_hip_programming.md §5.4 rule 24).  Usage: python tools/kbench.py [M C2 C4 ...]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from packos_amd.api import CompiledSchema, DeviceColumns, EncodePlan  # noqa: E402
from packos_amd.configs import CONFIGS, algorithmic_bytes, make_columns  # noqa: E402

VARIANTS = {k: int(v) << 4 for k, v in (x.split("=") for x in os.environ.get(
    "KBENCH_VARIANTS", "v13=13,v2=2,v8=8").split(","))}
TILES = [int(x) for x in os.environ.get("KBENCH_TILES", "16384").split(",")]


def time_plan(plan, reps):
    st = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in evs:
        a.record(st)
        plan.run()
        b.record(st)
    torch.cuda.synchronize()
    return [a.elapsed_time(b) for a, b in evs]


def main():
    names = sys.argv[1:] or ["M", "C2", "C4"]
    res = {}
    for name in names:
        cfg = CONFIGS[name]
        n = cfg.n if name != "C4" else cfg.n
        hc = make_columns(cfg, n=n)
        plans = {}
        for tb in TILES:
            os.environ["PACKOS_TILE_BYTES"] = str(tb)
            s = CompiledSchema(cfg.chain, cfg.mode)
            dc = DeviceColumns.from_host(s, hc, "cuda:0")
            for k, f in VARIANTS.items():
                plans[f"{k}_t{tb // 1024}k"] = EncodePlan(s, dc, flags=f)
        first = next(iter(plans))
        for p in plans.values():
            p.run()
        torch.cuda.synchronize()
        outs = {k: p.out[: p.total].clone() for k, p in plans.items()}
        same = all(torch.equal(outs[first], o) for o in outs.values())
        times = {k: [] for k in plans}
        for _ in range(5):
            for k, p in plans.items():
                times[k] += time_plan(p, 20)
        alg = algorithmic_bytes(hc, plans[first].total, False)
        res[name] = {"same_output": same, "B": plans[first].B, "n": n}
        for k, t in times.items():
            med = float(np.median(t))
            res[name][k] = {"median_ms": round(med, 4), "min_ms": round(float(np.min(t)), 4),
                            "GBs": round(alg / med / 1e6, 1), "Mblobs_s": round(n / med / 1e3, 1)}
        print(json.dumps({name: res[name]}), flush=True)


if __name__ == "__main__":
    main()


def copy_ref(nbytes=256 << 20, reps=50):
    """torch D2D copy of nbytes: the practical read+write streaming ceiling."""
    a = torch.empty(nbytes, dtype=torch.uint8, device="cuda:0")
    b = torch.empty_like(a)
    b.copy_(a)
    st = torch.cuda.current_stream()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        b.copy_(a)
        e1.record(st)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    med = float(np.median(ts))
    print(json.dumps({"copy_ref": {"bytes_moved": 2 * nbytes, "median_ms": round(med, 4),
                                   "GBs": round(2 * nbytes / med / 1e6, 1)}}), flush=True)


if __name__ == "__main__" and os.environ.get("KBENCH_COPY", "1") == "1":
    copy_ref()
