#!/usr/bin/env python3
"""Host-side cost per encode launch (metric M): plan.run() alone, with two
event records, and the GPU time per step when launches are back to back."""
import json, os, sys, time
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from packos_amd.api import CompiledSchema, DeviceColumns, EncodePlan  # noqa
from packos_amd.configs import CONFIGS, make_columns  # noqa
from packos_amd import _lib  # noqa

cfg = CONFIGS["M"]
hc = make_columns(cfg, n=cfg.n)
s = CompiledSchema(cfg.chain, cfg.mode)
dc = DeviceColumns.from_host(s, hc, "cuda:0")
st = torch.cuda.current_stream()
plan = EncodePlan(s, dc, stream=st)
for _ in range(10): plan.run()
torch.cuda.synchronize()
res = {}
# host cost of a call into a tiny batch (GPU never the bottleneck)
dc_small = DeviceColumns.from_host(s, make_columns(cfg, n=64), "cuda:0")
small = EncodePlan(s, dc_small, stream=st)
for _ in range(100): small.run()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(2000): small.run()
res["host_us_per_run_small"] = (time.perf_counter() - t0) / 2000 * 1e6
torch.cuda.synchronize()
e = [torch.cuda.Event(enable_timing=True) for _ in range(4000)]
t0 = time.perf_counter()
for i in range(2000):
    e[2 * i].record(st); small.run(); e[2 * i + 1].record(st)
res["host_us_per_run_small_with_events"] = (time.perf_counter() - t0) / 2000 * 1e6
torch.cuda.synchronize()
# back-to-back M launches: wall per step, no events
for K in (50,):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(K): plan.run()
    torch.cuda.synchronize(); res["wall_us_per_step_noevents"] = (time.perf_counter() - t0) / K * 1e6
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for a, b in ev:
        a.record(st); plan.run(); b.record(st)
    torch.cuda.synchronize(); res["wall_us_per_step_events"] = (time.perf_counter() - t0) / K * 1e6
    res["event_us_mean"] = float(np.mean([a.elapsed_time(b) for a, b in ev])) * 1e3
    # one pair of events around K launches
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); a.record(st)
    for _ in range(K): plan.run()
    b.record(st); torch.cuda.synchronize()
    res["event_us_per_step_batched"] = a.elapsed_time(b) / K * 1e3
print(json.dumps({k: round(v, 2) for k, v in res.items()}))
