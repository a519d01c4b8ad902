#!/usr/bin/env python3
"""Per-config GPU vs CPU rates: for every BASELINE config,
device-resident encode (EncodePlan replay: for var schemas the size kernel +
the encode kernel) and decode (DecodeBuffer semantics) on cuda:0, the CPU oracle
(C restatement of the reference, 'port') on the host cores over a bounded
sample, the speed-ups, and for var configs a chunked pinned
H2D + encode + D2H rate.  One JSON line per config.

    python tools/config_bench.py [C1 C2 C3 C4 C5 M] [--cpu-seconds S]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from packos_amd.api import CompiledSchema, DeviceColumns, EncodePlan, decode_batch, DecodedColumns  # noqa: E402
from packos_amd.configs import CONFIGS, algorithmic_bytes, make_columns  # noqa: E402
import oracle_bridge as ob  # noqa: E402  (CPU baseline only)

GPU_N = {"C1": 1000, "C2": 1 << 20, "C3": 1 << 20, "C4": 1 << 22, "C5": 1 << 21, "M": 1 << 20}


def tmed(fn, reps, group=10):
    """Median over `reps` groups of `group` back-to-back calls, one HIP event
    pair per group (a timing event record costs ~9 us of GPU time on the box,
    tools/hostcost.py — one pair per call would inflate short kernels)."""
    st = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(group):
            fn()
        b.record(st)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / group)
    return float(np.median(ts))


def cpu_rates(cfg, n, seconds):
    """Oracle encode and decode, threads = min(16, cores), bounded passes."""
    th = max(1, min(16, os.cpu_count() or 1))
    hc = make_columns(cfg, n=n)
    arena, offs, _ = ob.encode(cfg.chain, hc, cfg.mode, nthreads=th)
    os_ = ob.OracleSchema(cfg.chain)
    keep = []
    cols = ob.make_cols(hc, keep)
    out_a = np.empty_like(arena)
    out_o = np.empty_like(offs)
    res = {}
    passes, t0 = 0, time.perf_counter()
    while True:
        ob.lib().or_encode_batch(ob.C.byref(os_.s), cols, n, cfg.mode, out_a.ctypes.data, out_a.size,
                                 out_o.ctypes.data, None, th)
        passes += 1
        if time.perf_counter() - t0 >= seconds:
            break
    res["encode"] = passes * n / (time.perf_counter() - t0)
    passes, t0 = 0, time.perf_counter()
    while True:
        ob.decode(cfg.chain, arena, offs, n, nthreads=th)
        passes += 1
        if time.perf_counter() - t0 >= seconds:
            break
    res["decode"] = passes * n / (time.perf_counter() - t0)
    res["threads"] = th
    res["sample"] = n
    return res


def e2e_var(schema, hc, plan_total, reps=1):
    """Chunked pinned H2D (columns) + size kernel + encode kernel + D2H (arena),
    two streams double-buffered.  Offsets per chunk come from the size kernel;
    the D2H byte count from the host-side layout (flat chains: base + var)."""
    from packos_amd import _lib
    L = _lib.lib()
    n = hc.n
    nch = 8
    chunk = (n + nch - 1) // nch
    specs = schema.specs
    base = schema.all_present_size()
    widths = hc.var_widths().astype(np.int64)
    sizes = base + widths.sum(axis=1) if widths.size else np.full(n, base, np.int64)
    boff = np.concatenate([[0], np.cumsum(sizes)])
    pin = []
    for c, sp in enumerate(specs):
        pin.append(None if hc.data[c] is None else torch.from_numpy(hc.data[c]).pin_memory())
    out_host = torch.empty(int(boff[-1]), dtype=torch.uint8).pin_memory()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    dev = torch.device("cuda", 0)
    # per-chunk rebased var offsets (pinned)
    chunk_offs = []
    for s0 in range(0, n, chunk):
        m = min(chunk, n - s0)
        co = []
        for c, sp in enumerate(specs):
            if sp.var:
                o = hc.offsets[c][s0:s0 + m + 1].astype(np.int64)
                co.append(torch.from_numpy((o - o[0]).astype(np.uint32)).pin_memory())
            else:
                co.append(None)
        chunk_offs.append(co)
    maxvar = [0] * len(specs)
    for c, sp in enumerate(specs):
        if sp.var:
            o = hc.offsets[c].astype(np.int64)
            maxvar[c] = max(int(o[min(s0 + chunk, n)] - o[s0]) for s0 in range(0, n, chunk))
    bufs = []
    for k in range(2):
        cols = []
        offs_d = []
        for c, sp in enumerate(specs):
            if sp.fixed:
                cols.append(torch.empty(chunk * sp.width, dtype=torch.uint8, device=dev))
                offs_d.append(None)
            elif sp.var:
                cols.append(torch.empty(max(maxvar[c], 16), dtype=torch.uint8, device=dev))
                offs_d.append(torch.empty(chunk + 1, dtype=torch.int32, device=dev))
            else:
                cols.append(None)
                offs_d.append(None)
        outd = torch.empty(int(max(boff[min(s0 + chunk, n)] - boff[s0] for s0 in range(0, n, chunk))) + 16,
                           dtype=torch.uint8, device=dev)
        od = torch.empty(chunk + 1, dtype=torch.int64, device=dev)
        wsb = L.packos_encode_workspace_size(schema.handle, chunk)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        bufs.append((cols, offs_d, outd, od, ws, wsb))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        for j, s0 in enumerate(range(0, n, chunk)):
            k = j % 2
            m = min(chunk, n - s0)
            st = streams[k]
            cols, offs_d, outd, od, ws, wsb = bufs[k]
            with torch.cuda.stream(st):
                for c, sp in enumerate(specs):
                    if sp.fixed:
                        cols[c][: m * sp.width].copy_(pin[c][s0 * sp.width:(s0 + m) * sp.width], non_blocking=True)
                    elif sp.var:
                        o = hc.offsets[c]
                        a, b = int(o[s0]), int(o[s0 + m])
                        cols[c][: b - a].copy_(pin[c][a:b], non_blocking=True)
                        offs_d[c][: m + 1].copy_(chunk_offs[j][c].view(torch.int32), non_blocking=True)
                dc = DeviceColumns(schema, m, cols, offs_d, [None] * len(cols))
                arr = dc.ctypes_array()
                sp_ = st.cuda_stream
                L.packos_encode_batch(schema.handle, arr, m, outd.data_ptr(), outd.numel(), od.data_ptr(), None,
                                      ws.data_ptr(), wsb, 0, sp_)
                nb = int(boff[s0 + m] - boff[s0])
                out_host[int(boff[s0]):int(boff[s0]) + nb].copy_(outd[:nb], non_blocking=True)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / reps
    ok = bool(int(boff[-1]) == plan_total)
    return {"million_blobs_per_s": round(n / el / 1e6, 3), "gib_per_s_out": round(int(boff[-1]) / el / 2 ** 30, 3),
            "chunks": nch, "size_check": ok, "note": "pinned H2D + size kernel + encode kernel + D2H, 2 streams"}, out_host


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["C1", "C2", "C3", "C4", "C5", "M"])
    ap.add_argument("--cpu-seconds", type=float, default=3.0)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    for name in args.configs:
        cfg = CONFIGS[name]
        n = GPU_N[name]
        hc = make_columns(cfg, n=n)
        s = CompiledSchema(cfg.chain, cfg.mode)
        dc = DeviceColumns.from_host(s, hc, "cuda:0")
        plan = EncodePlan(s, dc, stream=torch.cuda.current_stream())
        plan.run()
        torch.cuda.synchronize()
        fixed = plan.fixed
        enc_ms = tmed(plan.run, args.reps)
        enc_ms1 = tmed(plan.run, args.reps, group=1)
        alg_enc = algorithmic_bytes(hc, plan.total, with_offsets=not fixed)
        offs = plan.offsets
        stride = 0 if offs is not None else s.fixed_blob_size
        out = DecodedColumns(s, n, torch.device("cuda", 0))
        st = torch.empty(n, dtype=torch.int32, device="cuda:0")
        decode_batch(s, plan.out, offs, n, stride=stride, out=out, status=st)
        torch.cuda.synchronize()
        bad = int((st != 0).sum().item())
        dec_ms = tmed(lambda: decode_batch(s, plan.out, offs, n, stride=stride, out=out, status=st), args.reps)
        dec_ms1 = tmed(lambda: decode_batch(s, plan.out, offs, n, stride=stride, out=out, status=st), args.reps,
                       group=1)
        vals = sum(n * sp.width for sp in s.specs if sp.fixed) + sum(12 * n for sp in s.specs if sp.var)
        # var values are returned as (start, length) views into the arena
        # (GetBytes / GetStringUnsafe aliasing): their bytes are never read
        var_bytes = sum(int(hc.offsets[c][-1]) for c, sp in enumerate(hc.specs) if sp.var)
        alg_dec = plan.total - var_bytes + (8 * n if offs is not None else 0) + vals + 4 * n
        cpu = cpu_rates(cfg, min(n, 1 << 18 if name != "C5" else 1 << 16), args.cpu_seconds)
        g_enc = n / enc_ms / 1e3
        g_dec = n / dec_ms / 1e3
        line = {"config": name, "note": cfg.note, "n_gpu": n, "blob_bytes_mean": round(plan.total / n, 1),
                "encode": {"ms": round(enc_ms, 4), "ms_one_event_pair_per_call": round(enc_ms1, 4),
                           "million_blobs_per_s": round(g_enc, 2),
                           "GBps_algorithmic": round(alg_enc / enc_ms / 1e6, 1),
                           "roofline_frac": round(alg_enc / enc_ms / 1e6 / 8000.0, 4),
                           "includes": "encode" if fixed else "size kernel (closed-form map or look-back scan) + encode kernel"},
                "decode": {"ms": round(dec_ms, 4), "ms_one_event_pair_per_call": round(dec_ms1, 4),
                           "million_blobs_per_s": round(g_dec, 2),
                           "GBps_algorithmic": round(alg_dec / dec_ms / 1e6, 1),
                           "fast_path": s.decode_fast, "nonzero_status": bad},
                "cpu_oracle": {"encode_million_blobs_per_s": round(cpu["encode"] / 1e6, 3),
                               "decode_million_blobs_per_s": round(cpu["decode"] / 1e6, 3),
                               "threads": cpu["threads"], "sample_blobs": cpu["sample"], "kind": "port"},
                "speedup": {"encode": round(g_enc * 1e6 / cpu["encode"], 1),
                            "decode": round(g_dec * 1e6 / cpu["decode"], 1)}}
        if not fixed and name in ("C5", "C3"):
            e2e, host = e2e_var(s, hc, plan.total)
            ref = plan.out[: plan.total].cpu()
            e2e["bytes_equal_device_encode"] = bool(torch.equal(host, ref))
            line["e2e_pinned"] = e2e
        print(json.dumps(line), flush=True)
        del dc, plan, out, st
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
