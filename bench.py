#!/usr/bin/env python3
"""Device-resident bulk PackOS encode throughput (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config M|C2|C3|C4|C5] [--sets S]

One step = one encode of this GPU's whole shard with its inputs already
resident in HBM (metric config M: 1M x 256 B fixed-schema tuples per GPU;
C5: one 8,388,608-blob shard of the 64M mixed batch).

Ranks: `--gpus N` (N > 1) with no launcher around it starts N rank processes
itself (a child `torch.distributed.run --nproc-per-node N` on this script,
before any GPU call; the parent waits and exits with the job's status); under
an external launcher every rank checks WORLD_SIZE == N and, under nccl
(RCCL), a distinct GPU per rank, and exits non-zero otherwise.

Batch and shards: the N ranks encode N disjoint contiguous shards of ONE
global synthetic batch of N x (blobs per GPU) blobs (weak scaling), planned
byte-balanced by packos_amd.shard.plan_shards; each rank generates exactly
its slice (the generator is indexed by global blob number).  There is no
collective on the data path: the only communication is the harness barrier
and the max-over-ranks timing all-reduce.

Cold vs warm: the timed loop rotates over S >= 3 device copies of the shard
(distinct input columns AND output arenas, > 750 MiB for M), so no set is
still resident in the 256 MiB Infinity Cache when it is reused; `value`,
`ms_per_step` and `roofline` are these cold figures.  A second loop replays
set 0 only ("warm", labelled).

Rank 0 at N=1 also times the CPU oracle (a C restatement of the reference
encoder, test infrastructure) on every host core over the same shard, and
checks the GPU arena of the timed run against it byte for byte (`parity`).
"""
import argparse
import hashlib
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md), GB/s


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", default="M")
    p.add_argument("--blobs-per-gpu", type=int, default=0, help="blobs per GPU (default: the config's shard)")
    p.add_argument("--sets", type=int, default=3, help="device copies rotated in the timed loop (cold)")
    p.add_argument("--passes", type=int, default=3,
                   help="timed cold passes (the headline is their median); warm passes interleave between them")
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline / parity leg")
    p.add_argument("--no-host", action="store_true", help="skip the host-resident library leg")
    p.add_argument("--no-warm", action="store_true", help="skip the warm (single-set) loop, e.g. for PMC passes")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--parity-piece", type=int, default=1 << 20, help="N > 1: blobs per piece of the shard parity check")
    p.add_argument("--op", default="encode", choices=["encode", "decode", "validate", "get"],
                   help="decode: schema.DecodeBuffer over the encoded shard; validate: schema.ValidateBuffer "
                        "(status only); get: GetAccess GetInt of top-level field --get-pos with the typed "
                        "gather (per-config tables, not the metric)")
    p.add_argument("--get-spans", action="store_true",
                   help="--op get: also write start / length / tag (GetInt itself returns only value + error)")
    p.add_argument("--get-pos", type=int, default=-1,
                   help="top-level field GetInt reads (default: the config's first int64 field)")
    return p.parse_args()


# ----------------------------------------------------------------- bytes
LINE = 128   # L2 cache line (bytes): the smallest unit a scattered read fetches


def lines_touched(a0, end, line=LINE):
    """Distinct `line`-byte lines covered by the ordered, disjoint byte windows
    [a0[i], end[i]) (empty windows skipped)."""
    a0 = np.asarray(a0, dtype=np.uint64)
    end = np.asarray(end, dtype=np.uint64)
    m = end > a0
    a0, end = a0[m], end[m]
    if a0.size == 0:
        return 0
    first = a0 // np.uint64(line)
    last = (end - np.uint64(1)) // np.uint64(line)
    return int((last - first + np.uint64(1)).sum()) - int(np.count_nonzero(first[1:] == last[:-1]))


def top_layout(chain):
    """(header bytes, [(kind, width) per top-level field]) of a flat chain;
    width 0 = variable."""
    fields = []
    for node in chain.Schemas:
        if node.kind in ("int", "uint", "float", "bool") or (node.kind in ("string", "bytes", "match")):
            fields.append((node.kind, node.width if node.width and node.width > 0 else 0))
        else:
            fields.append((node.kind, -1))   # container
    return 2 * (len(fields) + 1), fields


def static_prefix(chain):
    """Bytes of a flat blob before its first variable payload (header block +
    the fixed fields in front), and whether any fixed payload follows a var
    one; None for chains with containers."""
    H, fields = top_layout(chain)
    if any(w < 0 for _, w in fields):
        return None, True
    pre, seen_var, tail_fixed = H, False, False
    for _, w in fields:
        if w == 0:
            seen_var = True
        elif seen_var:
            tail_fixed = True
        else:
            pre += w
    return pre, tail_fixed


def validate_reads(chain, mode):
    """(bytes ValidateBuffer reads per all-present blob, window): the header
    blocks, Match literals and Range / date / prefix / suffix payloads
    (schema.go:880-891 over the Validate methods), and the leading bytes that
    hold all of them when none follows a var payload (else None) - the
    packos_schema val_win rule of compile.cpp."""
    from packos_amd.schema import CHK_DATE, CHK_MAX, CHK_MIN, CHK_PREFIX, CHK_SUFFIX
    st = {"pos": 0, "need": 0, "var": False, "after": False, "bytes": 0}

    def item(size, reads, var=False):
        if var:
            st["var"] = True
        if reads:
            st["bytes"] += size
            if st["var"]:
                st["after"] = True
        if not st["var"]:
            st["pos"] += size
            if reads:
                st["need"] = st["pos"]

    def container(kids):
        item(2 * (len(kids) + 1) if kids else (2 if mode == 0 else 0), True)
        for k in kids:
            node(k)

    def node(x):
        if x.kind in ("tuple", "map"):
            container(x.ordered_children())
        elif x.kind == "match":
            item(len(x.literal), True)
        elif x.kind in ("string", "bytes") and x.width <= 0:
            item(0, bool(x.check & (CHK_PREFIX | CHK_SUFFIX)), var=True)
        else:
            item(x.width, bool(x.check & (CHK_MIN | CHK_MAX | CHK_DATE | CHK_PREFIX | CHK_SUFFIX)))
    container(list(chain.Schemas))
    return st["bytes"], (None if st["after"] else st["need"])


def first_int64(chain):
    for j, node in enumerate(chain.Schemas):
        if node.kind == "int" and node.width == 8:
            return j
    return 0


# ----------------------------------------------------------------- provenance
PRODUCT_FILES = ("packos_amd/csrc", "include/packos.h", "__graft_entry__.py")


def product_tree_hash():
    """sha256 (16 hex) over the product sources libpackos.so is built from
    (packos_amd/csrc/*, include/packos.h, the build line in __graft_entry__.py):
    a PMC summary measured on a tree with the same hash measured this code."""
    h = hashlib.sha256()
    for rel in PRODUCT_FILES:
        path = os.path.join(ROOT, rel)
        files = sorted(os.path.join(path, f) for f in os.listdir(path)) if os.path.isdir(path) else [path]
        for f in files:
            if os.path.isfile(f):
                h.update(os.path.relpath(f, ROOT).encode() + b"\0")
                with open(f, "rb") as fh:
                    h.update(fh.read())
    return h.hexdigest()[:16]


def pmc_traffic(config, op):
    """HBM bytes per launch from bench_pmc/pmc_<config>[_<op>].json (separate
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this bench command,
    summarised by tools/pmc_summary.py), reported only when that summary's
    product-tree hash equals this tree's."""
    name = f"pmc_{config}.json" if op == "encode" else f"pmc_{config}_{op}.json"
    path = os.path.join(ROOT, "bench_pmc", name)
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        pmc = json.load(f)
    here = product_tree_hash()
    if pmc.get("product_tree") != here:
        return None, f"bench_pmc/{name} is stale: product tree {pmc.get('product_tree')} != this tree's {here}"
    return pmc.get("hbm_bytes_per_launch"), (
        f"bench_pmc/{name}: rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + WRITE_SIZE of kernel {pmc.get('kernel', '?')[:60]}, "
        f"measured at commit {pmc.get('commit', '?')} on product tree {here} (= this tree's); "
        f"traffic / algorithmic = {pmc.get('traffic_over_algorithmic')}")


# ----------------------------------------------------------------- host info
def host_info():
    info = {"nproc": os.cpu_count() or 1}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except Exception:
        info["affinity"] = None
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except Exception:
        pass
    info["cpu_model"] = model or platform.processor() or "unknown"
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as f:
                q, per = f.read().split()[:2]
            if q != "max":
                quota = round(int(q) / int(per), 2)
        except Exception:
            pass
    info["cgroup_cpu_quota"] = quota
    return info


def cpu_leg(cfg, hc, seconds, gpu_arena, gpu_offsets):
    """CPU oracle ('port') timed on this host's cores over the same shard
    (bounded: `seconds` of all-core passes, half that single-threaded), and
    the bit-exact comparison of the GPU output with the oracle's."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_bridge as ob  # checker / baseline only
    hi = host_info()
    aff = max(1, min(1024, hi["affinity"] or hi["nproc"]))
    quota = hi["cgroup_cpu_quota"]
    eff = max(1, min(aff, int(quota))) if quota else aff   # CPUs this process can actually keep busy
    hi["effective_cpus"] = eff
    cap = max(1, hc.n // 4096)   # >= 4096 blobs per thread (C1's 1k blobs: one)
    cands = sorted({min(eff, cap), min(aff, cap)})
    os_ = ob.OracleSchema(cfg.chain)
    keep = []
    cols = ob.make_cols(hc, keep)
    n = hc.n
    total = int(gpu_offsets[n]) if gpu_offsets is not None else len(gpu_arena)
    arena = np.empty(max(total, 1), np.uint8)
    offs = np.empty(n + 1, np.uint64)
    res = {}
    legs = [(f"mt{th}", th) for th in cands] + [("st", 1)]
    for label, th in legs:
        passes, t0 = 0, time.perf_counter()
        budget = seconds / len(cands) if label != "st" else seconds / 2
        while True:
            r = ob.lib().or_encode_batch(ob.C.byref(os_.s), cols, n, cfg.mode, arena.ctypes.data, arena.size,
                                         offs.ctypes.data, None, th)
            assert r == total, (r, total)
            passes += 1
            el = time.perf_counter() - t0
            if el >= budget:
                break
        res[label] = (passes * n / el, passes, el, th)
    res["mt"] = max((v for k, v in res.items() if k.startswith("mt")), key=lambda v: v[0])
    res["tried"] = {v[3]: round(v[0] / 1e6, 3) for k, v in res.items() if k.startswith("mt")}
    same = bool(np.array_equal(arena[:total], gpu_arena[:total]))
    if gpu_offsets is not None:
        same = same and bool(np.array_equal(offs, gpu_offsets.astype(np.uint64)))
    digest = hashlib.sha256(gpu_arena[:total].tobytes()).hexdigest()[:16]
    return res, hi, same, digest, total


def shard_parity(cfg, hc, out_dev, offs_dev, blob_size, threads, piece=1 << 20):
    """This rank's whole shard vs the CPU oracle, piece by piece (a C5 shard
    is 8 GB: each piece's GPU bytes come to the host, the oracle encodes the
    same rows, compare, free).  Returns (same, checked blobs, digest)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_bridge as ob  # checker only
    from packos_amd.shard import slice_columns
    n = hc.n
    offs_all = None if offs_dev is None else offs_dev[: n + 1].cpu().numpy().astype(np.uint64)
    h = hashlib.sha256()
    same, checked = True, 0
    for a in range(0, n, piece):
        b = min(n, a + piece)
        if offs_all is not None:
            a0, b0 = int(offs_all[a]), int(offs_all[b])
        else:
            a0, b0 = a * blob_size, b * blob_size
        g = out_dev[a0:b0].cpu().numpy()
        sub = slice_columns(hc, a, b)
        os_ = ob.OracleSchema(cfg.chain)
        keep = []
        cols = ob.make_cols(sub, keep)
        arena = np.empty(max(b0 - a0, 1), np.uint8)
        offs = np.empty(b - a + 1, np.uint64)
        r = ob.lib().or_encode_batch(ob.C.byref(os_.s), cols, b - a, cfg.mode, arena.ctypes.data, arena.size,
                                     offs.ctypes.data, None, threads)
        same = same and r == b0 - a0 and bool(np.array_equal(arena[: b0 - a0], g))
        if offs_all is not None:
            same = same and bool(np.array_equal(offs, offs_all[a: b + 1] - np.uint64(a0)))
        h.update(g.tobytes())
        checked += b - a
        del g, arena, sub, keep
    return same, checked, h.hexdigest()[:16]


def decode_parity(cfg, arena, offsets, stride, n, gout, gst, threads):
    """Whole-shard check of a timed decode: the CPU oracle's DecodeBuffer of
    the same arena must give the same status word for every blob and the same
    columns (fixed values, validity, views) for every blob that decodes."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_bridge as ob  # checker only
    o_out, o_st = ob.decode(cfg.chain, arena, offsets, n, stride=stride, nthreads=threads, mode=cfg.mode)
    g_st = gst[:n].cpu().numpy().astype(np.uint32)
    same = bool(np.array_equal(o_st[:n], g_st))
    ok = o_st[:n] == 0
    h = hashlib.sha256(g_st.tobytes())
    for c, sp in enumerate(o_out.specs):
        for name in ("data", "valid", "start", "length"):
            a = getattr(o_out, name)[c]
            if a is None or not same:
                continue
            b = getattr(gout, name)[c].cpu().numpy()
            b = b.view(np.uint64) if name == "start" else b.view(np.uint32) if name == "length" else b
            if name == "data":
                a2, b2 = a[: n * sp.width].reshape(n, sp.width), b[: n * sp.width].reshape(n, sp.width)
                same = same and bool(np.array_equal(a2[ok], b2[ok]))
            else:
                same = same and bool(np.array_equal(a[:n][ok], b[:n][ok]))
            h.update(np.ascontiguousarray(b[: n * (sp.width if name == "data" else 1)]).tobytes())
    return same, int(ok.sum()), h.hexdigest()[:16]


def validate_parity(cfg, arena, offsets, stride, n, gst, threads):
    """Whole-shard check of a timed ValidateBuffer against the CPU oracle's."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_bridge as ob  # checker only
    o_st = ob.validate(cfg.chain, arena, offsets, n, stride=stride, nthreads=threads, mode=cfg.mode & 0x100)
    g_st = gst[:n].cpu().numpy().astype(np.uint32)
    same = bool(np.array_equal(o_st[:n], g_st))
    return same, int((o_st[:n] == 0).sum()), hashlib.sha256(g_st.tobytes()).hexdigest()[:16]


def get_parity(arena, offsets, stride, n, path, getter, gvals, gst):
    """Whole-shard check of a timed GetAccess gather against the CPU oracle's
    getter: status for every blob, the typed value for every blob it returns."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_bridge as ob  # checker only
    o_vals, _, _, _, o_st = ob.get_batch(arena, offsets, n, path, getter, stride=stride)
    g_st = gst[:n].cpu().numpy()
    g_vals = gvals[:n].cpu().numpy()
    ok = o_st[:n] == 0
    same = bool(np.array_equal(o_st[:n], g_st)) and bool(np.array_equal(o_vals[:n][ok], g_vals[ok]))
    return same, int(ok.sum()), hashlib.sha256(g_vals.tobytes() + g_st.tobytes()).hexdigest()[:16]


def pcie_ceiling(dev, nbytes=1 << 30, repeats=3, pieces=(4 << 20, 16 << 20, 64 << 20, 256 << 20)):
    """Pinned host <-> device copy rates of this box (GB/s) with plain HIP
    calls (libamdhip64 through ctypes): H2D alone, D2H alone, and both at once
    on two streams, each the BEST over `repeats` runs at every copy size in
    `pieces` (the host pipeline moves 4-64 MiB chunks, three in flight), so the
    ceiling is the link's, not one copy shape's.  1 GiB per run: with 256 MiB
    runs the per-copy launch overhead held the probe ~1 % under what the C5
    host pipeline then reached (frac_of_pcie 1.006).  `bidir_total_gbs` =
    both directions' bytes / time."""
    import ctypes as C
    import torch
    torch.cuda.synchronize()
    hip = C.CDLL("libamdhip64.so")
    vp = C.c_void_p
    hip.hipHostMalloc.argtypes = [C.POINTER(vp), C.c_size_t, C.c_uint]
    hip.hipMalloc.argtypes = [C.POINTER(vp), C.c_size_t]
    hip.hipMemcpyAsync.argtypes = [vp, vp, C.c_size_t, C.c_int, vp]
    hip.hipStreamCreate.argtypes = [C.POINTER(vp)]
    hip.hipStreamSynchronize.argtypes = [vp]
    hip.hipFree.argtypes = [vp]
    hip.hipHostFree.argtypes = [vp]
    hip.hipStreamDestroy.argtypes = [vp]
    h_in, h_out, d_in, d_out, s1, s2 = (vp() for _ in range(6))
    ok = (hip.hipHostMalloc(C.byref(h_in), nbytes, 0) == 0 and hip.hipHostMalloc(C.byref(h_out), nbytes, 0) == 0 and
          hip.hipMalloc(C.byref(d_in), nbytes) == 0 and hip.hipMalloc(C.byref(d_out), nbytes) == 0 and
          hip.hipStreamCreate(C.byref(s1)) == 0 and hip.hipStreamCreate(C.byref(s2)) == 0)
    if not ok:
        return {"error": "HIP allocation failed"}
    H2D, D2H = 1, 2

    def run(h2d, d2h, piece):
        hip.hipStreamSynchronize(s1)
        hip.hipStreamSynchronize(s2)
        t0 = time.perf_counter()
        for off in range(0, nbytes, piece):
            if h2d:
                hip.hipMemcpyAsync(vp(d_in.value + off), vp(h_in.value + off), piece, H2D, s1)
            if d2h:
                hip.hipMemcpyAsync(vp(h_out.value + off), vp(d_out.value + off), piece, D2H, s2)
        hip.hipStreamSynchronize(s1)
        hip.hipStreamSynchronize(s2)
        return nbytes * (int(h2d) + int(d2h)) / (time.perf_counter() - t0) / 1e9
    run(True, True, pieces[-1])
    best = {"h2d": 0.0, "d2h": 0.0, "both": 0.0}
    for piece in pieces:
        for _ in range(repeats):
            best["h2d"] = max(best["h2d"], run(True, False, piece))
            best["d2h"] = max(best["d2h"], run(False, True, piece))
            best["both"] = max(best["both"], run(True, True, piece))
    for p_ in (d_in, d_out):
        hip.hipFree(p_)
    for p_ in (h_in, h_out):
        hip.hipHostFree(p_)
    hip.hipStreamDestroy(s1)
    hip.hipStreamDestroy(s2)
    return {"h2d_gbs": round(best["h2d"], 2), "d2h_gbs": round(best["d2h"], 2), "bidir_total_gbs": round(best["both"], 2),
            "note": f"hipMemcpyAsync of pinned (hipHostMalloc) {nbytes >> 20} MiB in "
                    f"{'/'.join(str(p >> 20) for p in pieces)} MiB copies, best of {repeats} per size; bidir = H2D "
                    "and D2H on two streams at once, both directions' bytes / time"}


def pcie_time(pcie, b_in, b_out):
    """Seconds the box's PCIe needs for b_in bytes H2D and b_out bytes D2H
    moving at once: each direction at most its one-way rate, both together at
    most the measured bidirectional total."""
    if "error" in pcie:
        return float("nan")
    return max(b_in / (pcie["h2d_gbs"] * 1e9), b_out / (pcie["d2h_gbs"] * 1e9),
               (b_in + b_out) / (pcie["bidir_total_gbs"] * 1e9))


def host_leg(schema, hc, dev):
    """packos_encode_host_batch: pinned host columns -> pipelined H2D / encode /
    D2H through the library (the entry point a cgo shim binds) -> pinned host
    arena, and packos_decode_host_batch back.  Best of 2 per chunk size after
    one warm-up call (the schema's cached pipeline keeps its buffers); never
    `value`.  `frac_of_pcie` = the time the bytes need at the box's measured
    full-duplex copy rates / the measured time."""
    import torch
    from packos_amd.api import encode_host_batch, host_batch_bound
    pcie = pcie_ceiling(dev)
    pinned = []
    for lst in (hc.data, hc.offsets, hc.valid):
        for c, a in enumerate(lst):
            if a is not None:
                t = torch.from_numpy(np.ascontiguousarray(a)).pin_memory()
                pinned.append(t)
                lst[c] = t.numpy()
    cap = host_batch_bound(schema, hc)
    out = torch.empty(cap, dtype=torch.uint8).pin_memory().numpy()
    offs = torch.empty(hc.n + 1, dtype=torch.int64).pin_memory().numpy().view(np.uint64)
    best = None
    encode_host_batch(schema, hc, chunk_blobs=1 << 17, want_status=False, out=out, offsets=offs)   # warm-up
    for chunk in (1 << 15, 1 << 16, 1 << 17, 1 << 18):
        for _ in range(2):
            t0 = time.perf_counter()
            encode_host_batch(schema, hc, chunk_blobs=chunk, want_status=False, out=out, offsets=offs)
            el = time.perf_counter() - t0
            if best is None or el < best[0]:
                best = (el, chunk)
    el, chunk = best
    tot = int(offs[hc.n])
    b_in = hc.nbytes_in()
    b_out = tot + (0 if schema.fixed_blob_size > 0 else 8 * hc.n)   # arena + blob offsets
    ideal = pcie_time(pcie, b_in, b_out)
    enc = {"million_blobs_per_s": round(hc.n / el / 1e6, 3), "gib_per_s_out": round(tot / el / 2 ** 30, 3),
           "gib_per_s_in_plus_out": round((tot + b_in) / el / 2 ** 30, 3),
           "bytes_in": b_in, "bytes_out": b_out, "ms": round(el * 1e3, 3),
           "frac_of_pcie": round(ideal / el, 3), "pcie": pcie,
           "chunk_blobs": chunk, "note": "pinned host columns -> packos_encode_host_batch -> pinned host arena"}
    # the read side: the pinned arena just produced -> packos_decode_host_batch
    # -> pinned host columns (views into the host arena)
    from packos_amd.api import HostDecoded, decode_host_batch

    def pinned(shape, dtype):
        return torch.empty(shape, dtype=getattr(torch, np.dtype(dtype).name.replace("uint64", "int64")
                                                .replace("uint32", "int32"))).pin_memory().numpy().view(dtype)
    hd = HostDecoded(schema, hc.n, alloc=pinned)
    hst = pinned(max(hc.n, 1), np.uint32)
    fixed = schema.fixed_blob_size > 0 and all(v is None for v in hc.valid)
    dbest = None
    for chunk in (1 << 15, 1 << 16, 1 << 17, 1 << 18):
        for _ in range(2):
            t0 = time.perf_counter()
            if fixed:
                decode_host_batch(schema, out[:tot], None, hc.n, stride=schema.fixed_blob_size, chunk_blobs=chunk,
                                  out=hd, status=hst)
            else:
                decode_host_batch(schema, out[:tot], offs, hc.n, chunk_blobs=chunk, out=hd, status=hst)
            el = time.perf_counter() - t0
            if dbest is None or el < dbest[0]:
                dbest = (el, chunk)
    ok = bool((hst[:hc.n] == 0).all())
    d_out = 4 * hc.n
    for sp in schema.specs:
        d_out += hc.n * sp.width if sp.fixed else (12 * hc.n if sp.var else 0)
        d_out += hc.n if sp.has_valid else 0
    d_in = tot + (0 if fixed else 8 * (hc.n + 1))
    dideal = pcie_time(pcie, d_in, d_out)
    enc["decode"] = {"million_blobs_per_s": round(hc.n / dbest[0] / 1e6, 3),
                     "gib_per_s_in": round(tot / dbest[0] / 2 ** 30, 3), "chunk_blobs": dbest[1], "all_ok": ok,
                     "bytes_in": d_in, "bytes_out": d_out, "ms": round(dbest[0] * 1e3, 3),
                     "frac_of_pcie": round(dideal / dbest[0], 3),
                     "note": "pinned host arena -> packos_decode_host_batch -> pinned host columns"}
    return enc


# ----------------------------------------------------------------- ranks
def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_cmd(gpus, env, argv, port=None):
    """The command that starts `gpus` rank processes of this bench, or None
    when this process is itself a rank (gpus == 1, or a launcher already set
    WORLD_SIZE).  `python bench.py --gpus N` with no launcher around it runs
    `torch.distributed.run --nproc-per-node N` on itself as a child, before
    anything here touches the GPU; the parent only waits for it."""
    if gpus <= 1 or "WORLD_SIZE" in env or env.get("PACKOS_BENCH_RANK_CHILD"):
        return None
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(gpus),
            "--master-addr", "127.0.0.1", "--master-port", str(port or _free_port()),
            os.path.abspath(__file__)] + list(argv)


def world_error(gpus, world, backend, device_count, local_world, local):
    """Why this rank must not run (a message), or None: the job must have
    exactly --gpus ranks, and under nccl (RCCL) every local rank needs a
    device of its own."""
    if world != gpus:
        return f"bench.py: --gpus {gpus} but the job has {world} rank(s) (WORLD_SIZE); refusing to label the run"
    if backend == "nccl" and world > 1:
        if device_count < local_world:
            return (f"bench.py: {local_world} ranks on this node but torch.cuda.device_count() = {device_count}: "
                    f"--gpus {gpus} needs a GPU per rank")
        if not 0 <= local < device_count:
            return f"bench.py: local rank {local} has no device (device_count {device_count})"
    return None


# ----------------------------------------------------------------- main
def main():
    args = parse()
    cmd = launch_cmd(args.gpus, os.environ, sys.argv[1:])
    if cmd is not None:
        # parent of N ranks: no GPU work here; exit with the job's status
        import subprocess
        env = dict(os.environ, PACKOS_BENCH_RANK_CHILD="1")
        sys.exit(subprocess.run(cmd, env=env, cwd=ROOT).returncode)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    # rehearsal knobs (tests only): every rank on one device, gloo for the
    # harness barrier / timing all-reduce; the driver's runs use neither
    if os.environ.get("PACKOS_BENCH_DEVICE") is not None:
        local = int(os.environ["PACKOS_BENCH_DEVICE"])
    backend = os.environ.get("PACKOS_BENCH_BACKEND", "nccl")
    err = world_error(args.gpus, world, backend, torch.cuda.device_count(), local_world, local)
    if err:
        print(err, file=sys.stderr, flush=True)
        sys.exit(3)
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    # rank -> device map (PCI bus of each rank's GPU), reported in `config`
    props = torch.cuda.get_device_properties(dev)
    me = {"rank": rank, "device": dev.index, "pci_bus": getattr(props, "pci_bus_id", None),
          "host": platform.node()}
    rank_map = [me]
    if world > 1:
        rank_map = [None] * world
        dist.all_gather_object(rank_map, me)
        if backend == "nccl" and len({(m["host"], m["device"]) for m in rank_map}) != world:
            print(f"bench.py: ranks share a device under nccl: {rank_map}", file=sys.stderr, flush=True)
            sys.exit(3)

    from packos_amd.api import CompiledSchema, DeviceColumns, EncodePlan
    from packos_amd.configs import CONFIGS, algorithmic_bytes, make_columns
    from packos_amd.shard import config_shard

    cfg = CONFIGS[args.config]
    schema = CompiledSchema(cfg.chain, cfg.mode)
    fixed = schema.fixed_blob_size > 0
    per_gpu = args.blobs_per_gpu or cfg.shard
    lo, hi, n_global = config_shard(cfg, schema, per_gpu, world, rank)
    n = hi - lo
    hc = make_columns(cfg, n=n, lo=lo)
    stream = torch.cuda.current_stream()

    # S device copies of the shard: distinct column buffers and output arenas
    sets = []
    base = DeviceColumns.from_host(schema, hc, dev)
    for s in range(max(1, args.sets)):
        if s == 0:
            dc = base
        else:
            cl = lambda xs: [None if x is None else x.clone() for x in xs]  # noqa: E731
            dc = DeviceColumns(schema, n, cl(base.data), cl(base.offsets), cl(base.valid))
        sets.append(EncodePlan(schema, dc, stream=stream))
    torch.cuda.synchronize()
    total_out = sets[0].total
    footprint = sum(p.cols.nbytes() + p.out.numel() for p in sets)

    runs = [p.run for p in sets]
    if args.op == "decode":
        from packos_amd.api import DecodedColumns, decode_batch
        for p in sets:
            p.run()
        torch.cuda.synchronize()

        outs = []

        def dec_runner(p):
            dcols = DecodedColumns(schema, n, dev)
            st = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
            outs.append((dcols, st))
            if fixed:
                return lambda: decode_batch(schema, p.out, None, n, stride=p.B, stream=stream, out=dcols, status=st)
            return lambda: decode_batch(schema, p.out, p.offsets, n, stream=stream, out=dcols, status=st)
        runs = [dec_runner(p) for p in sets]
    elif args.op == "validate":
        from packos_amd.api import validate_batch
        for p in sets:
            p.run()
        torch.cuda.synchronize()
        outs = []

        def val_runner(p):
            st = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
            outs.append((None, st))
            if fixed:
                return lambda: validate_batch(schema, p.out, None, n, stride=p.B, stream=stream, status=st)
            return lambda: validate_batch(schema, p.out, p.offsets, n, stream=stream, status=st)
        runs = [val_runner(p) for p in sets]
    elif args.op == "get":
        from packos_amd import _lib
        import ctypes as C
        for p in sets:
            p.run()
        torch.cuda.synchronize()
        L = _lib.lib()
        if args.get_pos < 0:
            args.get_pos = first_int64(cfg.chain)
        path = (C.c_int32 * 1)(args.get_pos)

        def get_runner(p):
            vals = torch.empty((max(n, 1), 8), dtype=torch.uint8, device=dev)
            sps = [torch.empty(max(n, 1), dtype=dt, device=dev) for dt in (torch.int64, torch.int32, torch.uint8)]
            st = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
            offs = None if fixed else p.offsets.data_ptr()
            stride = p.B if fixed else 0
            sp = C.c_void_p(stream.cuda_stream)
            s0, ln, tg = (t.data_ptr() for t in sps) if args.get_spans else (None, None, None)
            outs.append((vals, st))
            return lambda: L.packos_get_batch(p.out.data_ptr(), offs, stride, n, path, 1, _lib_get_int, 0, 0,
                                              vals.data_ptr(), 8, s0, ln, tg, st.data_ptr(), sp)
        _lib_get_int = 3   # PACKOS_GET_INT
        outs = []
        runs = [get_runner(p) for p in sets]

    def timed(plans, steps, warmup):
        for k in range(warmup):
            plans[k % len(plans)]()
        torch.cuda.synchronize()
        # HIP events on the launch stream bracket the timed region: elapsed / K
        # is the average step duration on the GPU (a fixed schema's step is the
        # one encode kernel; agrees with rocprofv3 --kernel-trace).
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0.record(stream)
        for k in range(steps):
            plans[k % len(plans)]()
        ev1.record(stream)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if world > 1:
            dist.barrier()
            t = torch.tensor([el], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el, ev0.elapsed_time(ev1) / steps

    # Every timed pass starts from a scrubbed cache: a 512 MiB write evicts the
    # L2s and the 256 MiB Infinity Cache (MALL), so no pass inherits another's
    # lines.  Cold passes (rotated sets) and warm passes (set 0 replayed)
    # interleave, cold first and last (cold, warm, cold, warm, cold for 3
    # passes): the headline is the median cold pass, and the spread over the
    # passes, in both orders, is reported.
    scrub_buf = torch.empty(512 << 20, dtype=torch.uint8, device=dev)

    def scrub(k):
        scrub_buf.fill_(k & 0xFF)
        torch.cuda.synchronize()

    order = []
    for k in range(max(1, args.passes)):
        order.append("cold")
        if not args.no_warm and k + 1 < max(1, args.passes):
            order.append("warm")
    if not args.no_warm and args.passes <= 1:
        order.append("warm")
    passes = []
    # the first pass primes with K more untimed steps: in a fresh process the
    # first timed pass of a long step ran up to 20 % slow (C4 decode 0.383 vs
    # 0.317-0.324 ms in passes 2..9; 0.331 after 40 warmup steps), a
    # start-up effect, not the kernel's
    prime = args.warmup + args.steps
    for k, kind in enumerate(order):
        scrub(k)
        e, km = timed(runs if kind == "cold" else runs[:1], args.steps, prime if k == 0 else args.warmup)
        passes.append({"kind": kind, "kernel_ms": round(km, 5), "ms_per_step": round(e / args.steps * 1e3, 4),
                       "_el": e})
    colds = sorted((p for p in passes if p["kind"] == "cold"), key=lambda p: p["kernel_ms"])
    warms = sorted((p for p in passes if p["kind"] == "warm"), key=lambda p: p["kernel_ms"])
    mid = colds[(len(colds) - 1) // 2]
    el, kernel_ms = mid["_el"], mid["kernel_ms"]
    warm_el, warm_kms = (None, None) if not warms else (warms[(len(warms) - 1) // 2]["_el"],
                                                       warms[(len(warms) - 1) // 2]["kernel_ms"])
    for p_ in passes:
        del p_["_el"]
    cold_spread = (colds[-1]["kernel_ms"] - colds[0]["kernel_ms"]) / kernel_ms if kernel_ms else 0.0
    del scrub_buf

    alg = algorithmic_bytes(hc, total_out, with_offsets=not fixed)
    gran = None   # granularity-aware bytes: reads counted as whole 128-B lines
    if args.op != "encode":
        if fixed:
            b0 = np.arange(n, dtype=np.uint64) * np.uint64(schema.fixed_blob_size)
            b1 = b0 + np.uint64(schema.fixed_blob_size)
        else:
            o = sets[0].offsets.cpu().numpy().astype(np.uint64)
            b0, b1 = o[:-1], o[1:]
    if args.op == "decode":
        # DecodeBuffer reads every blob byte except var payloads (returned as
        # views, never read) + the offsets; writes columns, views, validity, status
        var_bytes = sum(int(o[-1]) - int(o[0]) for o in hc.offsets if o is not None)
        out_b = 4 * n
        for sp in schema.specs:
            out_b += n * sp.width if sp.fixed else (12 * n if sp.var else 0)
            out_b += n if sp.has_valid else 0
        alg = total_out - var_bytes + (0 if fixed else 8 * (n + 1)) + out_b
        pre, tail_fixed = static_prefix(cfg.chain)
        end = b1 if (pre is None or tail_fixed) else np.minimum(b1, b0 + np.uint64(pre))
        gran = LINE * lines_touched(b0, end) + (0 if fixed else 8 * (n + 1)) + out_b
    elif args.op == "validate":
        # ValidateBuffer reads the header blocks, Match literals and checked
        # payloads (+ the blob offsets for var layouts) and writes the status
        rb, win = validate_reads(cfg.chain, cfg.mode & 1)
        alg = n * (rb + 4) + (0 if fixed else 8 * (n + 1))
        end = b1 if win is None else np.minimum(b1, b0 + np.uint64(win))
        gran = LINE * lines_touched(b0, end) + n * 4 + (0 if fixed else 8 * (n + 1))
    elif args.op == "get":
        # GetAccess rangeAt: h0 + the two header words around the field + its
        # payload (8 B for an int64) in; GetInt's (value, error) out = value 8 +
        # status 1 (--get-spans: + start 8 + len 4 + tag 1); + the blob offsets
        # for var layouts
        wout = 22 if args.get_spans else 9
        alg = n * (2 + 4 + 8) + n * wout + (0 if fixed else 8 * (n + 1))
        H, flds = top_layout(cfg.chain)
        pay_end = H + sum(w for _, w in flds[:args.get_pos + 1])
        end = np.minimum(b1, b0 + np.uint64(max(pay_end, 2 * args.get_pos + 4)))
        gran = LINE * lines_touched(b0, end) + n * wout + (0 if fixed else 8 * (n + 1))
    blobs = n_global * args.steps
    value = blobs / el / 1e6
    achieved = alg / (kernel_ms * 1e-3) / 1e9
    warm_achieved = alg / (warm_kms * 1e-3) / 1e9 if warm_kms else None

    # PMC traffic is not collected in this process (rocprofv3 --pmc runs are
    # separate passes of this same command): bench_pmc/ holds their summary,
    # used when it was measured on this same product tree.
    traffic, traffic_src = pmc_traffic(args.config, args.op)

    cpu, parity, host = None, None, None
    if args.op != "encode":
        args.no_cpu = args.no_host = True
    if rank == 0 and world == 1 and not args.no_cpu:
        gpu_arena = sets[0].out[:total_out].cpu().numpy()
        gpu_offs = None if fixed else sets[0].offsets.cpu().numpy()
        res, hi_, same, digest, tot = cpu_leg(cfg, hc, args.cpu_seconds, gpu_arena, gpu_offs)
        mt = res["mt"]
        cpu = {"value": round(mt[0] / 1e6, 4), "unit": "million blobs/s", "cores": hi_["effective_cpus"],
               "kind": "port",
               "sample": f"the whole shard ({n} blobs of config {args.config}), {mt[1]} passes in {mt[2]:.1f} s; "
                         f"C restatement of PutAccess/Pack (oracle/) on {mt[3]} threads, the faster of "
                         f"{sorted(res['tried'])} threads (cgroup-quota CPUs and affinity CPUs)",
               "threads": mt[3], "threads_tried_mblobs_s": res["tried"],
               "single_thread_value": round(res['st'][0] / 1e6, 4),
               "nproc": hi_["nproc"], "affinity": hi_["affinity"], "cgroup_cpu_quota": hi_["cgroup_cpu_quota"],
               "cpu_model": hi_["cpu_model"]}
        parity = {"result": "bit-exact" if same else "MISMATCH", "blobs": n, "bytes": tot,
                  "sha256_16": digest, "checked": "GPU arena of the timed run vs the CPU oracle, whole shard"}
    if world > 1 and not args.no_cpu and args.op == "encode":
        # every rank checks its WHOLE shard against the CPU oracle's encoding of
        # the same global slice, piece by piece (SCALE runs carry the same
        # correctness as the 1-GPU line); flags meet in a MIN
        hi_ = host_info()
        th = max(1, (int(hi_["cgroup_cpu_quota"] or 0) or hi_["affinity"] or 1) // max(1, int(
            os.environ.get("LOCAL_WORLD_SIZE", world))))
        same, checked, digest = shard_parity(cfg, hc, sets[0].out, None if fixed else sets[0].offsets,
                                             schema.fixed_blob_size, th, piece=max(1, args.parity_piece))
        flag = torch.tensor([1 if same and checked == n else 0, checked], dtype=torch.int64,
                            device=dev if backend == "nccl" else "cpu")
        mins = flag.clone()
        dist.all_reduce(mins, op=dist.ReduceOp.MIN)
        parity = {"result": "bit-exact" if int(mins[0].item()) == 1 else "MISMATCH", "ranks": world,
                  "blobs_rank0": n, "checked_blobs_per_rank_min": int(mins[1].item()), "sha256_16_rank0": digest,
                  "checked": f"every rank: its whole GPU shard (in {max(1, args.parity_piece)}-blob pieces) vs the CPU "
                             "oracle's encoding of the same global slice"}
    if args.op != "encode" and os.environ.get("PACKOS_BENCH_NO_PARITY") is None:
        # the timed run's set-0 outputs vs the CPU oracle over this rank's whole
        # shard (every rank; flags meet in a MIN)
        arena_np = sets[0].out[:total_out].cpu().numpy()
        offs_np = None if fixed else sets[0].offsets.cpu().numpy().astype(np.uint64)
        stride = schema.fixed_blob_size if fixed else 0
        hi_ = host_info()
        th = max(1, (int(hi_["cgroup_cpu_quota"] or 0) or hi_["affinity"] or 1) // max(1, int(
            os.environ.get("LOCAL_WORLD_SIZE", world))))
        if args.op == "decode":
            same, n_ok, digest = decode_parity(cfg, arena_np, offs_np, stride, n, outs[0][0], outs[0][1], th)
            what = "status of every blob + columns / validity / views of every blob that decodes"
        elif args.op == "validate":
            same, n_ok, digest = validate_parity(cfg, arena_np, offs_np, stride, n, outs[0][1], th)
            what = "ValidateBuffer status of every blob"
        else:
            same, n_ok, digest = get_parity(arena_np, offs_np, stride, n, [args.get_pos], 3, outs[0][0], outs[0][1])
            what = "status of every blob + GetInt value of every blob that has one"
        del arena_np
        if world > 1:
            flag = torch.tensor([1 if same else 0], dtype=torch.int64, device=dev if backend == "nccl" else "cpu")
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            same = int(flag.item()) == 1
        parity = {"result": "bit-exact" if same else "MISMATCH", "ranks": world, "blobs": n, "blobs_ok": n_ok,
                  "sha256_16": digest,
                  "checked": f"GPU {args.op} outputs of the timed run (set 0) vs the CPU oracle over the whole "
                             f"shard{' of every rank' if world > 1 else ''}: {what}"}
    if rank == 0 and world == 1 and not args.no_host:
        try:
            host = host_leg(schema, make_columns(cfg, n=min(n, 1 << 22), lo=lo), dev)
        except Exception as e:  # reported, never fatal for the device-resident metric
            host = {"error": str(e)[:200]}

    if rank == 0:
        line = {
            "metric": "million blobs/s + GiB/s device-resident encode, 1M×256B fixed-schema tuples"
                      if args.op == "encode" else f"million blobs/s device-resident {args.op} (per-config table)",
            "value": round(value, 3),
            "unit": "million blobs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 indexed by global blob, seed 0x%X)" % cfg.seed,
            "config": {"workload": f"{args.config}: {cfg.note}", "op": args.op, "blobs_per_gpu": n, "global_blobs": n_global,
                       "blob_bytes": schema.fixed_blob_size if fixed else round(total_out / n, 1),
                       "parallelism": f"dp{world} (byte-balanced disjoint shards, no collective)",
                       "backend": backend if world > 1 else None, "world_size": world,
                       "rank_devices": [[m["rank"], m["device"], m["pci_bus"]] for m in rank_map],
                       "sets_rotated": len(sets), "footprint_mib": round(footprint / 2 ** 20, 1),
                       **({"get": f"GetInt(pos {args.get_pos}) -> " + ("value, start, len, tag, status" if args.get_spans
                                                                       else "value, status")}
                          if args.op == "get" else {})},
            "gib_per_s": round(total_out * n_global / n * args.steps / el / 2 ** 30, 2),
            "kernel_ms": round(kernel_ms, 5),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": alg,
                         **({} if gran is None else {
                             "granularity_bytes_per_launch": gran,
                             "frac_granularity": round(gran / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                             "granularity_rule": f"reads counted as whole {LINE}-B lines (union over blobs)"}),
                         "cache_state": f"cold: {len(sets)} sets rotated ({footprint / 2 ** 20:.0f} MiB > 256 MiB "
                                        "Infinity Cache), every pass after a 512 MiB scrub write"},
            "passes": {"order": [p_["kind"] for p_ in passes], "kernel_ms": [p_["kernel_ms"] for p_ in passes],
                       "warmup_first_pass": prime,
                       "ms_per_step": [p_["ms_per_step"] for p_ in passes],
                       "cold_spread": round(cold_spread, 4),
                       "headline": "median cold pass (each pass: W warmup + exactly K timed steps)"},
            "warm": None if warm_kms is None else {
                "kernel_ms": round(warm_kms, 5), "achieved": round(warm_achieved, 1),
                "frac": round(warm_achieved / HBM_PEAK_GBS, 4), "ms_per_step": round(warm_el / args.steps * 1e3, 4),
                "note": "set 0 replayed back to back (inputs may stay in the Infinity Cache)"},
            "cpu_baseline": cpu,
            "parity": parity,
            "host_resident": host,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
