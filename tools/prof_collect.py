#!/usr/bin/env python3
"""Summarise a tools/prof_ops.sh pass into profiles/<round>/<tag>/:

    python tools/prof_collect.py gpurun_out/p3 profiles/r03/<tag> [commit]

For every <cfg>_<op> found: the bench line, the rocprofv3 kernel-stats CSV,
the FETCH_SIZE / WRITE_SIZE / SQ counter CSVs (copied), and a summary JSON
<cfg>_<op>.json with the dominant kernel's rocprof average, its FETCH / WRITE
bytes per launch (FETCH_SIZE and WRITE_SIZE are KiB; fetch reported raw and
with MI355X_MICROARCH.md's gfx950 x2 for 16-B/lane streaming reads, the
factor measured by tools/fetch_calib.hip for scattered shapes is applied when
given in calib.json), and the SQ counters per wave.  Also writes
profiles/<round>/pmc_<cfg>[_<op>].json and bench_pmc/pmc_<cfg>[_<op>].json,
which bench.py reads for `traffic` when its product_tree (the hash
tools/prof_ops.sh recorded on the box, bench.product_tree_hash) equals the
running tree's.
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

KSUB = {"decode": ("k_decode",), "validate": ("k_decode", "k_validate"), "get": ("k_get_field",), "encode": ("k_encode",)}


def last_json(path):
    try:
        lines = [l for l in open(path) if l.startswith("{")]
        return json.loads(lines[-1]) if lines else None
    except OSError:
        return None


def one(pattern):
    m = sorted(glob.glob(pattern, recursive=True))
    return m[0] if m else None


def dominant(stats_csv, op):
    rows = [r for r in csv.DictReader(open(stats_csv)) if any(k in r["Name"] for k in KSUB[op])]
    return max(rows, key=lambda r: float(r["TotalDurationNs"])) if rows else None


def per_launch(path, kname):
    per = {}
    for r in csv.DictReader(open(path)):
        if r["Kernel_Name"] != kname:
            continue
        k = (r["Counter_Name"], r["Dispatch_Id"])
        per[k] = per.get(k, 0.0) + float(r["Counter_Value"])
    by = {}
    for (c, _), v in per.items():
        by.setdefault(c, []).append(v)
    return {c: statistics.median(v) for c, v in by.items()}, {c: len(v) for c, v in by.items()}


def main():
    src, dst = sys.argv[1], sys.argv[2]
    commit = sys.argv[3] if len(sys.argv) > 3 else "unknown"
    rnd_dir = os.path.dirname(dst.rstrip("/"))
    os.makedirs(dst, exist_ok=True)
    calib = {}
    cpath = os.path.join(dst, "calib.json")
    if os.path.exists(cpath):
        calib = json.load(open(cpath))
    out = []
    tree = None
    tpath = os.path.join(src, "product_tree.txt")
    if os.path.exists(tpath):
        tree = open(tpath).read().strip() or None
    bench_pmc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench_pmc")
    os.makedirs(bench_pmc, exist_ok=True)
    for line_log in sorted(glob.glob(os.path.join(src, "*.line.log"))):
        tag = os.path.basename(line_log)[: -len(".line.log")]
        cfg, op = tag.rsplit("_", 1)
        line = last_json(line_log)
        if line is None:
            continue
        with open(os.path.join(dst, f"{tag}_line.json"), "w") as f:
            json.dump(line, f)
        res = {"config": cfg, "op": op, "commit": commit, "bench_kernel_ms": line.get("kernel_ms"),
               "algorithmic_bytes_per_launch": line["roofline"]["algorithmic_bytes_per_launch"],
               "granularity_bytes_per_launch": line["roofline"].get("granularity_bytes_per_launch"),
               "frac_algorithmic": line["roofline"]["frac"],
               "frac_granularity": line["roofline"].get("frac_granularity")}
        st = one(os.path.join(src, f"{tag}_trace", "**", "*kernel_stats.csv"))
        if st:
            shutil.copy(st, os.path.join(dst, f"{tag}_kernel_stats.csv"))
            d = dominant(st, op)
            if d:
                res["kernel"] = d["Name"]
                res["rocprof_avg_us"] = round(float(d["AverageNs"]) / 1e3, 3)
                res["rocprof_calls"] = int(d["Calls"])
        kname = res.get("kernel")
        for pass_ in ("FETCH_SIZE", "WRITE_SIZE", "SQ"):
            pc = one(os.path.join(src, f"{tag}_{pass_}", "**", "*counter_collection.csv"))
            if not pc or not kname:
                continue
            if pass_ != "SQ":   # the SQ pass is kept as its per-wave summary in <tag>.json only
                shutil.copy(pc, os.path.join(dst, f"{tag}_pmc_{pass_.lower()}.csv"))
            med, cnt = per_launch(pc, kname)
            if pass_ == "FETCH_SIZE" and "FETCH_SIZE" in med:
                raw = med["FETCH_SIZE"] * 1024
                res["fetch_bytes_raw"] = raw
                res["fetch_bytes_x2"] = 2 * raw
            elif pass_ == "WRITE_SIZE" and "WRITE_SIZE" in med:
                res["write_bytes"] = med["WRITE_SIZE"] * 1024
            elif pass_ == "SQ" and "SQ_WAVES" in med:
                w = med["SQ_WAVES"]
                res["sq_per_wave"] = {c: round(v / w, 1) for c, v in sorted(med.items()) if c != "SQ_WAVES"}
                res["sq_waves"] = w
                if "SQ_WAVE_CYCLES" in med and med["SQ_WAVE_CYCLES"]:
                    res["wait_any_frac_of_wave_cycles"] = round(med.get("SQ_WAIT_ANY", 0) / med["SQ_WAVE_CYCLES"], 3)
        if "fetch_bytes_raw" in res and "write_bytes" in res:
            fac = calib.get(f"{cfg}_{op}", {}).get("factor", 2.0)
            res["fetch_factor"] = fac
            res["fetch_factor_source"] = calib.get(f"{cfg}_{op}", {}).get(
                "source", "gfx950 x2 for 16-B/lane streaming reads (MI355X_MICROARCH.md HBM)")
            res["hbm_bytes_per_launch"] = res["fetch_bytes_raw"] * fac + res["write_bytes"]
            res["traffic_over_algorithmic"] = round(res["hbm_bytes_per_launch"] / res["algorithmic_bytes_per_launch"], 4)
            if res.get("granularity_bytes_per_launch"):
                res["traffic_over_granularity"] = round(res["hbm_bytes_per_launch"] / res["granularity_bytes_per_launch"], 4)
            pmc = {"kernel": kname, "commit": commit, "product_tree": tree,
                   "hbm_bytes_per_launch": res["hbm_bytes_per_launch"],
                   "fetch_bytes_per_launch": res["fetch_bytes_raw"] * fac, "write_bytes_per_launch": res["write_bytes"],
                   "algorithmic_bytes_per_launch": res["algorithmic_bytes_per_launch"],
                   "traffic_over_algorithmic": res["traffic_over_algorithmic"],
                   "correction": f"fetch = FETCH_SIZE KiB x 1024 x {fac} ({res['fetch_factor_source']}); "
                                 "write = WRITE_SIZE KiB x 1024",
                   "source": f"{dst}/{tag}_pmc_fetch_size.csv, {dst}/{tag}_pmc_write_size.csv "
                             "(rocprofv3 --pmc, separate passes)"}
            name = f"pmc_{cfg}.json" if op == "encode" else f"pmc_{cfg}_{op}.json"
            for d in (rnd_dir, bench_pmc):
                with open(os.path.join(d, name), "w") as f:
                    json.dump(pmc, f, indent=1)
        with open(os.path.join(dst, f"{tag}.json"), "w") as f:
            json.dump(res, f, indent=1)
        out.append(res)
        print(json.dumps({k: v for k, v in res.items() if k != "kernel"}))
    with open(os.path.join(dst, "summary.jsonl"), "a") as f:
        for r in out:
            f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
