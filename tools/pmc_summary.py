#!/usr/bin/env python3
"""Turn the two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of
`bench.py --no-cpu` into profiles/pmc_<config>.json (HBM bytes per launch of
the dominant encode kernel), applying MI355X_MICROARCH.md's gfx950
correction: FETCH_SIZE counts half the bytes of a wide coalesced streaming
read (x2); WRITE_SIZE is exact for streaming stores; both are in KiB.

    python tools/pmc_summary.py FETCH.csv WRITE.csv KERNEL_SUBSTR ALG_BYTES OUT.json
"""
import csv
import json
import statistics
import sys


def med(path, counter, kern):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
         if r["Counter_Name"] == counter and kern in r["Kernel_Name"]]
    return statistics.median(v), len(v), next(r["Kernel_Name"] for r in csv.DictReader(open(path))
                                               if kern in r["Kernel_Name"])


def main():
    fpath, wpath, kern, alg, out = sys.argv[1:6]
    f, nf, name = med(fpath, "FETCH_SIZE", kern)
    w, nw, _ = med(wpath, "WRITE_SIZE", kern)
    fb, wb = f * 1024 * 2, w * 1024
    res = {"kernel": name, "FETCH_SIZE_kB_median": f, "WRITE_SIZE_kB_median": w, "launches": [nf, nw],
           "correction": "fetch bytes = FETCH_SIZE*1024*2 (gfx950 half-count on 16-B/lane streaming reads, "
                         "LDS-DMA included); write bytes = WRITE_SIZE*1024",
           "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb, "hbm_bytes_per_launch": fb + wb,
           "algorithmic_bytes_per_launch": int(alg), "traffic_over_algorithmic": round((fb + wb) / int(alg), 4),
           "source": f"{fpath}, {wpath} (rocprofv3 --pmc, separate passes)"}
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
