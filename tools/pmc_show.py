#!/usr/bin/env python3
"""Median per-launch value of every counter in rocprofv3 --pmc CSV dirs, for
kernels whose name contains KEY:  python tools/pmc_show.py KEY dir1 [dir2 ...]"""
import csv
import glob
import os
import statistics
import sys


def main():
    key, dirs = sys.argv[1], sys.argv[2:]
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = {}
            with open(path) as f:
                for row in csv.DictReader(f):
                    if key not in row.get("Kernel_Name", ""):
                        continue
                    k = (row["Counter_Name"], row.get("Dispatch_Id", ""))
                    per[k] = per.get(k, 0.0) + float(row["Counter_Value"])
            byname = {}
            for (name, _), v in per.items():
                byname.setdefault(name, []).append(v)
            for name, vs in sorted(byname.items()):
                print(f"{os.path.basename(d)} {name}: median {statistics.median(vs):.4g} over {len(vs)} launches")


if __name__ == "__main__":
    main()
