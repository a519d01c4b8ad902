#!/usr/bin/env python3
"""Median duration per (kernel, grid) from a rocprofv3 kernel_trace.csv."""
import csv
import sys
from collections import defaultdict

d = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    d[(r["Kernel_Name"][:60], r["Grid_Size_X"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for (name, grid), v in d.items():
    v.sort()
    print(f"{name:60s} grid={grid:>9} n={len(v):3d} med={v[len(v) // 2] / 1000:9.1f}us")
