#!/usr/bin/env python3
"""Per-kernel duration summary from a rocprofv3 sqlite result (rocpd):
    python tools/kstats.py gpurun_out/prof_stream/run_results.db [name-filter]"""
import collections
import re
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
d = collections.defaultdict(list)
for n, du, g in db.execute("select name, duration, grid_x from kernels order by start"):
    if flt in n:
        m = re.search(r"(k_\w+(<\d+>)?)", n)
        d[((m.group(1) if m else n.split("(")[0])[-40:], g)].append(du / 1e3)
for (n, g), v in d.items():
    v = sorted(v)
    print(f"{n:42s} grid={g:9d} n={len(v):3d} median_us={v[len(v)//2]:9.1f} min_us={v[0]:9.1f}")
