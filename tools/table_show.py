#!/usr/bin/env python3
"""Print a gpu_table.sh table.jsonl compactly: config, op, kernel ms, frac, line-granular frac, parity."""
import json
import sys

for l in open(sys.argv[1]):
    d = json.loads(l)
    r = d["roofline"]
    c = d["config"]["workload"].split(":")[0]
    op = d["config"]["op"]
    cpu = d.get("cpu_baseline") or {}
    host = d.get("host_resident") or {}
    print(f"{c:3s} {op:8s} {d['kernel_ms']:.5f} ms  frac {r['frac']:.3f}  gran {r.get('frac_granularity') or 0:.3f}  "
          f"spread {d.get('passes', {}).get('cold_spread', 0):.3f}  traffic {'y' if r.get('traffic') else '-'}  "
          f"parity {(d.get('parity') or {}).get('result', '-')}  cpu {cpu.get('value', '-')}  "
          f"host {host.get('million_blobs_per_s', '-')}/{(host.get('decode') or {}).get('million_blobs_per_s', '-')}")
