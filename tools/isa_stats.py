#!/usr/bin/env python3
"""Static instruction mix of one kernel in a device assembly listing
(hipcc --cuda-device-only -S):  python tools/isa_stats.py kernels.s NAME_SUBSTR"""
import collections
import re
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\S*:\s*(;.*)?$", l) and key in l]
    for s0 in starts:
        name = lines[s0].split(":")[0]
        cnt = collections.Counter()
        meta = {}
        for l in lines[s0 + 1:]:
            t = l.strip()
            if t.startswith(".Lfunc_end"):
                break
            if not t or t.startswith((";", ".")) or t.endswith(":"):
                continue
            op = t.split()[0]
            cls = ("salu" if op.startswith("s_") and not op.startswith(("s_load", "s_buffer", "s_waitcnt", "s_cbranch",
                                                                        "s_branch", "s_barrier", "s_endpgm"))
                   else "smem" if op.startswith(("s_load", "s_buffer")) else "branch" if op.startswith(("s_cbranch", "s_branch"))
                   else "wait" if op.startswith("s_waitcnt") else "valu" if op.startswith("v_")
                   else "vmem" if op.startswith(("global_", "buffer_", "flat_", "scratch_")) else "lds" if op.startswith("ds_")
                   else "other")
            cnt[cls] += 1
            if op.startswith(("global_", "scratch_")):
                cnt[op] += 1
        for l in lines[s0:]:
            m = re.search(r"\.(vgpr_count|sgpr_count|private_segment_fixed_size|group_segment_fixed_size):\s*(\d+)", l)
            if m and m.group(1) not in meta and name in "".join(lines[max(0, lines.index(l) - 40):lines.index(l)]):
                meta[m.group(1)] = int(m.group(2))
        print(name[:90], dict(cnt))


if __name__ == "__main__":
    main()
