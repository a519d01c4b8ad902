#!/bin/bash
# SQ counters (3 groups) of one kernel of a bench line:  CFG=M OP=decode KSUB=k_decode_fixed tools/pmc_sq.sh
set -u
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp; mkdir -p "$R/gpurun_out"
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_INSTS_VMEM"
G2="SQ_WAVES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU"
G3="SQ_WAVES SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC"
tag=${TAG:-${CFG}_${OP}}
for g in 1 2 3; do
  eval ctr=\$G$g
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d "$R/gpurun_out/pmc_${tag}_$g" -o run --output-format csv -- python3 "$R/bench.py" --config $CFG --op $OP --steps 3 --warmup 1 --no-cpu --no-host --no-warm --sets 1 > "$R/gpurun_out/pmc_${tag}_$g.log" 2>&1
  rc=$?; echo "$tag group $g rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$R/gpurun_out/pmc_${tag}_$g.log"; exit $rc; }
  KSUB=$KSUB python3 - "$R/gpurun_out/pmc_${tag}_$g/run_counter_collection.csv" <<'PY'
import csv, sys, collections, os
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    if os.environ["KSUB"] not in r["Kernel_Name"]: continue
    agg[r["Kernel_Name"][:48]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    med = {c: sorted(v)[len(v) // 2] for c, v in d.items()}
    w = med["SQ_WAVES"]
    print(k, "waves", w, {c: round(v / w, 1) for c, v in sorted(med.items()) if c != "SQ_WAVES"})
PY
done
