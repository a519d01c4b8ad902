# SQ counters (one --pmc pass, <= 8 SQ counters) of bench.py --config $CFG
set -u
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp
CFG=${CFG:-C3}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA -d "$R/gpurun_out/pmc_sq_$CFG" -o run --output-format csv -- python3 "$R/bench.py" --config $CFG --steps 6 --warmup 2 --no-cpu --no-host --no-warm ${BARGS:-} > "$R/gpurun_out/pmc_sq_$CFG.log" 2>&1
rc=$?; echo "pmc sq $CFG rc=$rc"
python3 - "$R/gpurun_out/pmc_sq_$CFG/run_counter_collection.csv" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    k = r["Kernel_Name"].split("(")[0].split("::")[-1]
    agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    med = {c: sorted(v)[len(v) // 2] for c, v in d.items()}
    wc = med.get("SQ_WAVE_CYCLES", 1) or 1
    print(k, {c: round(v / wc, 3) if c not in ("SQ_WAVES", "SQ_WAVE_CYCLES") else v for c, v in sorted(med.items())})
PY
exit $rc
