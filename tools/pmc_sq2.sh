# Two SQ passes (<= 8 SQ counters each) of bench.py --config $CFG: wave states
# and instruction / LDS counts, normalised per wave cycle
set -u
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp
CFG=${CFG:-C3}
summ() {
python3 - "$1" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    k = r["Kernel_Name"].split("(")[0].split("::")[-1]
    agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    med = {c: sorted(v)[len(v) // 2] for c, v in d.items()}
    print(k[:60], {c: v for c, v in sorted(med.items())})
PY
}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA -d "$R/gpurun_out/pmc_sqa_$CFG" -o run --output-format csv -- python3 "$R/bench.py" --config $CFG --steps 6 --warmup 2 --no-cpu --no-host --no-warm > "$R/gpurun_out/pmc_sqa_$CFG.log" 2>&1
rc=$?; echo "pass a rc=$rc"; [ $rc -eq 0 ] || exit $rc
summ "$R/gpurun_out/pmc_sqa_$CFG/run_counter_collection.csv"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU -d "$R/gpurun_out/pmc_sqb_$CFG" -o run --output-format csv -- python3 "$R/bench.py" --config $CFG --steps 6 --warmup 2 --no-cpu --no-host --no-warm > "$R/gpurun_out/pmc_sqb_$CFG.log" 2>&1
rc=$?; echo "pass b rc=$rc"; [ $rc -eq 0 ] || exit $rc
summ "$R/gpurun_out/pmc_sqb_$CFG/run_counter_collection.csv"
