# Issue-unit utilisation of one kernel: SQ cycle counters + GRBM_GUI_ACTIVE (one --pmc pass per group)
set -u
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_BRANCH"; do
  tag=$(echo $grp | awk '{print $2}')
  timeout -s KILL 90 rocprofv3 --pmc $grp -d "$R/gpurun_out/sq_$tag" -o run --output-format csv -- python3 "$R/bench.py" --config ${CFG:-C3} --op ${OP:-encode} --steps 4 --warmup 1 --no-cpu --no-host --no-warm > "$R/gpurun_out/sq_$tag.log" 2>&1
  rc=$?; echo "pmc $tag rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$R/gpurun_out/sq_$tag.log"; exit $rc; }
  python3 - "$R/gpurun_out/sq_$tag/run_counter_collection.csv" "${KSUB:-k_encode_tiles}" <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r["Kernel_Name"]:
        d[r["Counter_Name"]].append(float(r["Counter_Value"]))
print({c: sorted(v)[len(v) // 2] for c, v in sorted(d.items())})
PY
done
