# C3 encode experiments: cold A/B of abl variants, then SQ wait / instruction-fetch counters
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
SPECS="${SPECS:-C3:encode}" VARS="${VARS:-or}" REP=${REP:-3} bash tools/gpu_ab_ops.sh || exit $?
[ -n "${NOPMC:-}" ] && exit 0
cd /tmp && export TMPDIR=/tmp
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY" "SQ_WAVES SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH"; do
  tag=$(echo $ctr | awk '{print $NF}')
  for v in head ${VARS:-or}; do
    if [ $v = head ]; then L=""; else L="$R/abl/libpackos_$v.so"; fi
    PACKOS_LIB=$L timeout -s KILL 90 rocprofv3 --pmc $ctr -d "$R/gpurun_out/c3pmc_${v}_$tag" -o run --output-format csv -- python3 "$R/bench.py" --config ${CFG:-C3} --steps 4 --warmup 1 --no-cpu --no-host --no-warm > "$R/gpurun_out/c3pmc_${v}_$tag.log" 2>&1
    rc=$?; echo "pmc $v $tag rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$R/gpurun_out/c3pmc_${v}_$tag.log"; exit $rc; }
    python3 - "$R/gpurun_out/c3pmc_${v}_$tag/run_counter_collection.csv" $v <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    if "k_encode_tiles" in r["Kernel_Name"]:
        d[r["Counter_Name"]].append(float(r["Counter_Value"]))
med = {c: sorted(v)[len(v) // 2] for c, v in d.items()}
w = med.get("SQ_WAVES", 1)
print(sys.argv[2], {c: (round(v / w, 1), v) for c, v in sorted(med.items())})
PY
  done
done
exit 0
