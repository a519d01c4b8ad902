# SQ counters (one --pmc pass each) of bench.py --op OP for the in-tree lib and
# abl/libpackos_$BASE.so, kernel filter KSUB, per-wave medians printed.
set -u
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp; mkdir -p "$R/gpurun_out"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_INSTS_VMEM"
for spec in ${SPECS:-C5:decode}; do
  c=${spec%%:*}; op=${spec##*:}
  for v in base head; do
    if [ $v = head ]; then L=""; else L="$R/abl/libpackos_${BASE:-base}.so"; fi
    PACKOS_LIB=$L timeout -s KILL 240 rocprofv3 --pmc $SQ -d "$R/gpurun_out/pmcab_${c}_${op}_$v" -o run --output-format csv -- python3 "$R/bench.py" --config $c --op $op --steps 6 --warmup 2 --no-cpu --no-host --no-warm > "$R/gpurun_out/pmcab_${c}_${op}_$v.log" 2>&1
    rc=$?; echo "$c $op $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python3 - "$R/gpurun_out/pmcab_${c}_${op}_$v" "${KSUB:-k_decode}" <<'PY'
import csv, glob, sys, collections
path = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
per = collections.defaultdict(float)
for r in csv.DictReader(open(path)):
    if sys.argv[2] in r["Kernel_Name"]:
        per[(r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
by = collections.defaultdict(list)
for (c, _), v in per.items(): by[c].append(v)
med = {c: sorted(v)[len(v) // 2] for c, v in by.items()}
w = med.get("SQ_WAVES", 1)
print({c: round(v / w, 1) for c, v in sorted(med.items()) if c != "SQ_WAVES"}, "waves", w)
PY
  done
done
