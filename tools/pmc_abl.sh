# SQ instruction counts of k_encode_tiles for every abl/*.so on C3 (one --pmc pass each)
set -u
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp
for so in "$R"/abl/libpackos_*.so; do
  v=$(basename $so .so)
  PACKOS_LIB=$so timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_INSTS_VMEM -d "$R/gpurun_out/pmc_abl_$v" -o run --output-format csv -- python3 "$R/bench.py" --config ${CFG:-C3} --steps 4 --warmup 1 --no-cpu --no-host --no-warm ${BARGS:-} > "$R/gpurun_out/pmc_abl_$v.log" 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 - "$R/gpurun_out/pmc_abl_$v/run_counter_collection.csv" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    if __import__("os").environ.get("KSUB", "k_encode_tiles") not in r["Kernel_Name"]: continue
    agg["t"][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    med = {c: sorted(v)[len(v) // 2] for c, v in d.items()}
    w = med["SQ_WAVES"]
    print({c: round(v / w, 1) for c, v in sorted(med.items())})
PY
done
