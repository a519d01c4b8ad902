# Cold A/B of bench.py --op OPS lines: the in-tree libpackos vs abl/libpackos_<v>.so for v in $VARS,
# interleaved REP times per config (kernel_ms + frac), after a pytest selection.
# HEADENV="K=V ...": extra environment for the head runs only (tuning knobs); ALLENV: for every run.
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
if [ -n "${PYK:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$PYK" > gpurun_out/pytest_ab.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_ab.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
: > gpurun_out/ab.jsonl
for spec in ${SPECS:-C3:decode C5:decode}; do
  c=${spec%%:*}; op=${spec##*:}
  for rep in $(seq ${REP:-2}); do
    for v in ${VARS:-base} head; do
      if [ $v = head ]; then L=""; else L="$R/abl/libpackos_$v.so"; fi
      HE="${ALLENV:-}"; [ $v = head ] && HE="$HE ${HEADENV:-}"
      env $HE PACKOS_LIB=$L timeout -k 10 300 python bench.py --config $c --op $op --steps ${STEPS:-20} --no-cpu --no-host --no-warm > gpurun_out/ab_${c}_${op}_$v.log 2>&1
      rc=$?; [ $rc -eq 0 ] || { echo "$c $op $v rc=$rc"; tail -3 gpurun_out/ab_${c}_${op}_$v.log; exit $rc; }
      python3 -c "import json,sys; l=json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1]); print(sys.argv[2], sys.argv[3], sys.argv[4], l['kernel_ms'], l['roofline']['frac'], l['roofline'].get('frac_granularity'), l.get('parity'))" gpurun_out/ab_${c}_${op}_$v.log $c $op $v | tee -a gpurun_out/ab.jsonl
    done
  done
done
exit 0
