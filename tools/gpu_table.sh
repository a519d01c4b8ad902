#!/bin/bash
# Evidence pass: GPU suite + smoke (TESTS=1), then the per-config table:
# encode (CPU baseline + parity + host legs), decode, validate and GetInt
# lines with whole-shard parity, cold -> gpurun_out/$OUT/table.jsonl
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/${OUT:-table}; mkdir -p $O
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
: > $O/table.jsonl
for c in ${CFGS:-M C1 C2 C3 C4 C5 X1}; do
  for op in ${OPS:-encode decode validate get}; do
    [ $op = get ] && [ $c = C1 -o $c = X1 ] && continue
    extra=""; [ $op = encode ] && extra="--cpu-seconds ${CPUS:-5}"
    timeout -k 10 400 python bench.py --config $c --op $op --steps ${STEPS:-20} $extra > $O/t_${op}_$c.log 2>&1
    rc=$?; echo "$op $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
    grep '^{' $O/t_${op}_$c.log | tail -1 >> $O/table.jsonl
  done
done
timeout -k 10 300 python bench.py > $O/default.log 2>&1; rc=$?; echo "default rc=$rc"
exit $rc
