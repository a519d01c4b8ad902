#!/bin/bash
# Round-4 evidence pass, part PART:
#   A: parity suite + smoke + per-config table (encode with CPU baseline,
#      parity and host legs; decode and GetInt with whole-shard parity)
#      -> gpurun_out/table.jsonl
#   B: tools/prof_ops.sh (line + rocprofv3 kernel trace + FETCH / WRITE / SQ
#      passes) for SPECS -> gpurun_out/p3/
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
if [ "${PART:-A}" = A ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
  : > gpurun_out/table.jsonl
  for c in ${CFGS:-M C1 C2 C3 C4 C5 X1}; do
    timeout -k 10 400 python bench.py --config $c --steps ${STEPS:-20} --cpu-seconds ${CPUS:-5} > gpurun_out/t_enc_$c.log 2>&1
    rc=$?; echo "enc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
    grep '^{' gpurun_out/t_enc_$c.log | tail -1 >> gpurun_out/table.jsonl
    for op in decode get; do
      [ $op = get ] && [ $c = C1 -o $c = X1 ] && continue
      timeout -k 10 300 python bench.py --config $c --op $op --steps ${STEPS:-20} > gpurun_out/t_${op}_$c.log 2>&1
      rc=$?; echo "$op $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
      grep '^{' gpurun_out/t_${op}_$c.log | tail -1 >> gpurun_out/table.jsonl
    done
  done
  exit 0
fi
SPECS="${SPECS:-M:encode C3:encode C5:encode M:decode C3:decode C5:decode M:get C5:get}" bash tools/prof_ops.sh
