# Round-3 end pass, part PART:
#   A: parity suite + smoke + per-config table (encode with CPU baseline,
#      parity and host legs; decode) for CFGS -> gpurun_out/table.jsonl
#   B: tools/prof_ops.sh evidence (line + rocprofv3 kernel trace + FETCH /
#      WRITE / SQ passes) for SPECS -> gpurun_out/p3/
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
if [ "${PART:-A}" = A ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
  CFGS="${CFGS:-M C1 C2 C3 C4 C5 X1}" bash tools/config_table.sh
  exit $?
fi
SPECS="${SPECS:-M:encode C3:encode C5:encode M:decode C3:decode C5:decode M:get C3:get C5:get}" bash tools/prof_ops.sh
