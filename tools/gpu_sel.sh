# GPU pytest selection: K="expr" (required)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/pytest_sel.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_sel.log
exit $rc
