# Extended-mode GPU tests + a regression selection of the parity suite.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ext.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ext.log 2>&1
rc=$?; echo "ext rc=$rc"; tail -30 gpurun_out/pytest_ext.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "all rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
exit $rc
