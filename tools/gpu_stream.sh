# Stream-kernel check: var encode parity subset, then the A/B bench.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "${PYK:-encode or stream or tile or configs or golden}" > gpurun_out/pytest_stream.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_stream.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/sbench.py ${SB_ARGS:-C3 C5} > gpurun_out/sbench.log 2>&1
rc=$?; echo "sbench rc=$rc"; grep -v amdgpu.ids gpurun_out/sbench.log | tail -8
exit $rc
