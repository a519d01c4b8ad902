# GPU check: parity suite, then encode/decode timings for the var and decode paths.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/vbench.py ${VB_ARGS:-C3 C5 M C4} > gpurun_out/vbench.log 2>&1
rc=$?; echo "vbench rc=$rc"; grep -v amdgpu.ids gpurun_out/vbench.log
exit $rc
