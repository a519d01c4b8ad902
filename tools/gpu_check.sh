set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python tools/kbench.py M C2 C4 > gpurun_out/kbench.log 2>&1
rc=$?; echo "kbench rc=$rc"; cat gpurun_out/kbench.log | grep -v amdgpu.ids
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/pytest_gpu.log
