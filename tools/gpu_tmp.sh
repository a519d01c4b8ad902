set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
KBENCH_VARIANTS=v2=2,v14=14 KBENCH_COPY=0 timeout -k 10 200 python tools/kbench.py M C2 C4 2>&1 | grep -v amdgpu.ids
PACKOS_PIPE_WGS=4 KBENCH_VARIANTS=v14=14 KBENCH_COPY=0 timeout -k 10 200 python tools/kbench.py M 2>&1 | grep -v amdgpu.ids
