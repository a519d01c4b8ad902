set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
KBENCH_COPY=1 KBENCH_TILES=16384,8192 KBENCH_VARIANTS=v1=1,v2=2,v3=3,v4=4,v9=9,v10=10,v6=6,v8=8 timeout -k 10 600 python tools/kbench.py M C2 C4 > gpurun_out/kbench.log 2>&1
rc=$?; echo "kbench rc=$rc"; grep -v amdgpu.ids gpurun_out/kbench.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
