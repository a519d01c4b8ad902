set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
KBENCH_COPY=1 KBENCH_TILES=16384 KBENCH_VARIANTS=v2=2,v4=4,v6=6,v11=11,v12=12,v13=13,v1=1 timeout -k 10 600 python tools/kbench.py M C2 C4 > gpurun_out/kbench.log 2>&1
rc=$?; echo "kbench rc=$rc"; grep -v amdgpu.ids gpurun_out/kbench.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
