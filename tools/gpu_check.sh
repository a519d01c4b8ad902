set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
KBENCH_COPY=0 timeout -k 10 600 python tools/kbench.py M C2 C4 > gpurun_out/kbench.log 2>&1
rc=$?; echo "kbench rc=$rc"; grep -v amdgpu.ids gpurun_out/kbench.log
