set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
KBENCH_COPY=0 KBENCH_TILES=8192,16384,32768 KBENCH_VARIANTS=v2=2,v4=4,v9=9,v10=10 timeout -k 10 600 python tools/kbench.py M C2 C4 > gpurun_out/kbench.log 2>&1
rc=$?; echo "kbench rc=$rc"; grep -v amdgpu.ids gpurun_out/kbench.log
