# Kernel-level breakdown of the var encode / decode paths (rocprofv3 kernel trace).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_var -o run --output-format csv -- python3 tools/vbench.py ${VB_ARGS:-C3 C5} > gpurun_out/prof_var.log 2>&1
rc=$?; echo "rocprof rc=$rc"; grep -v amdgpu.ids gpurun_out/prof_var.log | tail -8
f=$(find gpurun_out/prof_var -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cut -d, -f1-8 "$f" | head -20
exit $rc
