# rocprofv3 kernel trace of the var-size encode A/B (tools/sbench.py)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
SB_REPS=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stream -o run -- python3 tools/sbench.py ${SB_ARGS:-C3 C5} > gpurun_out/prof_stream.log 2>&1
rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/prof_stream.log | tail -3
f=$(find gpurun_out/prof_stream -name 'run_kernel_stats.csv' | head -1); cut -d, -f1-4 "$f" | head -20
exit $rc
