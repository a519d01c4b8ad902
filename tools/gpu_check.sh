set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 ./tools/membench > gpurun_out/membench.log 2>&1
rc=$?; echo "membench rc=$rc"; cat gpurun_out/membench.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_M" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 3 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/prof_M.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 "$GRAFT_REPO_ROOT/gpurun_out/prof_M.log"
