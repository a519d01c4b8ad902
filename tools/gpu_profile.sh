# Round profile: bench line, rocprofv3 kernel-trace stats of the same command,
# then FETCH_SIZE and WRITE_SIZE in separate --pmc passes (no trace domains).
set -u
R="$GRAFT_REPO_ROOT"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python bench.py --e2e > gpurun_out/bench_full.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_full.log | tail -2
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_M" -o run --output-format csv -- python3 "$R/bench.py" --steps 50 --warmup 5 --no-cpu > "$R/gpurun_out/prof_M.log" 2>&1
rc=$?; echo "rocprof trace rc=$rc"; grep -v amdgpu.ids "$R/gpurun_out/prof_M.log" | tail -1; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_fetch" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu > "$R/gpurun_out/pmc_fetch.log" 2>&1
rc=$?; echo "rocprof fetch rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmc_write" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu > "$R/gpurun_out/pmc_write.log" 2>&1
rc=$?; echo "rocprof write rc=$rc"
exit $rc
