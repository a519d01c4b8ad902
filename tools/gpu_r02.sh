# Round-2 GPU pass: parity suite, smoke, cold/warm bench line, rocprofv3
# kernel trace of the cold loop, FETCH_SIZE / WRITE_SIZE in separate --pmc
# passes (no trace domains).  CFG=M by default.
set -u
R="$GRAFT_REPO_ROOT"
CFG=${CFG:-M}
cd "$R"; mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python bench.py --config $CFG > gpurun_out/bench_$CFG.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_$CFG.log | tail -2
[ $rc -eq 0 ] || exit $rc
[ "${PROF:-1}" = 1 ] || exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$CFG" -o run --output-format csv -- python3 "$R/bench.py" --config $CFG --steps 50 --warmup 5 --no-cpu --no-host --no-warm > "$R/gpurun_out/prof_$CFG.log" 2>&1
rc=$?; echo "rocprof trace rc=$rc"; grep -v amdgpu.ids "$R/gpurun_out/prof_$CFG.log" | tail -1; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_fetch_$CFG" -o run --output-format csv -- python3 "$R/bench.py" --config $CFG --steps 12 --warmup 3 --no-cpu --no-host --no-warm > "$R/gpurun_out/pmc_fetch_$CFG.log" 2>&1
rc=$?; echo "rocprof fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmc_write_$CFG" -o run --output-format csv -- python3 "$R/bench.py" --config $CFG --steps 12 --warmup 3 --no-cpu --no-host --no-warm > "$R/gpurun_out/pmc_write_$CFG.log" 2>&1
rc=$?; echo "rocprof write rc=$rc"
exit $rc
