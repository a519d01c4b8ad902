# Full GPU pass: parity suite, smoke, bench line, per-config table.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --e2e > gpurun_out/bench_full.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_full.log | tail -2
[ $rc -eq 0 ] || exit $rc
if [ "${CONFIGS:-1}" = 1 ]; then
timeout -k 10 600 python tools/config_bench.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err
rc=$?; echo "configs rc=$rc"; cat gpurun_out/configs.jsonl | cut -c1-400
fi
exit $rc
