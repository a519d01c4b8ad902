# Quick GPU check: a pytest selection (-k EXPR) + optional config bench.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
K=${K:-"configs_vs_oracle or var_ or random_schema_encode or size_pass or stream_plan or overflow or empty_batch or host_batch or capacity"}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/pytest_quick.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_quick.log
[ $rc -eq 0 ] || exit $rc
for c in ${BENCH:-}; do
  timeout -k 10 300 python bench.py --config $c --no-cpu --no-host --steps 30 > gpurun_out/bench_$c.log 2>&1
  rc=$?; echo "bench $c rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_$c.log | tail -1 | cut -c1-900
  [ $rc -eq 0 ] || exit $rc
done
exit 0
