set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r05v
timeout -k 10 600 python -u -m pytest tests/test_gpu_validate.py tests/test_c_abi_harness.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05v/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r05v/pytest.log; [ $rc -eq 0 ] || exit $rc
for c in C4 C2 M C3; do
  timeout -k 10 300 python bench.py --config $c --op validate --steps 20 > gpurun_out/r05v/v_$c.log 2>&1; rc=$?; echo "val $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python bench.py --config C4 --op decode --steps 20 --passes 5 > gpurun_out/r05v/d_C4_p5.log 2>&1; echo "p5 rc=$?"
timeout -k 10 300 python bench.py --config C4 --op decode --steps 20 --warmup 40 > gpurun_out/r05v/d_C4_w40.log 2>&1; echo "w40 rc=$?"
