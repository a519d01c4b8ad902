timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "flat or configs_vs_oracle or config_roundtrip or decode or get" > gpurun_out/pytest_flat.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_flat.log; [ $rc -eq 0 ] || exit $rc
PACKOS_LIB=$PWD/abl/libpackos_fedge16.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "flat" > gpurun_out/pytest_fe16.log 2>&1; rc=$?; echo "fedge16 rc=$rc"; tail -3 gpurun_out/pytest_fe16.log; [ $rc -eq 0 ] || exit $rc
SPECS="C5:encode C3:decode" VARS="nofull" REP=3 bash tools/gpu_ab_ops.sh || exit 1
SPECS="M:get C5:get" VARS="getnt" REP=2 bash tools/gpu_ab_ops.sh
