# Parity selection on the in-tree library, then cold A/B of abl/*.so.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
K=${K:-"var_ or random_schema_encode or size_pass or configs_vs_oracle or overflow or capacity or host_batch or checked_schema_encode or roundtrip"}
env ${TESTLIB:+PACKOS_LIB=$PWD/$TESTLIB} timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/pytest_ab.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_ab.log
[ $rc -eq 0 ] || exit $rc
bash tools/abl_run.sh
