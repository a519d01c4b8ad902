# Parity selection of the encode tests against each abl/libpackos_<v>.so in
# $VARS (PACKOS_LIB), then the cold A/B of tools/gpu_ab_ops.sh.
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
for v in ${VARS}; do
  PACKOS_LIB=$R/abl/libpackos_$v.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${PYK:-random_schema_encode or var_ or configs_vs_oracle or golden_encode or checked_schema_encode or config_roundtrip}" > gpurun_out/pytest_abl_$v.log 2>&1
  rc=$?; echo "pytest $v rc=$rc"; tail -3 gpurun_out/pytest_abl_$v.log
  [ $rc -eq 0 ] || exit $rc
done
bash tools/gpu_ab_ops.sh
