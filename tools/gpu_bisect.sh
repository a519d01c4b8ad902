# one pytest selection against each abl/libpackos_<v>.so (PACKOS_LIB) and the in-tree build
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/bisect
for v in ${VARS:-prev} head; do
  if [ $v = head ]; then L=""; else L="$PWD/abl/libpackos_$v.so"; fi
  PACKOS_LIB=$L timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -k "${PYK:-test_random_schema_encode}" > gpurun_out/bisect/$v.log 2>&1
  rc=$?; echo "$v rc=$rc $(tail -1 gpurun_out/bisect/$v.log)"
  [ $rc -le 1 ] || exit $rc
done
exit 0
