# Round-3 evidence pass, part A: FETCH_SIZE calibration of the scattered read
# shapes (tools/fetch_calib), then prof_ops.sh over SPECS.
set -u
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
if [ "${CALIB:-1}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 120 "$R/tools/fetch_calib" > "$R/gpurun_out/calib_plain.log" 2>&1
  rc=$?; echo "calib rc=$rc"; cat "$R/gpurun_out/calib_plain.log"; [ $rc -eq 0 ] || exit $rc
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/calib_fetch" -o run --output-format csv -- "$R/tools/fetch_calib" > "$R/gpurun_out/calib_fetch.log" 2>&1
  rc=$?; echo "calib pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
SPECS="${SPECS:-M:decode C2:decode C3:decode M:get C3:get}" bash "$R/tools/prof_ops.sh"
