# Round-3 pass C: decode/get-related GPU tests, then evidence for C3/C5/C4
# decode, C5 get, M get (SPECS), then the frame-less ablation on C5 once.
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${PYK:-decode or get or host or pipeline or map or round}" > gpurun_out/pytest_sel.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_sel.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
SPECS="${SPECS:-C3:decode C5:decode C5:get M:get C4:decode}" bash "$R/tools/prof_ops.sh" || exit $?
if [ -f "$R/abl/libpackos_noframe.so" ] && [ "${ABL:-1}" = 1 ]; then
  PACKOS_LIB="$R/abl/libpackos_noframe.so" timeout -k 10 300 python bench.py --config C5 --steps 10 --no-cpu --no-host --no-warm > gpurun_out/abl_noframe_C5.log 2>&1
  echo "ablation noframe C5 rc=$?"; grep '^{' gpurun_out/abl_noframe_C5.log | cut -c1-400
fi
exit 0
