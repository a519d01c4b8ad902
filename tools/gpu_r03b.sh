# Round-3 pass: a pytest selection (PYK), then the evidence pass (gpu_r03a.sh).
# A failing test does not stop the profile; a crash / timeout / abort does.
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${PYK:-get or host or pipeline or map}" > gpurun_out/pytest_sel.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_sel.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash "$R/tools/gpu_r03a.sh"
