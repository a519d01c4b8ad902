#!/bin/bash
# Run GPU steps in order on the box, each under its own time limit, output to
# gpurun_out/$OUT/<name>.log.  A step ending with rc 0 or 1 (e.g. pytest with
# failing tests) lets the next one start; any other rc (timeout, abort, fault)
# ends the call there.
#   OUT=r06a tools/gpu_steps.sh "suite|900|python -u -m pytest tests -m gpu -q" "bench|300|python bench.py"
set -u
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${OUT:-steps}; mkdir -p $O
for step in "$@"; do
  name=${step%%|*}; rest=${step#*|}; lim=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($lim s): $cmd"
  timeout -k 10 $lim bash -c "$cmd" > $O/$name.log 2>&1
  rc=$?; echo "== $name rc=$rc"; tail -4 $O/$name.log
  [ $rc -le 1 ] || exit $rc
done
exit 0
