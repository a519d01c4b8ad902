#!/bin/bash
# full GPU suite + smoke + default bench line + C3 / C5 encode lines -> gpurun_out/$OUT/
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${OUT:-check}; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/default.log 2>&1; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
for c in ${CFGS:-C3 C5}; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --cpu-seconds 1 > $OUT/enc_$c.log 2>&1; rc=$?; echo "enc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
