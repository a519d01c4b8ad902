#!/bin/bash
# GPU suite (or a subset: TESTS="tests/test_x.py ..." / KEXPR="-k expr") -> gpurun_out/<OUT>/pytest_gpu.log
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${OUT:-tests}; mkdir -p $OUT
timeout -k 10 ${TLIM:-1000} python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread ${KEXPR:-} > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; exit $rc
