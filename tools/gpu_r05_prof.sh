#!/bin/bash
# round-5 evidence: default bench line + prof_ops (trace + FETCH/WRITE/SQ) for SPECS -> gpurun_out/
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r05p
timeout -k 10 400 python bench.py > gpurun_out/r05p/default.log 2>&1; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
grep '^{' gpurun_out/r05p/default.log | tail -1 | cut -c1-400
SPECS="${SPECS:-M:encode}" bash tools/prof_ops.sh
