#!/bin/bash
# round-5 A/B driver: pytest selection + gpu_ab_ops (SPECS / VARS / REP) + optional phase clocks (VPROF=1)
set -u
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_ab_ops.sh; rc=$?; [ $rc -eq 0 ] || exit $rc
if [ "${VPROF:-0}" = 1 ]; then CFGS="${VCFGS:-C3}" bash tools/vprof2.sh; fi
