#!/bin/bash
# fixed decode: column loops with two elements in flight, unswitched 16-B units,
# 8-wave variant under 128-B blobs: GPU suite, then cold A/B against abl/libpackos_old.so
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 720 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_i.log 2>&1 || { tail -30 gpurun_out/pytest_i.log; exit 5; }
tail -2 gpurun_out/pytest_i.log
SPECS="${SPECS:-M:decode C2:decode C4:decode}" STEPS=20 bash tools/gpu_abl_multi.sh
