#!/bin/bash
# round-4 check of the load-ordering change: GPU suite, then a cold A/B of the
# previous library (abl/libpackos_old.so) over decode / get / var-encode lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 720 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_e.log 2>&1 || { tail -30 gpurun_out/pytest_e.log; exit 5; }
tail -2 gpurun_out/pytest_e.log
SPECS="${SPECS:-M:decode C2:decode C3:decode C4:decode C3:encode C5:encode M:get C5:decode}" STEPS=20 bash tools/gpu_abl_multi.sh
