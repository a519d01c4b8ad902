#!/bin/bash
# persistent double-buffered fixed decode: GPU suite, then cold A/B against
# abl/libpackos_old.so (the one-tile-per-workgroup decoder)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 720 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_h.log 2>&1 || { tail -30 gpurun_out/pytest_h.log; exit 5; }
tail -2 gpurun_out/pytest_h.log
SPECS="${SPECS:-C2:decode M:decode C4:decode}" STEPS=20 bash tools/gpu_abl_multi.sh
