#!/bin/bash
# fixed decode: column ranges per wave (small columns written by one wave):
# decode parity tests, then cold A/B against abl/libpackos_old.so
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "decode or fixed or roundtrip or golden" --timeout 120 --timeout-method thread > gpurun_out/pytest_n.log 2>&1 || { tail -30 gpurun_out/pytest_n.log; exit 5; }
tail -2 gpurun_out/pytest_n.log
SPECS="${SPECS:-M:decode C2:decode C4:decode}" STEPS=20 bash tools/gpu_abl_multi.sh
