#!/bin/bash
# fixed encode with 24-KiB tiles (k_encode_fixed_tile<24>): encode parity tests,
# then cold env A/B on M / C4 / C2 encode
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "fixed or encod or tail" --timeout 120 --timeout-method thread > gpurun_out/pytest_o.log 2>&1 || { tail -30 gpurun_out/pytest_o.log; exit 5; }
tail -2 gpurun_out/pytest_o.log
for c in M C4 C2; do CFG=$c OP=encode VAR=PACKOS_TILE_BYTES VALS="default 24576" bash tools/gpu_env_ab.sh || exit 6; done
