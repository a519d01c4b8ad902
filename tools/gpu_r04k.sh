#!/bin/bash
# fixed decode with LDS rows padded to B + 16 (PACKOS_DEC_PAD): the fixed-decode
# parity tests, then cold env A/B on M / C4 / C2 decode
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "fixed or decode" --timeout 120 --timeout-method thread > gpurun_out/pytest_k.log 2>&1 || { tail -30 gpurun_out/pytest_k.log; exit 5; }
tail -2 gpurun_out/pytest_k.log
for c in M C4 C2; do CFG=$c OP=decode VAR=PACKOS_DEC_PAD VALS="default 1" bash tools/gpu_env_ab.sh || exit 6; done
