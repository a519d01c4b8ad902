#!/bin/bash
# fixed decode tile bytes between 16 and 24 KB (M / C4: 80-row tiles admit 7 workgroups per CU)
set -o pipefail
for c in M C4; do CFG=$c OP=decode VAR=PACKOS_DEC_TILE_BYTES VALS="default 20480 28672" bash tools/gpu_env_ab.sh || exit 6; done
