#!/bin/bash
# flat encoder tile size (PACKOS_FT builds in abl/) on C5 encode, cold A/B
set -o pipefail
SPECS="${SPECS:-C5:encode}" STEPS=10 bash tools/gpu_abl_multi.sh
