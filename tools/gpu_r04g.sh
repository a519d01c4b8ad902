#!/bin/bash
# decode occupancy A/B: abl/libpackos_w8.so (k_decode_fixed at 8 waves/SIMD, 64 VGPRs)
set -o pipefail
SPECS="C2:decode M:decode C4:decode" STEPS=20 bash tools/gpu_abl_multi.sh
