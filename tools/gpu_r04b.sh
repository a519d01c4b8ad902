#!/bin/bash
# streaming flat encoder A/B: flat tests, C5 (window sizes, chunk-gather),
# C3 through the flat encoders (lane groups) vs the tile encoder
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_flat.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_flat.log 2>&1 || { tail -30 gpurun_out/t_flat.log; exit 3; }
tail -2 gpurun_out/t_flat.log
line() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['kernel_ms'], d['roofline']['frac'], (d.get('parity') or {}).get('result'))" "$@"; }
b() {  # name, config, env...
  local nm=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 2 --no-warm --no-cpu --no-host > gpurun_out/b_$nm.json 2> gpurun_out/b_$nm.err || exit 5
  line gpurun_out/b_$nm.json "$nm"
}
b C5_w8192 C5 PACKOS_FLAT_W=8192
b C5_w0 C5 PACKOS_FLAT_W=0
b C5_w4096 C5 PACKOS_FLAT_W=4096
b C5_w12288 C5 PACKOS_FLAT_W=12288
b C5_w8192_gl16 C5 PACKOS_FLAT_W=8192 PACKOS_FLAT_GL=16
b C3_tiles C3 PACKOS_ENC_FLAT=0
b C3_gl8_w4096 C3 PACKOS_ENC_FLAT=1 PACKOS_FLAT_GL=8 PACKOS_FLAT_W=4096
b C3_gl8_w8192 C3 PACKOS_ENC_FLAT=1 PACKOS_FLAT_GL=8 PACKOS_FLAT_W=8192
b C3_gl16_w4096 C3 PACKOS_ENC_FLAT=1 PACKOS_FLAT_GL=16 PACKOS_FLAT_W=4096
