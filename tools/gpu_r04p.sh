#!/bin/bash
# fixed encode with 24-KiB tiles (k_encode_fixed_tile<24>), cold env A/B with
# whole-shard parity on M / C4 / C2 encode
set -o pipefail
mkdir -p gpurun_out
line() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['kernel_ms'], d['roofline']['frac'], d['parity']['result'])" "$@"; }
for rep in 1 2; do for c in M C4 C2; do for v in default 24576; do
  if [ $v = default ]; then unset PACKOS_TILE_BYTES; else export PACKOS_TILE_BYTES=$v; fi
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-warm --cpu-seconds 2 --no-host > gpurun_out/p.json 2> gpurun_out/p.err || { tail -3 gpurun_out/p.err; exit 6; }
  line gpurun_out/p.json "$c encode TILE=$v"
done; done; done
