#!/bin/bash
# cold A/B of environment variants of one bench line:
#   CFG=C3 OP=encode VAR="PACKOS_EK4" VALS="default 1,5,6 2,5,6" tools/gpu_env_ab.sh
set -o pipefail
mkdir -p gpurun_out
line() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['kernel_ms'], d['roofline']['frac'])" "$@"; }
for rep in 1 2; do for v in $VALS; do
  if [ "$v" = default ]; then unset $VAR; else export $VAR=$v; fi
  timeout -k 10 200 python bench.py --config ${CFG:-C3} --op ${OP:-encode} --steps ${STEPS:-20} --warmup 3 --no-warm --no-cpu --no-host > gpurun_out/env_ab.json 2> gpurun_out/env_ab.err || { tail -3 gpurun_out/env_ab.err; exit 6; }
  line gpurun_out/env_ab.json "${CFG:-C3} ${OP:-encode} $VAR=$v"
done; done
