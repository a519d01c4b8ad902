#!/bin/bash
# cold A/B of abl/libpackos_*.so against the in-tree library over several lines:
#   SPECS="M:encode M:decode C3:encode C5:encode" tools/gpu_abl_multi.sh
set -o pipefail
mkdir -p gpurun_out
line() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['kernel_ms'], d['roofline']['frac'])" "$@"; }
for rep in 1 2; do for spec in $SPECS; do c=${spec%%:*}; op=${spec##*:}; for so in head abl/libpackos_*.so; do
  nm=$(basename $so .so)
  if [ $so = head ]; then unset PACKOS_LIB; else export PACKOS_LIB=$PWD/$so; fi
  timeout -k 10 200 python bench.py --config $c --op $op --steps ${STEPS:-20} --warmup 3 --no-warm --no-cpu --no-host > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -3 gpurun_out/ab.err; exit 6; }
  line gpurun_out/ab.json "$c $op $nm"
done; done; done
