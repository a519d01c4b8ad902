#!/bin/bash
# cold A/B of abl/libpackos_*.so builds against the in-tree library:  CFG=C5 OP=encode tools/gpu_abl_lib.sh
set -o pipefail
mkdir -p gpurun_out
line() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['kernel_ms'], d['roofline']['frac'])" "$@"; }
for rep in 1 2; do for so in head abl/libpackos_*.so; do
  nm=$(basename $so .so)
  if [ $so = head ]; then unset PACKOS_LIB; else export PACKOS_LIB=$PWD/$so; fi
  timeout -k 10 200 python bench.py --config ${CFG:-C5} --op ${OP:-encode} --steps ${STEPS:-10} --warmup 2 --no-warm --no-cpu --no-host > gpurun_out/ab_$nm.json 2> gpurun_out/ab_$nm.err || { tail -3 gpurun_out/ab_$nm.err; exit 6; }
  line gpurun_out/ab_$nm.json "${CFG:-C5} ${OP:-encode} $nm"
done; done
