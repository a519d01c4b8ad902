#!/bin/bash
# round-3 library vs HEAD on the same box: M / C4 / C2 decode and encode
set -o pipefail
mkdir -p gpurun_out
line() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['kernel_ms'], d['roofline']['frac'])" "$@"; }
for rep in 1 2; do for c in C4 M C2; do for op in decode encode; do for lib in r03 head; do
  if [ $lib = r03 ]; then export PACKOS_LIB=$PWD/abl/libpackos_r03.so; else unset PACKOS_LIB; fi
  timeout -k 10 200 python bench.py --config $c --op $op --steps 20 --warmup 3 --no-warm --no-cpu --no-host > gpurun_out/b_${c}_${op}_$lib.json 2> gpurun_out/b_${c}_${op}_$lib.err || { tail -3 gpurun_out/b_${c}_${op}_$lib.err; exit 6; }
  line gpurun_out/b_${c}_${op}_$lib.json "$c $op $lib"
done; done; done; done
