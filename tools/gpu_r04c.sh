#!/bin/bash
# fixed decoder A/B: decode parity tests, then M / C4 / C2 decode with and without the 16-B unit path
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "decode or golden" > gpurun_out/t_dec.log 2>&1 || { tail -30 gpurun_out/t_dec.log; exit 3; }
tail -2 gpurun_out/t_dec.log
line() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['kernel_ms'], d['roofline']['frac'], (d.get('parity') or {}).get('result'))" "$@"; }
for rep in 1 2; do for c in M C4 C2; do for w16 in 1 0; do
  PACKOS_DEC_W16=$w16 timeout -k 10 200 python bench.py --config $c --op decode --steps 20 --warmup 3 --no-warm > gpurun_out/b_${c}_dec_w16$w16.json 2> gpurun_out/b_${c}_dec_w16$w16.err || exit 6
  line gpurun_out/b_${c}_dec_w16$w16.json "$c decode w16=$w16"
done; done; done
