#!/bin/bash
# round-4 check: flat-encoder tests first (new streaming kernel), full GPU
# suite, then C5 encode (streaming window sizes vs chunk-gather), the fixed
# decoder's row padding A/B, and M / C5 decode + get lines with whole-shard parity
set -o pipefail
mkdir -p gpurun_out
#timeout -k 10 300 python -u -m pytest tests/test_gpu_flat.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_flat.log 2>&1 || { tail -30 gpurun_out/t_flat.log; exit 3; }
#tail -3 gpurun_out/t_flat.log
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1
rc=$?; grep -E "^FAILED|passed|failed" gpurun_out/t_all.log | tail -15
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit 4   # a crash / timeout: stop; test failures: go on to the benches
line() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['kernel_ms'], d['roofline']['frac'], (d.get('parity') or {}).get('result'))" "$@"; }
for w in 12288 0 8192 16384 4096; do
  PACKOS_FLAT_W=$w timeout -k 10 200 python bench.py --config C5 --steps 10 --warmup 2 --no-warm --no-cpu --no-host > gpurun_out/b_C5_enc_w$w.json 2> gpurun_out/b_C5_enc_w$w.err || exit 5
  line gpurun_out/b_C5_enc_w$w.json "C5 enc W=$w"
done
for c in M C2 C4; do for pad in 0 16; do
  PACKOS_DEC_PAD=$pad timeout -k 10 200 python bench.py --config $c --op decode --steps 20 --warmup 3 --no-warm > gpurun_out/b_${c}_dec_p$pad.json 2> gpurun_out/b_${c}_dec_p$pad.err || exit 6
  line gpurun_out/b_${c}_dec_p$pad.json "$c decode pad=$pad"
done; done
for c in M C5; do
  timeout -k 10 200 python bench.py --config $c --op get --steps 20 --warmup 3 --no-warm > gpurun_out/b_${c}_get.json 2> gpurun_out/b_${c}_get.err || exit 7
  line gpurun_out/b_${c}_get.json "$c get"
done
timeout -k 10 200 python bench.py --config C5 --op decode --steps 20 --warmup 3 --no-warm > gpurun_out/b_C5_decode.json 2> gpurun_out/b_C5_decode.err || exit 8
line gpurun_out/b_C5_decode.json "C5 decode"
