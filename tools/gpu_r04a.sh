#!/bin/bash
# round-4 check: flat-encoder tests first (new streaming kernel), full GPU
# suite, then C5 encode (streaming vs chunk-gather) and M / C5 decode + get
# bench lines with whole-shard parity
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_flat.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_flat.log 2>&1 || { tail -30 gpurun_out/t_flat.log; exit 3; }
tail -3 gpurun_out/t_flat.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 4; }
tail -3 gpurun_out/t_all.log
for w in 12288 0 8192 16384; do
  PACKOS_FLAT_W=$w timeout -k 10 200 python bench.py --config C5 --steps 10 --warmup 2 --no-warm --no-cpu --no-host > gpurun_out/b_C5_enc_w$w.json 2> gpurun_out/b_C5_enc_w$w.err || exit 5
  python -c "import json;d=json.load(open('gpurun_out/b_C5_enc_w$w.json'));print('C5 W=$w', d['kernel_ms'], d['roofline']['frac'])"
done
for c in M C5; do for op in decode get; do
  timeout -k 10 200 python bench.py --config $c --op $op --steps 20 --warmup 3 --no-warm > gpurun_out/b_${c}_${op}.json 2> gpurun_out/b_${c}_${op}.err || exit 6
  python -c "import json;d=json.load(open('gpurun_out/b_${c}_${op}.json'));print('$c $op', d['kernel_ms'], d['roofline']['frac'], d['parity']['result'])"
done; done
