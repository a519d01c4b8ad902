#!/bin/bash
# bench order check: cold (headline) pass before the warm replay
set -o pipefail
mkdir -p gpurun_out
for spec in M:decode M:encode C4:decode C3:decode M:decode; do c=${spec%%:*}; op=${spec##*:}
  timeout -k 10 300 python bench.py --config $c --op $op --steps 20 --no-cpu --no-host > gpurun_out/l.json 2> gpurun_out/l.err || { tail -3 gpurun_out/l.err; exit 6; }
  python -c "import json;d=json.load(open('gpurun_out/l.json'));print('$c $op cold',d['kernel_ms'],'warm',d['warm']['kernel_ms'],d['parity']['result'])"
done
