#!/bin/bash
# cold bench lines of SPECS (cfg:op) under each environment setting of ENVS
# ("-" = none; "K=V,K2=V2" = several), interleaved REP times -> gpurun_out/sweep.jsonl
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; : > gpurun_out/sweep.jsonl
for spec in ${SPECS:-C2:decode}; do
  c=${spec%%:*}; op=${spec##*:}
  for rep in $(seq ${REP:-2}); do
    for e in ${ENVS:--}; do
      E=""; [ "$e" != "-" ] && E="${e//,/ }"
      env $E timeout -k 10 300 python bench.py --config $c --op $op --steps ${STEPS:-20} --no-cpu --no-host --no-warm > gpurun_out/sw.log 2>&1
      rc=$?; [ $rc -eq 0 ] || { echo "$c $op $e rc=$rc"; tail -3 gpurun_out/sw.log; exit $rc; }
      python3 -c "import json,sys; l=json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1]); print(sys.argv[2], sys.argv[3], sys.argv[4], l['kernel_ms'], l['roofline']['frac'], l.get('parity',{}).get('result') if l.get('parity') else '')" gpurun_out/sw.log $c $op "$e" | tee -a gpurun_out/sweep.jsonl
    done
  done
done
