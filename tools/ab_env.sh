#!/bin/bash
# Cold A/B of the in-tree library under environment variants, interleaved
# (variant 1, 2, ..., 1, 2, ... for REPS rounds) so box drift hits every
# variant alike.  One line per run into gpurun_out/$OUT/ab.txt.
#   OUT=x CFG=C5 OP=encode REPS=3 ENVS="PACKOS_FLAT_SLICE=0;PACKOS_FLAT_SLICE=16384" tools/ab_env.sh
set -u
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${OUT:-ab}; mkdir -p $O
IFS=';' read -ra EV <<< "${ENVS:-X=0}"
for r in $(seq 1 ${REPS:-2}); do
  for e in "${EV[@]}"; do
    env $e timeout -k 10 ${TLIM:-300} python bench.py --config ${CFG:-C5} --op ${OP:-encode} --no-cpu --no-host --no-warm \
      --steps ${STEPS:-20} --warmup 3 ${EXTRA:-} > $O/run.log 2>&1
    rc=$?
    res=$(grep '^{' $O/run.log | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['kernel_ms'], d['roofline']['frac'], d['passes']['kernel_ms'], (d.get('parity') or {}).get('result'))" 2>/dev/null)
    echo "${CFG:-C5} ${OP:-encode} rep$r [$e] rc=$rc $res" | tee -a $O/ab.txt
    [ $rc -eq 0 ] || exit $rc
  done
done
