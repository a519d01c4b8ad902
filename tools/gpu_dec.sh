# Decode timings (bench --op decode, cold) for CFGS.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for c in ${CFGS:-C3 C5 M}; do
  timeout -k 10 300 python bench.py --config $c --op decode --steps 20 --no-warm > gpurun_out/dec_$c.log 2>&1
  rc=$?; echo "dec $c rc=$rc $(grep '^{' gpurun_out/dec_$c.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernel_ms"], d["roofline"]["frac"])')"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
