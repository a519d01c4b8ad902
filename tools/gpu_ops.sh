# Decode and GetAccess lines (cold) for the fixed-layout configs and M / C3 / X1
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; : > gpurun_out/ops.jsonl
for spec in "M decode" "C2 decode" "C4 decode" "M get" "C3 get" "C5 get"; do
  set -- $spec
  timeout -k 10 300 python bench.py --config $1 --op $2 --steps 20 > gpurun_out/ops_$1_$2.log 2>&1
  rc=$?; echo "$1 $2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' gpurun_out/ops_$1_$2.log | tail -1 >> gpurun_out/ops.jsonl
done
