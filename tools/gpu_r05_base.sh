set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r05a
timeout -k 10 300 python bench.py > gpurun_out/r05a/default.log 2>&1; rc=$?; echo "default rc=$rc"; [ $rc -eq 0 ] || exit $rc
for c in C3 C5 C2; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --cpu-seconds 1 > gpurun_out/r05a/enc_$c.log 2>&1; rc=$?; echo "enc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for c in M C2; do
  timeout -k 10 300 python bench.py --config $c --op decode --steps 20 > gpurun_out/r05a/dec_$c.log 2>&1; rc=$?; echo "dec $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
