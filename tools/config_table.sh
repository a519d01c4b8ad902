# Per-config table: cold encode line (CPU baseline + parity +
# host legs) and cold decode line for every BASELINE config, one JSON line each
# into gpurun_out/table.jsonl.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; : > gpurun_out/table.jsonl
for c in ${CFGS:-C1 C2 C3 C4 C5 M}; do
  timeout -k 10 400 python bench.py --config $c --steps ${STEPS:-20} --cpu-seconds ${CPUS:-5} > gpurun_out/t_enc_$c.log 2>&1
  rc=$?; echo "enc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' gpurun_out/t_enc_$c.log | tail -1 >> gpurun_out/table.jsonl
  timeout -k 10 300 python bench.py --config $c --op decode --steps ${STEPS:-20} > gpurun_out/t_dec_$c.log 2>&1
  rc=$?; echo "dec $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' gpurun_out/t_dec_$c.log | tail -1 >> gpurun_out/table.jsonl
done
exit 0
