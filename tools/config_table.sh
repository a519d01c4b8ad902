# Per-config table: cold encode line (CPU baseline + parity +
# host legs) and cold decode / validate / get lines (whole-shard parity) for
# every BASELINE config, one JSON line each into gpurun_out/$OUT/table.jsonl.
#   CFGS="C1 C2 C3 C4 C5 M" OPS="decode validate get" tools/config_table.sh
set -u
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${OUT:-table}; mkdir -p $O; : > $O/table.jsonl
for c in ${CFGS:-C1 C2 C3 C4 C5 M}; do
  timeout -k 10 400 python bench.py --config $c --steps ${STEPS:-20} --cpu-seconds ${CPUS:-5} > $O/t_encode_$c.log 2>&1
  rc=$?; echo "encode $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' $O/t_encode_$c.log | tail -1 >> $O/table.jsonl
  for op in ${OPS:-decode}; do
    [ $c = C1 ] && [ $op = get ] && continue   # C1 has no int field GetInt reads
    timeout -k 10 300 python bench.py --config $c --op $op --steps ${STEPS:-20} > $O/t_${op}_$c.log 2>&1
    rc=$?; echo "$op $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
    grep '^{' $O/t_${op}_$c.log | tail -1 >> $O/table.jsonl
  done
done
exit 0
