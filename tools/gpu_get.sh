# GetAccess typed-gather figures (bench --op get) + rocprofv3 kernel stats of k_get_field.
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
for c in M C3; do
  timeout -k 10 300 python bench.py --config $c --op get --steps 20 > gpurun_out/get_$c.log 2>&1
  rc=$?; echo "get $c rc=$rc"; grep '^{' gpurun_out/get_$c.log | tail -1 | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_get" -o run --output-format csv -- python3 "$R/bench.py" --config M --op get --steps 20 --no-warm > "$R/gpurun_out/prof_get.log" 2>&1
rc=$?; echo "rocprof get rc=$rc"; cut -d, -f1-4 "$R/gpurun_out/prof_get/run_kernel_stats.csv" | head -4
exit $rc
