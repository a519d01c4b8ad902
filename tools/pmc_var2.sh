# PMC passes (one counter group per run, no trace domains) over the var
# encoder on config $CFG: traffic (FETCH_SIZE / WRITE_SIZE) and EA request mix.
set -u
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
CFG=${CFG:-C5}
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$R/gpurun_out/pmcv_${CFG}_$i" -o run --output-format csv -- python3 "$R/bench.py" --config $CFG --steps 4 --warmup 1 --no-cpu --no-host --no-warm ${BARGS:-} > "$R/gpurun_out/pmcv_${CFG}_$i.log" 2>&1
  rc=$?; echo "pmc $i ($grp) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
