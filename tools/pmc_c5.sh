# PMC traffic of the var-size encode (C3 / C5), separate FETCH / WRITE passes
set -u
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp; mkdir -p "$R/gpurun_out"
for c in FETCH_SIZE WRITE_SIZE; do
  SB_REPS=3 timeout -s KILL 150 rocprofv3 --pmc $c -d "$R/gpurun_out/pmc_var_$c" -o run --output-format csv -- python3 "$R/tools/sbench.py" C3 C5 > "$R/gpurun_out/pmc_var_$c.log" 2>&1
  rc=$?; echo "$c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
