# PMC traffic of the fixed-layout decode (metric M), separate FETCH / WRITE passes
set -u
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp; mkdir -p "$R/gpurun_out"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_dfetch" -o run --output-format csv -- python3 "$R/tools/dbench.py" M > "$R/gpurun_out/pmc_dfetch.log" 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmc_dwrite" -o run --output-format csv -- python3 "$R/tools/dbench.py" M > "$R/gpurun_out/pmc_dwrite.log" 2>&1
rc=$?; echo "write rc=$rc"; exit $rc
