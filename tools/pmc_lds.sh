# LDS bank conflicts of the fixed-layout decode and encode (metric M), one --pmc pass each
set -u
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp; mkdir -p "$R/gpurun_out"
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAVES SQ_BUSY_CYCLES -d "$R/gpurun_out/pmc_lds" -o run --output-format csv -- python3 "$R/tools/dbench.py" M > "$R/gpurun_out/pmc_lds.log" 2>&1
rc=$?; echo "lds rc=$rc"; exit $rc
