# SQ activity counters of the var-size stream encoder (C3), one --pmc pass
set -u
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp; mkdir -p "$R/gpurun_out"
SB_REPS=3 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d "$R/gpurun_out/pmc_sq" -o run --output-format csv -- python3 "$R/tools/sbench.py" C3 > "$R/gpurun_out/pmc_sq.log" 2>&1
rc=$?; echo "sq rc=$rc"; exit $rc
