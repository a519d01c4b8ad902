# SQ counters for the var encode/decode kernels (separate --pmc pass; no tracing domains).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc ${PMC:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS} -d gpurun_out/pmc_var -o run --output-format csv -- python3 tools/vbench.py ${VB_ARGS:-C3} > gpurun_out/pmc_var.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/pmc_var.log
exit $rc
