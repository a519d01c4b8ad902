# Round-end GPU pass: parity suite + smoke + M bench with rocprof / PMC
# (tools/gpu_r02.sh), the per-config encode/decode table incl. X1, and
# rocprofv3 kernel stats of the var-size encoders (C3, C5, X1).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/gpu_r02.sh || exit $?
CFGS="${CFGS:-C1 C2 C3 C4 C5 X1}" bash tools/config_table.sh || exit $?
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp
for c in C3 C5 X1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_enc_$c" -o run --output-format csv -- python3 "$R/bench.py" --config $c --steps 10 --warmup 2 --no-cpu --no-host --no-warm > "$R/gpurun_out/prof_enc_$c.log" 2>&1
  rc=$?; echo "rocprof $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
