# Var-size encode measurement pass: cold bench lines (C3, C5 full shard),
# rocprofv3 kernel stats of each, and the per-phase clocks of the debug build
# (packos_amd/libpackos_prof.so from tools/build_prof.sh).
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
for c in ${CFGS:-C3 C5}; do
  timeout -k 10 300 python bench.py --config $c --no-cpu --no-host --steps 20 --warmup 3 > gpurun_out/bench_$c.log 2>&1
  rc=$?; echo "bench $c rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_$c.log | tail -1 | cut -c1-1200; [ $rc -eq 0 ] || exit $rc
done
if [ "${PROF:-1}" = 1 ]; then
cd /tmp && export TMPDIR=/tmp
for c in ${CFGS:-C3 C5}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$c" -o run --output-format csv -- python3 "$R/bench.py" --config $c --steps 20 --warmup 3 --no-cpu --no-host --no-warm > "$R/gpurun_out/prof_$c.log" 2>&1
  rc=$?; echo "rocprof $c rc=$rc"; cut -d, -f1-4 "$R/gpurun_out/prof_$c/run_kernel_stats.csv" | head -5; [ $rc -eq 0 ] || exit $rc
done
cd "$R"
fi
if [ -f packos_amd/libpackos_prof.so ] && [ "${VPROF:-1}" = 1 ]; then
for c in ${CFGS:-C3 C5}; do
  PACKOS_LIB=$PWD/packos_amd/libpackos_prof.so timeout -k 10 200 python bench.py --config $c --no-cpu --no-host --no-warm --steps 3 --warmup 1 --sets 1 > gpurun_out/vprof_$c.log 2>&1
  rc=$?; echo "vprof $c rc=$rc"; grep "k_encode_tiles" gpurun_out/vprof_$c.log | tail -1; [ $rc -eq 0 ] || exit $rc
done
fi
exit 0
