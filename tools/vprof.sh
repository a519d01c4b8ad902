# Debug build of libpackos with per-phase clocks of k_encode_tiles
# (-DPACKOS_PHASE_PROF): gpurun_out/libpackos_prof.so; run a config through it.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for c in ${CFGS:-C3 C5}; do
  PACKOS_LIB=$PWD/packos_amd/libpackos_prof.so timeout -k 10 200 python bench.py --config $c --no-cpu --no-host --no-warm --steps 3 --warmup 1 ${BARGS:-} > gpurun_out/vprof_$c.log 2>&1
  rc=$?; echo "vprof $c rc=$rc"; grep -v amdgpu.ids gpurun_out/vprof_$c.log | grep "k_encode_tiles" | tail -2
  grep -v amdgpu.ids gpurun_out/vprof_$c.log | tail -1 | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
done
