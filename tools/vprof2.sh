# Per-phase clocks (debug builds abl/prof/*.so, -DPACKOS_PHASE_PROF) on configs CFGS
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for c in ${CFGS:-C3}; do
  for so in abl/prof/*.so; do
    PACKOS_LIB=$PWD/$so timeout -k 10 200 python bench.py --config $c --no-cpu --no-host --no-warm --steps 3 --warmup 1 > gpurun_out/vprof2.log 2>&1
    rc=$?; echo "$c $(basename $so) rc=$rc"; grep "k_encode_tiles" gpurun_out/vprof2.log | tail -1
    [ $rc -eq 0 ] || exit $rc
  done
done
