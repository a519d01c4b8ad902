# A/B of library builds: for each LIB in $LIBS (files under packos_amd/), run
# bench.py for each config in $CFGS with PACKOS_LIB pointing at it.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for L in $LIBS; do for c in ${CFGS:-C3 C5}; do
  PACKOS_LIB=$PWD/packos_amd/$L timeout -k 10 300 python bench.py --config $c --no-cpu --no-host --no-warm --steps ${STEPS:-20} > gpurun_out/ab_${L}_$c.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$L $c rc=$rc"; tail -3 gpurun_out/ab_${L}_$c.log; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_${L}_$c.log').read().strip().splitlines()[-1]); print('$L $c', d['kernel_ms'], d['roofline']['frac'])"
done; done
