# A/B timing of libpackos variants (PACKOS_LIB) on bench configs (cold sets).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for lib in ${LIBS:-libpackos}; do
  for c in ${CFGS:-C3 C5}; do
    PACKOS_LIB=$PWD/packos_amd/$lib.so timeout -k 10 200 python bench.py --config $c --no-cpu --no-host --no-warm --steps ${STEPS:-20} --warmup 3 ${BARGS:-} > gpurun_out/abl_${lib}_$c.log 2>&1
    rc=$?; echo "$lib $c rc=$rc $(grep -v amdgpu.ids gpurun_out/abl_${lib}_$c.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernel_ms"], d["roofline"]["frac"])' 2>&1 | tail -1)"
    [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
