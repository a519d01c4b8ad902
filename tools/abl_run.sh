# Time every abl/libpackos_*.so on the cold encode bench (configs in CFGS).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; : > gpurun_out/abl.txt
for c in ${CFGS:-C3 C5}; do
  for so in abl/libpackos_*.so; do
    v=$(basename $so .so)
    PACKOS_LIB=$PWD/$so timeout -k 10 200 python bench.py --config $c --no-cpu --no-host --no-warm --steps ${STEPS:-30} --warmup 3 ${BARGS:-} > gpurun_out/abl_${c}_$v.log 2>&1
    rc=$?
    ms=$(grep '^{' gpurun_out/abl_${c}_$v.log | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['config'].get('op',''), d['kernel_ms'] if 'kernel_ms' in d else d['ms_per_step'], d.get('roofline',{}).get('frac'))" 2>/dev/null)
    echo "$c $v rc=$rc $ms" | tee -a gpurun_out/abl.txt
    [ $rc -eq 0 ] || exit $rc
  done
done
