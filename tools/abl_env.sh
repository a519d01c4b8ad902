# Cold C3/C5 encode of abl/*.so under environment variants (ENVS, ';'-separated)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; : > gpurun_out/abl_env.txt
IFS=';' read -ra EV <<< "${ENVS:-X=0;HIP_FORCE_DEV_KERNARG=1;HIP_FORCE_DEV_KERNARG=0}"
for c in ${CFGS:-C3}; do
  for so in abl/libpackos_*.so; do
    for e in "${EV[@]}"; do
      v=$(basename $so .so)
      env $e PACKOS_LIB=$PWD/$so timeout -k 10 200 python bench.py --config $c --no-cpu --no-host --no-warm --steps 30 --warmup 3 > gpurun_out/abl_env.log 2>&1
      rc=$?
      ms=$(grep '^{' gpurun_out/abl_env.log | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['kernel_ms'], d.get('roofline',{}).get('frac'))" 2>/dev/null)
      echo "$c $v $e rc=$rc $ms" | tee -a gpurun_out/abl_env.txt
      [ $rc -eq 0 ] || exit $rc
    done
  done
done
