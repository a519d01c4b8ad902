# Tile-size / LDS-budget sweep of the tiled var encode (run after the parity suite).
# SWEEP="vt,bud,in;vt,bud,in;..."
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
IFS=';' read -ra CFGS <<< "${SWEEP:-128,16384,16384;256,16384,16384;128,8192,12288;128,8192,8192}"
for cfg in "${CFGS[@]}"; do
  IFS=',' read -r vt bud inb <<< "$cfg"
  PACKOS_VAR_TILE=$vt PACKOS_VAR_BUD=$bud PACKOS_VAR_IN=$inb timeout -k 10 300 python tools/vbench.py ${VB_ARGS:-C3 C5} > gpurun_out/vsweep.log 2>&1 || exit $?
  echo "VT=$vt bud=$bud in=$inb"; grep -v amdgpu.ids gpurun_out/vsweep.log | sed 's/, "decode.*//'
done
