# Tile-size sweep of the tiled var encode (after the parity suite passed).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for vt in 64 128 256; do
  PACKOS_VAR_TILE=$vt timeout -k 10 300 python tools/vbench.py ${VB_ARGS:-C3 C5} > gpurun_out/vsweep_$vt.log 2>&1 || exit $?
  echo "VT=$vt"; grep -v amdgpu.ids gpurun_out/vsweep_$vt.log
done
