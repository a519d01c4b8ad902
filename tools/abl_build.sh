# Ablation builds of libpackos (experiments only, never committed as product):
# a copy of csrc with phase switches, one .so per variant under abl/.
#   tools/abl_build.sh "name ABLF ABLC" ...   (ABLF=0: skip the AFF frame phase,
#   ABLC=0: skip the chunk pass of k_encode_tiles)
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/ablsrc; rm -rf $W; mkdir -p $W/packos_amd/csrc $W/include $R/abl
cp $R/packos_amd/csrc/* $W/packos_amd/csrc/; cp $R/include/packos.h $W/include/
cd $W/packos_amd/csrc
sed -i 's/        if (j < rows \&\& k0 < k1) {/        if (ABLF \&\& j < rows \&\& k0 < k1) {/; s/    for (uint32_t cb = (uint32_t)wave \* kWave; cb < NC; cb += kVUnroll \* kVNT) {/    for (uint32_t cb = (uint32_t)wave * kWave; ABLC \&\& cb < NC; cb += kVUnroll * kVNT) {/' encode_var.inc
for v in "$@"; do
  set -- $v
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -shared -fPIC -DABLF=$2 -DABLC=$3 ${ABL_FLAGS:-} \
    -o $R/abl/libpackos_$1.so compile.cpp kernels.hip host_pipeline.cpp &
done
wait
