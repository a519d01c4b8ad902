# Ablation builds of libpackos (experiments only, never committed as product):
# a copy of csrc with phase switches, one .so per variant under abl/.
#   tools/abl_build.sh "name ABLF ABLC" ...   (ABLF=0: skip the AFF frame phase,
#   ABLC=0: skip the chunk pass of k_encode_tiles)
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/ablsrc; rm -rf $W; mkdir -p $W/packos_amd/csrc $W/include $R/abl
cp $R/packos_amd/csrc/* $W/packos_amd/csrc/; cp $R/include/packos.h $W/include/
cd $W/packos_amd/csrc
# ABLF=0 skips both frame forms AND declares the tile hole-free (HT = 0): the
# frame is what writes the hole table (hgs / hln / hsrc), so a frame-less build
# that kept HT > 0 made the chunk and edge passes form global addresses from
# never-written hsrc entries -> hipErrorIllegalAddress on C5 (round 2).  With
# HT = 0 the ablation streams the (unwritten) image: load + layout + chunks.
grep -q '        if (k0 < k1) {' encode_var.inc && grep -q '        if (j < rows) {' encode_var.inc && grep -q '        HT = rows \* H;' encode_var.inc && grep -q '    HT = (uint32_t)(tt >> 40);' encode_var.inc || { echo "abl_build.sh: encode_var.inc changed, update the patterns"; exit 1; }
sed -i 's/^        if (k0 < k1) {/        if (ABLF \&\& k0 < k1) {/; s/^        if (j < rows) {$/        if (ABLF \&\& j < rows) {/; s/^        HT = rows \* H;/        HT = ABLF ? rows * H : 0u;/; s/^    HT = (uint32_t)(tt >> 40);/    HT = ABLF ? (uint32_t)(tt >> 40) : 0u;/; s/    for (uint32_t cb = (uint32_t)wave \* kWave; cb < NC; cb += kVUnroll \* kVNT) {/    for (uint32_t cb = (uint32_t)wave * kWave; ABLC \&\& cb < NC; cb += kVUnroll * kVNT) {/' encode_var.inc
for v in "$@"; do
  set -- $v
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -shared -fPIC -DABLF=$2 -DABLC=$3 ${ABL_FLAGS:-} \
    -o $R/abl/libpackos_$1.so compile.cpp kernels.hip host_pipeline.cpp &
done
wait
