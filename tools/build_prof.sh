# Debug build with per-phase clocks of k_encode_tiles (-DPACKOS_PHASE_PROF):
# packos_amd/libpackos_prof.so, used by tools/vprof.sh (PACKOS_LIB override).
set -eu
cd "$(dirname "$0")/../packos_amd/csrc"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -shared -fPIC -Wall -DPACKOS_PHASE_PROF \
  -o ../libpackos_prof.so compile.cpp kernels.hip host_pipeline.cpp
