#!/bin/bash
# Experiment builds (never the product): abl/libpackos_<name>.so from a copy of
# packos_amd/csrc, optionally patched by a python script (stdin-free: PATCH=file.py
# run in the copy's csrc directory) and compiled with extra flags.
#   PATCH=/tmp/p.py tools/var_build.sh name "-DFOO=1"
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; flags=${2:-}
W=/tmp/varsrc_$name; rm -rf $W; mkdir -p $W/packos_amd/csrc $W/include $R/abl
cp $R/packos_amd/csrc/* $W/packos_amd/csrc/; cp $R/include/packos.h $W/include/
cd $W/packos_amd/csrc
[ -n "${PATCH:-}" ] && python3 "$PATCH"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -shared -fPIC $flags -o $R/abl/libpackos_$name.so \
  compile.cpp kernels.hip host_pipeline.cpp
echo "built abl/libpackos_$name.so"
