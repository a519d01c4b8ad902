# CPU-side sanitizer pass (this container, no GPU): the oracle and libpackos's
# host code (schema compiler, json_lite parser, host pipelines' argument
# checks) built with AddressSanitizer + UBSan (clang's shared runtime; device
# code unchanged), then the whole `-m "not gpu"` suite under them, including
# the corrupted-blob decode oracle tests and the schema-error tests.
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
make -s -C "$R/oracle" asan
mkdir -p "$R/build/asan"
S="$R/packos_amd/csrc"
/opt/rocm/bin/hipcc -O1 -g --offload-arch=gfx950 -std=c++17 -shared -fPIC -fno-omit-frame-pointer \
  -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -shared-libsan \
  -o "$R/build/asan/libpackos.so" "$S/compile.cpp" "$S/kernels.hip" "$S/host_pipeline.cpp"
cd "$R"
LD_PRELOAD="$RT" ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
  PACKOS_LIB="$R/build/asan/libpackos.so" PACKOS_ORACLE_LIB="$R/oracle/_asan/liboracle.so" \
  python -m pytest tests -x -q -m "not gpu" -p no:cacheprovider "$@"
