set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/alignshuf > gpurun_out/alignshuf.txt 2>&1 || { cat gpurun_out/alignshuf.txt; exit 5; }
cat gpurun_out/alignshuf.txt
CFG=C2 OP=decode VAR=PACKOS_DEC_TILE_BYTES VALS="default 8192 4096 12288" bash tools/gpu_env_ab.sh
