# Full GPU pass at HEAD: toolchain probe, parity suite + smoke + M bench with
# rocprof (tools/gpu_r02.sh), then the per-config table (tools/config_table.sh).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
{ command -v go && go version; command -v javac; nproc; } > gpurun_out/toolchains.txt 2>&1
bash tools/gpu_r02.sh || exit $?
CFGS="${CFGS:-C2 C3 C4 C5}" bash tools/config_table.sh
