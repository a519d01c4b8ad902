# C5 encode time per blob at several shard sizes / set counts (footprint effects)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
run() { timeout -k 10 300 python bench.py --no-cpu --no-host --no-warm --steps 20 "$@" > gpurun_out/sz.log 2>&1 || { tail -3 gpurun_out/sz.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/sz.log').read().strip().splitlines()[-1]); print('$*', d['config']['blobs_per_gpu'], d['kernel_ms'], d['roofline']['frac'], d['config']['footprint_mib'])"; }
run --config C5 --blobs-per-gpu 262144
run --config C5 --blobs-per-gpu 1048576
run --config C5 --blobs-per-gpu 1048576 --sets 1
run --config C5 --blobs-per-gpu 4194304
run --config C3 --sets 1
run --config C3 --sets 3
run --config C3 --blobs-per-gpu 4194304
