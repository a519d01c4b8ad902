#!/bin/bash
# Evidence pass of the in-tree product on the box: the GPU suite, smoke(),
# the driver's default bench command, and rocprofv3 --kernel-trace --stats
# of that same command — each under its own time limit, stopping at the
# first step that fails.  Output under gpurun_out/$OUT/.
#   OUT=r06F1 bash tools/evidence.sh
set -u
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUT:-evidence}"; mkdir -p "$O"
cd "$R"
python3 -c "import bench; print(bench.product_tree_hash())" > "$O/product_tree.txt"
echo "$(date +%T) suite"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
echo "$(date +%T) smoke"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1
rc=$?; tail -1 "$O/smoke.log"; [ $rc -eq 0 ] || exit $rc
echo "$(date +%T) bench"
timeout -k 10 400 python3 bench.py > "$O/bench.log" 2>&1
rc=$?; grep '^{' "$O/bench.log" | tail -1; [ $rc -eq 0 ] || exit $rc
echo "$(date +%T) rocprof"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- python3 "$R/bench.py" > "$O/prof_bench.log" 2>&1
rc=$?; grep '^{' "$O/prof_bench.log" | tail -1; exit $rc
