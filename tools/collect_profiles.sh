# Copy a tools/gpu_profile.sh run from gpurun_out/ into profiles/<round>/ and
# regenerate profiles/<round>/pmc_M.json from the copied PMC passes.
set -eu
R=${1:-r01}
mkdir -p profiles/$R
grep -v amdgpu.ids gpurun_out/bench_full.log > profiles/$R/M_bench.log
cp gpurun_out/prof_M/run_kernel_stats.csv profiles/$R/M_kernel_stats.csv
cp gpurun_out/pmc_fetch/run_counter_collection.csv profiles/$R/M_pmc_fetch_size.csv
cp gpurun_out/pmc_write/run_counter_collection.csv profiles/$R/M_pmc_write_size.csv
alg=$(python3 -c "import json;print(json.loads(open('profiles/$R/M_bench.log').read().strip().splitlines()[-1])['roofline']['algorithmic_bytes_per_launch'])")
k=$(python3 -c "import csv;print(max(csv.DictReader(open('profiles/$R/M_kernel_stats.csv')), key=lambda r: float(r['TotalDurationNs']))['Name'].split('<')[0].split('::')[-1].split('(')[0])")
python3 tools/pmc_summary.py profiles/$R/M_pmc_fetch_size.csv profiles/$R/M_pmc_write_size.csv "$k" "$alg" profiles/$R/pmc_M.json > /dev/null
cut -d, -f1-8 profiles/$R/M_kernel_stats.csv | head -3
