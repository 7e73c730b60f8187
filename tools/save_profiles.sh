#!/bin/bash
# Copy a gpu_session.sh run (test smoke bench prof pmc ...) into profiles/<round>/:
# bench line, rocprofv3 kernel stats, PMC CSVs + summary, test and smoke logs.
# usage: tools/save_profiles.sh <gpurun_out tag> <round dir, e.g. profiles/r2>
set -eu
src=gpurun_out/$1 dst=$2
mkdir -p "$dst"
grep '^{' "$src/bench.log" > "$dst/bench_n1.json"
cp "$src/prof/run_kernel_stats.csv" "$dst/bench_n40_kernel_stats.csv"
for d in pmc_fetch pmc_write pmc_sq pmc_lds; do cp "$src/$d/run_counter_collection.csv" "$dst/${d/pmc_/pmc_seg_}_n40.csv"; done
python3 tools/pmc_summary.py "$src" "$dst/pmc_seg_n40.json" 40 > /dev/null
cp "$src/pytest_gpu.log" "$dst/pytest_gpu.log"
cp "$src/smoke.log" "$dst/smoke.log"
