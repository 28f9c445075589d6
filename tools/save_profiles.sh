#!/usr/bin/env bash
# Copy the outputs of tools/refresh_d1.sh (gpurun_out/r2b after the GPU call
# merged them back) into profiles/<round>/ under the names bench.py and
# DESIGN.md read. usage: tools/save_profiles.sh <round dir, e.g. profiles/round3>
set -e
src=gpurun_out/r2b
dst="$1"
mkdir -p "$dst"
cp $src/c2/summary.json "$dst/config2_traj_summary.json"
cp $src/c2/trace/run_kernel_stats.csv "$dst/config2_traj_kernel_stats.csv"
for i in 1 2 3 4; do cp $src/c2/pmc$i/run_counter_collection.csv "$dst/config2_traj_pmc$i.csv"; done
cp $src/c2_sq_counters.txt "$dst/config2_sq_counters.txt"
cp $src/stamps.txt "$dst/config2_stamps.txt"
cp $src/issue/issue.json "$dst/issue_config234.json"
for f in $src/bench_*.json; do cp "$f" "$dst/"; done
ls "$dst"
