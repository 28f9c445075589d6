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
# tools/refresh_extra.sh: read-traffic split, config-5 kernel traces, loop split
if [ -d $src/tcc ]; then
  for d in $src/tcc/*/; do n=$(basename "$d"); cp "$d/run_counter_collection.csv" "$dst/config2_tcc_$n.csv"; done
fi
[ -f $src/c5p7/run_kernel_stats.csv ] && cp $src/c5p7/run_kernel_stats.csv "$dst/config5_policy_1e7_kernel_stats.csv"
[ -f $src/c5g/run_kernel_stats.csv ] && cp $src/c5g/run_kernel_stats.csv "$dst/config5_grad_kernel_stats.csv"
[ -f $src/loop_split_1e7.txt ] && cp $src/loop_split_1e7.txt "$dst/"
# the tree the profiles were taken from (bench.py labels the fields it copies from them)
head=$(git rev-parse --short=12 HEAD)$(git diff --quiet -- cost-and-carbon-aware-kubernetes-autoscaler_amd/csrc || echo "+dirty")
for f in "$dst/config2_traj_summary.json" "$dst/issue_config234.json"; do
  [ -f "$f" ] && python3 -c "import json,sys; p=sys.argv[1]; d=json.load(open(p)); d['source_head']=sys.argv[2]; json.dump(d,open(p,'w'),indent=1)" "$f" "$head"
done
ls "$dst"
