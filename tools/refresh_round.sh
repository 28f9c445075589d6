#!/usr/bin/env bash
# Every measurement committed under profiles/<round>/, in one GPU call:
# bench lines of configs 2-5 (with the CPU baselines), the config-2 kernel
# trace + HBM + SQ counters and the config-5 trace + MFMA counters
# (prof_round1.sh), issue-side counters of configs 2-4 (prof_issue.sh) and
# the MLP SQ counters (prof_mlp.sh). Output: gpurun_out/refresh/.
# usage: tools/refresh_round.sh
out=gpurun_out/refresh
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $out
for c in 2 3 4 5; do
  tools/gpu_step.sh bench_full_c$c 400 python bench.py --config $c || exit $?
  grep '^{' gpurun_out/bench_full_c$c.log | tail -1 > $out/bench_config$c.json || exit 1
done
tools/gpu_step.sh bench_full_c5p 400 python bench.py --config 5 --mode policy || exit $?
grep '^{' gpurun_out/bench_full_c5p.log | tail -1 > $out/bench_config5_policy.json || exit 1
tools/prof_round1.sh $out/p1 || exit $?
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d "$out/c5p/trace" -o run --output-format csv -- \
  python3 bench.py --config 5 --mode policy --steps 2 --warmup 1 --no-cpu > "$out/c5p_trace.log" 2>&1 || exit $?
tools/prof_issue.sh $out/issue || exit $?
tools/prof_mlp.sh $out/mlp || exit $?
echo refresh-done
