#!/usr/bin/env bash
# Re-measure the single-deployment kernel set of profiles/round2 after a kernel change:
# config-2 bench line (CPU baseline + full-size parity) with its kernel trace and HBM
# request counters (prof_round.sh), configs 3/4 lines, --drift and --drift --replace
# lines, SQ and issue counters and the stamped phase split. Output: gpurun_out/r2b/.
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r2b; mkdir -p $out
tools/gpu_step.sh pr 400 tools/prof_round.sh $out/c2 || exit $?
python3 tools/prof_report.py $out/c2 rollout_d1_kernel > $out/c2_report.log || exit $?
tools/gpu_step.sh b2 400 python bench.py --config 2 || exit $?
grep '^{' gpurun_out/b2.log | tail -1 > $out/bench_config2.json || exit 1
for c in 3 4; do
  tools/gpu_step.sh b$c 400 python bench.py --config $c || exit $?
  grep '^{' gpurun_out/b$c.log | tail -1 > $out/bench_config$c.json || exit 1
done
tools/gpu_step.sh b2d 300 python bench.py --config 2 --drift --no-cpu || exit $?
grep '^{' gpurun_out/b2d.log | tail -1 > $out/bench_config2_drift.json || exit 1
tools/gpu_step.sh b2dr 300 python bench.py --config 2 --drift --replace --no-cpu || exit $?
grep '^{' gpurun_out/b2dr.log | tail -1 > $out/bench_config2_drift_replace.json || exit 1
tools/gpu_step.sh sq 300 tools/prof_pmc.sh $out/c2sq || exit $?
python3 tools/pmc_summary.py $out/c2sq 1440 rollout_d1_kernel > $out/c2_sq_counters.txt || exit $?
tools/gpu_step.sh iss 400 tools/prof_issue.sh $out/issue || exit $?
tools/gpu_step.sh st 200 python tools/stamps.py || exit $?
cp gpurun_out/st.log $out/stamps.txt
echo r2b-done
