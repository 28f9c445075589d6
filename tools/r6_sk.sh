#!/usr/bin/env bash
# Round 6: the general kernel's lane-skewed schedule (rollout_sk.hip): parity,
# then the --deployments lines (skewed, and lockstep for the A/B).
# usage: tools/r6_sk.sh
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tools/gpu_step.sh sk_tests 600 python -u -m pytest tests/test_gpu_skew.py tests/test_gpu_multi_deploy.py -x -v --timeout 300 --timeout-method thread || exit $?
tools/gpu_step.sh dep2 300 python -u bench.py --deployments 2 --steps 10 --warmup 2 || exit $?
tools/gpu_step.sh dep4 300 python -u bench.py --deployments 4 --steps 5 --warmup 1 --no-cpu || exit $?
tools/gpu_step.sh dep12 400 python -u bench.py --deployments 12 --steps 3 --warmup 1 --no-cpu || exit $?
tools/gpu_step.sh dep2_lock 300 python -u bench.py --deployments 2 --lockstep --steps 3 --warmup 1 --no-cpu || exit $?
tools/gpu_step.sh dep4_lock 300 python -u bench.py --deployments 4 --lockstep --steps 3 --warmup 1 --no-cpu || exit $?
echo all-done
