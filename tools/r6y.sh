#!/usr/bin/env bash
cd "$GRAFT_REPO_ROOT" || exit 1
tools/gpu_step.sh sk_tests 600 python -u -m pytest tests/test_gpu_skew.py tests/test_gpu_multi_deploy.py tests/test_gpu_mlp.py tests/test_policy_rollout.py -x -q --timeout 300 --timeout-method thread || exit $?
tools/gpu_step.sh dep12 400 python -u bench.py --deployments 12 --steps 3 --warmup 1 --no-cpu || exit $?
tools/gpu_step.sh poolpmc 400 tools/pool_pmc.sh gpurun_out/poolpmc || exit $?
