#!/usr/bin/env bash
# the 12-deployment lockstep instantiation <12,16>: parity (12-deployment worlds), the bench line
cd "$GRAFT_REPO_ROOT" || exit 1
tools/gpu_step.sh d12_tests 600 python -u -m pytest tests/test_gpu_skew.py tests/test_gpu_multi_deploy.py -x -q --timeout 300 --timeout-method thread || exit $?
tools/gpu_step.sh dep12 400 python -u bench.py --deployments 12 --steps 3 --warmup 1 --no-cpu || exit $?
