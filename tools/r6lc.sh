#!/usr/bin/env bash
# lane-local vs cooperative provisioning on the skewed schedule: parity tests, then the A/B
cd "$GRAFT_REPO_ROOT" || exit 1
tools/gpu_step.sh sk_tests 600 python -u -m pytest tests/test_gpu_skew.py tests/test_gpu_multi_deploy.py -x -q --timeout 300 --timeout-method thread || exit $?
tools/gpu_step.sh lc_local 200 python -u tools/sk_stats.py --lib main 100000 1440 || exit $?
tools/gpu_step.sh lc_coop 200 python -u tools/sk_stats.py --lib main --mode 3 100000 1440 || exit $?
tools/gpu_step.sh dep2 300 python -u bench.py --deployments 2 --steps 10 --warmup 2 --no-cpu || exit $?
tools/gpu_step.sh dep4 300 python -u bench.py --deployments 4 --steps 5 --warmup 1 --no-cpu || exit $?
