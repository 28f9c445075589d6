#!/usr/bin/env bash
cd "$GRAFT_REPO_ROOT" || exit 1
tools/gpu_step.sh sk_tests 600 python -u -m pytest tests/test_gpu_skew.py tests/test_gpu_multi_deploy.py -x -q --timeout 300 --timeout-method thread || exit $?
tools/gpu_step.sh skab 500 python -u tools/sk_ab.py || exit $?
