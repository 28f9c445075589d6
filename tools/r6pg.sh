#!/usr/bin/env bash
cd "$GRAFT_REPO_ROOT" || exit 1
tools/gpu_step.sh pgtest 300 python -u -m pytest tests/test_gpu_pg.py -x -q --timeout 300 --timeout-method thread || exit $?
tools/gpu_step.sh pgab 400 python -u tools/variant_grad.py 250000 pgold pgpf2 pgpf8 || exit $?
