#!/usr/bin/env bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof
tools/gpu_step.sh pgtest 300 python -u -m pytest tests/test_gpu_pg.py -x -q --timeout 300 --timeout-method thread || exit $?
tools/gpu_step.sh grad 300 python -u bench.py --config 5 --mode grad --steps 5 --warmup 1 --no-cpu || exit $?
tools/gpu_step.sh p_grad 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/grad2 -o run --output-format csv -- python3 bench.py --config 5 --mode grad --steps 5 --warmup 1 --no-cpu || exit $?
