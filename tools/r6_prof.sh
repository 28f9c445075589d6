#!/usr/bin/env bash
# Round-6 rocprofv3 kernel traces (--kernel-trace --stats) of the headline
# line, the two-deployment skewed line and the policy gradient, plus the
# gradient's parity tests. usage: tools/r6_prof.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof
tools/gpu_step.sh pgtest 300 python -u -m pytest tests/test_gpu_pg.py -x -q --timeout 300 --timeout-method thread || exit $?
tools/gpu_step.sh p_c2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/c2 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu || exit $?
tools/gpu_step.sh p_dep2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/dep2 -o run --output-format csv -- python3 bench.py --deployments 2 --steps 10 --warmup 2 --no-cpu || exit $?
tools/gpu_step.sh p_grad 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/grad -o run --output-format csv -- python3 bench.py --config 5 --mode grad --steps 5 --warmup 1 --no-cpu || exit $?
tools/gpu_step.sh grad 300 python -u bench.py --config 5 --mode grad --steps 5 --warmup 1 --no-cpu || exit $?
echo all-done
