#!/usr/bin/env bash
# Round 6 full GPU pass: the GPU test suite, the default bench line, the
# multi-deployment lines, config 5 (MLP forward + kernel trace / counters,
# fused closed loop at 1e7, policy gradient). usage: tools/r6_full.sh
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tools/gpu_step.sh tests 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
tools/gpu_step.sh bench 300 python -u bench.py --steps 20 --warmup 3 || exit $?
tools/gpu_step.sh dep2 300 python -u bench.py --deployments 2 --steps 10 --warmup 2 || exit $?
tools/gpu_step.sh dep4 300 python -u bench.py --deployments 4 --steps 5 --warmup 1 --no-cpu || exit $?
tools/gpu_step.sh dep12 400 python -u bench.py --deployments 12 --steps 3 --warmup 1 --no-cpu || exit $?
tools/gpu_step.sh c5 300 python -u bench.py --config 5 --steps 20 --warmup 3 || exit $?
tools/gpu_step.sh c5loop 400 python -u bench.py --config 5 --mode policy --n 10000000 --steps 3 --warmup 1 --no-cpu || exit $?
tools/gpu_step.sh c5grad 400 python -u bench.py --config 5 --mode grad --steps 5 --warmup 1 --no-cpu || exit $?
tools/gpu_step.sh mlp 500 tools/prof_mlp.sh gpurun_out/mlp || exit $?
echo all-done
