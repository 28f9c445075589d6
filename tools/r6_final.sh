#!/usr/bin/env bash
# Round-6 closing GPU pass: the GPU test suite, smoke(), every bench line of
# DESIGN's measurement table, the MLP profile. usage: tools/r6_final.sh
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tools/gpu_step.sh tests 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
tools/gpu_step.sh smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
tools/gpu_step.sh bench 300 python -u bench.py --steps 20 --warmup 3 || exit $?
tools/gpu_step.sh keda 300 python -u bench.py --keda --steps 10 --warmup 2 --no-cpu || exit $?
tools/gpu_step.sh defaults 300 python -u bench.py --hpa-sync 15 --drift --replace --multi --steps 10 --warmup 2 --no-cpu || exit $?
tools/gpu_step.sh dep2 300 python -u bench.py --deployments 2 --steps 10 --warmup 2 || exit $?
tools/gpu_step.sh dep4 300 python -u bench.py --deployments 4 --steps 5 --warmup 1 --no-cpu || exit $?
tools/gpu_step.sh dep12 400 python -u bench.py --deployments 12 --steps 3 --warmup 1 --no-cpu || exit $?
tools/gpu_step.sh c3 400 python -u bench.py --config 3 --steps 5 --warmup 1 --no-cpu || exit $?
tools/gpu_step.sh c4 400 python -u bench.py --config 4 --steps 3 --warmup 1 --no-cpu || exit $?
tools/gpu_step.sh c5 300 python -u bench.py --config 5 --steps 20 --warmup 3 || exit $?
tools/gpu_step.sh c5loop 400 python -u bench.py --config 5 --mode policy --n 10000000 --steps 3 --warmup 1 --no-cpu || exit $?
tools/gpu_step.sh c5grad 400 python -u bench.py --config 5 --mode grad --steps 5 --warmup 1 --no-cpu || exit $?
echo all-done
