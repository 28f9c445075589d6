#!/usr/bin/env bash
# Round-6 baseline on one MI355X: the GPU test suite, the default bench line,
# the MLP kernel trace + counters (tools/prof_mlp.sh).
# usage: tools/r6_base.sh
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tools/gpu_step.sh tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
tools/gpu_step.sh bench 300 python -u bench.py --steps 20 --warmup 3 || exit $?
tools/gpu_step.sh mlp 500 tools/prof_mlp.sh gpurun_out/mlp || exit $?
echo all-done
