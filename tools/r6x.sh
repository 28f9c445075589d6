#!/usr/bin/env bash
cd "$GRAFT_REPO_ROOT" || exit 1
tools/gpu_step.sh dep12_lock 400 python -u bench.py --deployments 12 --lockstep --steps 2 --warmup 1 --no-cpu || exit $?
tools/gpu_step.sh dep8 400 python -u bench.py --deployments 8 --steps 2 --warmup 1 --no-cpu || exit $?
tools/gpu_step.sh dep8_lock 400 python -u bench.py --deployments 8 --lockstep --steps 2 --warmup 1 --no-cpu || exit $?
