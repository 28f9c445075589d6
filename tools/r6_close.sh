#!/usr/bin/env bash
# closing check of the in-tree build: the GPU suite, smoke(), the default bench line
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tools/gpu_step.sh tests 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
tools/gpu_step.sh smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
tools/gpu_step.sh bench 300 python -u bench.py --steps 20 --warmup 3 || exit $?
echo all-done
