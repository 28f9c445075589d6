#!/usr/bin/env bash
# Round-5 iteration loop: parity of the single-deployment kernel, then an
# interleaved A/B of the kernel variants built by tools/build_variants.py.
# usage: tools/r5_quick.sh [variant names...]
cd "$GRAFT_REPO_ROOT" || exit 1
tools/gpu_step.sh par 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_sync15.py tests/test_multi_consolidation.py tests/test_gpu_traj_layout.py || exit $?
tools/gpu_step.sh vb 300 python -u tools/variant_bench.py "$@" || exit $?
cat gpurun_out/vb.log
