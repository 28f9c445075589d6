#!/usr/bin/env bash
# GPU parity tests of the rollout engines, then one bench line per config
# (kernel ms and value). usage: tools/quick_bench.sh [configs...]
cd "$GRAFT_REPO_ROOT" || exit 1
tools/gpu_step.sh par 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_sweep.py || exit $?
for c in ${@:-2 3 4}; do
  tools/gpu_step.sh bench_c$c 300 python bench.py --config $c --steps 3 --no-cpu || exit $?
  tail -1 gpurun_out/bench_c$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('config', $c, d['value'], d['roofline']['kernel_ms_avg'])"
done
