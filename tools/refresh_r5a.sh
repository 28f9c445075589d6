#!/usr/bin/env bash
# Round-5 refresh, part 1 (one GPU call): the whole -m gpu suite, then
# tools/refresh_d1.sh (config-2 trace + HBM counters, configs 2-4 bench lines,
# drift lines, SQ / issue counters, stamps) and the KEDA line with its trace.
cd "$GRAFT_REPO_ROOT" || exit 1
tools/gpu_step.sh gput 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
tools/refresh_d1.sh || exit $?
out=gpurun_out/r2b
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d "$out/keda/trace" -o run --output-format csv -- \
  python3 bench.py --keda --steps 5 --warmup 1 --no-cpu > "$out/keda_trace.log" 2>&1 || exit $?
tools/gpu_step.sh bk 400 python bench.py --keda || exit $?
grep '^{' gpurun_out/bk.log | tail -1 > $out/bench_config2_keda.json || exit 1
echo r5a-done
