#!/usr/bin/env bash
# The profile passes of tools/refresh_round.sh after its bench lines (resume
# when a later pass failed): config-5 trace + MFMA / FETCH counters, the issue
# counters of configs 2-4, the MLP SQ counters, the closed-loop trace.
# usage: tools/refresh_rest.sh
out=gpurun_out/refresh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p $out/p1
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d "$out/p1/c5/trace" -o run --output-format csv -- \
  python3 bench.py --config 5 --steps 5 --warmup 1 --no-cpu > "$out/p1/c5_trace.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE \
  -d "$out/p1/c5/pmc1" -o run --output-format csv -- python3 bench.py --config 5 --steps 1 --warmup 0 --no-cpu \
  > "$out/p1/c5_pmc1.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$out/p1/c5/pmc2" -o run --output-format csv -- \
  python3 bench.py --config 5 --steps 1 --warmup 0 --no-cpu > "$out/p1/c5_pmc2.log" 2>&1 || exit $?
tools/prof_issue.sh $out/issue || exit $?
tools/prof_mlp.sh $out/mlp || exit $?
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d "$out/c5p/trace" -o run --output-format csv -- \
  python3 bench.py --config 5 --mode policy --steps 2 --warmup 1 --no-cpu > "$out/c5p_trace.log" 2>&1 || exit $?
echo refresh-rest-done
