#!/usr/bin/env bash
# SQ PMC passes over the general kernel on multi-deployment worlds
# (tools/multi_bench.py): instruction mix and memory instructions per wave-step.
# usage: tools/pmc_multi.sh <outdir> <world names...>
out="$1"; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$out"
for wname in "$@"; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES \
    SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_INSTS_BRANCH -d "$out/$wname/p1" -o run --output-format csv \
    -- python3 tools/multi_bench.py 100000 "$wname" > "$out/$wname.log" 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY -d "$out/$wname/p2" -o run --output-format csv \
    -- python3 tools/multi_bench.py 100000 "$wname" >> "$out/$wname.log" 2>&1 || exit $?
  echo "== $wname $(grep kernel "$out/$wname.log" | tail -1)"
  python3 tools/pmc_summary.py "$out/$wname" 1440 rollout_kernel
done
