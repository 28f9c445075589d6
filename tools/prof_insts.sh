#!/usr/bin/env bash
# Dynamic instruction counts of the single-deployment rollout kernel (config 2,
# trajectory mode): one PMC pass (never combined with tracing), summarised per
# wave-step by tools/insts_summary.py. usage: tools/prof_insts.sh <outdir>
out="$1"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$out"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES \
  SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU -d "$out/pmc" -o run --output-format csv -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu > "$out/pmc.log" 2>&1 || exit $?
python3 tools/insts_summary.py "$out" | tee "$out/insts.json"
