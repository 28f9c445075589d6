#!/usr/bin/env bash
# Issue-side counters of the rollout kernel for configs 2 (trajectory), 3 and 4
# (one PMC pass each, never combined with tracing), summarised by
# tools/issue_summary.py into <outdir>/issue.json.
# usage: tools/prof_issue.sh <outdir>
out="$1"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$out"
for c in 2 3 4; do
  timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA \
    SQ_ACTIVE_INST_LDS SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE \
    -d "$out/c$c" -o run --output-format csv -- python3 bench.py --config $c --steps 1 --warmup 0 --no-cpu \
    > "$out/c$c.log" 2>&1 || exit $?
done
python3 tools/issue_summary.py "$out" > "$out/issue.json" || exit $?
cat "$out/issue.json"
