#!/usr/bin/env bash
# Profile the bench command for profiles/: kernel-trace stats, then one PMC pass
# per counter group (never combined with tracing; each pass its own run).
# usage: tools/prof_round.sh <outdir> [bench args...]
out="$1"; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$out"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu "$@" > "$out/trace.log" 2>&1 || exit $?
i=0
for set in "TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B GRBM_GUI_ACTIVE" \
           "TCC_EA0_WRREQ TCC_EA0_WRREQ_64B GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d "$out/pmc$i" -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu "$@" > "$out/pmc$i.log" 2>&1 || exit $?
done
