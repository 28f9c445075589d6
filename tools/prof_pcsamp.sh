#!/usr/bin/env bash
# PC sampling (host trap, time-based) of the config-2 rollout: where the waves
# of the rollout kernel sit, per instruction. usage: tools/prof_pcsamp.sh <outdir>
out="$1"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$out"
timeout -s KILL 180 rocprofv3 -L > "$out/avail.txt" 2>&1
timeout -s KILL 180 rocprofv3 --pc-sampling-beta-enabled 1 --pc-sampling-method host_trap --pc-sampling-unit time \
  --pc-sampling-interval 1 -d "$out/pcs" -o run --output-format csv -- \
  python3 bench.py --steps 2 --warmup 0 --no-cpu > "$out/pcs.log" 2>&1
echo "rc=$?"
ls -R "$out" | head -30
