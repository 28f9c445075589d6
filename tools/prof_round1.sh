#!/usr/bin/env bash
# Round-1 profile set (each rocprofv3 pass its own run, never PMC + tracing):
#  config 2 (trajectory): kernel trace + HBM request counters + SQ counters
#  config 5 (MLP):        kernel trace + MFMA busy counters
# usage: tools/prof_round1.sh <outdir>
out="$1"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$out"
tools/prof_round.sh "$out/c2" || exit $?
python3 tools/prof_report.py "$out/c2" rollout_d1_kernel > "$out/c2_report.log" 2>&1 || exit $?
tools/prof_pmc.sh "$out/c2sq" || exit $?
python3 tools/pmc_summary.py "$out/c2sq" 1440 rollout_d1_kernel > "$out/c2_sq_counters.txt" || exit $?
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d "$out/c5/trace" -o run --output-format csv -- \
  python3 bench.py --config 5 --steps 5 --warmup 1 --no-cpu > "$out/c5_trace.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE \
  -d "$out/c5/pmc1" -o run --output-format csv -- python3 bench.py --config 5 --steps 1 --warmup 0 --no-cpu \
  > "$out/c5_pmc1.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$out/c5/pmc2" -o run --output-format csv -- \
  python3 bench.py --config 5 --steps 1 --warmup 0 --no-cpu > "$out/c5_pmc2.log" 2>&1 || exit $?
echo done
