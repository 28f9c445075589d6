#!/usr/bin/env bash
# MLP policy kernel (config 5): kernel trace + two SQ counter passes
# (MFMA / LDS / VALU activity) of the standalone forward (mlp16_kernel, the
# bench default). usage: tools/prof_mlp.sh <outdir>
out="$1"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$out"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- \
  python3 bench.py --config 5 --steps 20 --warmup 3 --no-cpu > "$out/trace.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS \
  SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS \
  -d "$out/pmc1" -o run --output-format csv -- python3 bench.py --config 5 --steps 1 --warmup 0 --no-cpu \
  > "$out/pmc1.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU \
  SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_WAVES \
  -d "$out/pmc2" -o run --output-format csv -- python3 bench.py --config 5 --steps 1 --warmup 0 --no-cpu \
  > "$out/pmc2.log" 2>&1 || exit $?
python3 tools/pmc_summary.py "$out" 1 mlp16_kernel > "$out/mlp_counters.txt" 2>&1 || exit $?
echo done
