#!/usr/bin/env bash
# PMC passes over one bench rollout (each pass its own run, <= 8 SQ counters).
# usage: tools/prof_pmc.sh <outdir> [bench args...]
out="$1"; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$out"
i=0
for set in \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH" \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_THREAD_CYCLES_VALU" \
  "SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VSKIPPED"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d "$out/p$i" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu "$@" > "$out/p$i.log" 2>&1 || exit $?
done
