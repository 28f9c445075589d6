#!/usr/bin/env bash
# One SQ PMC pass over three config-2 trajectory rollouts for the main build and
# each tools/build_variants.py variant: instruction mix per wave-step.
# usage: tools/pmc_variants.sh <outdir> [variant names...]
out="$1"; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$out"
for v in main "$@"; do
  arg=""; [ "$v" != main ] && arg="--variant=$v"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES \
    SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_INSTS_BRANCH -d "$out/$v/p1" -o run --output-format csv \
    -- python3 tools/one_rollout.py $arg > "$out/$v.log" 2>&1 || exit $?
  echo "== $v $(grep kernel "$out/$v.log" | tail -1)"
  python3 tools/pmc_summary.py "$out/$v" 1440 rollout_d1_kernel
done
