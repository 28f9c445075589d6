#!/usr/bin/env bash
# Issue/wait counters of the single-deployment rollout (config 2), one PMC
# pass per set (never combined with tracing). usage: tools/prof_d1.sh <outdir> [bench args...]
out="$1"; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$out"
i=0
for set in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
  "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d "$out/p$i" -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu "$@" > "$out/p$i.log" 2>&1 || exit $?
done
python3 - "$out" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
c = collections.defaultdict(list)
for f in glob.glob(f"{d}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "rollout_d1" in r["Kernel_Name"]:
            c[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(c.items()):
    print(f"{k:24s} {sum(v)/len(v):.4g}")
PY
