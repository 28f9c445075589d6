#!/usr/bin/env bash
# SQ counters of the general kernel's lane-skewed schedule (a variant lib, the
# tools/sk_stats.py world), one PMC pass per counter set (never combined with
# tracing). usage: tools/prof_sk.sh <outdir> <variant>
out="$1"; v="$2"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$out"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA \
  SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU -d "$out/p1" -o run --output-format csv -- \
  python3 tools/sk_stats.py --lib "$v" 100000 1440 > "$out/p1.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_LDS \
  SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_IFETCH -d "$out/p2" -o run --output-format csv -- \
  python3 tools/sk_stats.py --lib "$v" 100000 1440 > "$out/p2.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS -d "$out/p3" -o run --output-format csv -- \
  python3 tools/sk_stats.py --lib "$v" 100000 1440 > "$out/p3.log" 2>&1 || echo "p3 failed"
python3 - "$out" <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "rollout_kernel" not in r.get("Kernel_Name", ""):
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        n[r["Counter_Name"]] += 1
for k in sorted(tot):
    print(f"{k:28s} {tot[k] / max(n[k], 1):18.0f} per dispatch-row-avg  (rows {n[k]})")
PY
