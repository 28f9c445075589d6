#!/usr/bin/env bash
# Where the rollout kernel's waves spend their cycles (config 2, trajectory):
# parked in s_waitcnt (SQ_WAIT_ANY), stalled at issue (SQ_WAIT_INST_ANY) or
# issuing (SQ_ACTIVE_INST_ANY); one PMC pass. usage: tools/prof_waits.sh <outdir>
out="$1"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$out"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS -d "$out/pmc" -o run --output-format csv -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu > "$out/pmc.log" 2>&1 || exit $?
python3 - "$out" <<'PY'
import collections, csv, glob, json, sys
agg = collections.defaultdict(float)
for f in glob.glob(f"{sys.argv[1]}/pmc/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "rollout_d1_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
wc = agg["SQ_WAVE_CYCLES"]
print(json.dumps({k: round(v / wc, 4) for k, v in agg.items() if k != "SQ_WAVES"}, indent=1))
PY
