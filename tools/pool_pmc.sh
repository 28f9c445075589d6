#!/usr/bin/env bash
# SQ issue counters of the per-wave and pooled single-deployment kernels
# (tools/pool_pmc.py), two PMC passes, summarised per kernel.
# usage: tools/pool_pmc.sh <outdir>
out="$1"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$out"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU \
  SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY -d "$out/p1" -o run --output-format csv -- python3 tools/pool_pmc.py \
  > "$out/p1.log" 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE \
  -d "$out/p2" -o run --output-format csv -- python3 tools/pool_pmc.py > "$out/p2.log" 2>&1 || exit $?
python3 - "$out" <<'PY'
import csv, glob, sys, collections
# the last dispatch of each kernel (the measured rollout)
last = {}
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    rows = list(csv.DictReader(open(f)))
    for name, pat in (("pooled", "rollout_pool"), ("per-wave", "rollout_d1")):
        ids = sorted({int(r["Dispatch_Id"]) for r in rows if pat in r["Kernel_Name"]})
        if not ids:
            continue
        for r in rows:
            if int(r["Dispatch_Id"]) == ids[-1]:
                last.setdefault(name, {})[r["Counter_Name"]] = last.get(name, {}).get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for name, k in last.items():
    w = k.get("SQ_WAVES", 1)
    print(f"== {name}: waves {w:.0f}")
    for c in sorted(k):
        print(f"  {c:24s} {k[c]:16.0f}")
    if "SQ_THREAD_CYCLES_VALU" in k:
        print(f"  active lanes per VALU instruction {k['SQ_THREAD_CYCLES_VALU'] / k['SQ_INSTS_VALU']:.2f}")
        print(f"  VALU per wave {k['SQ_INSTS_VALU'] / w:.0f}, lane-VALU (x lanes) per scenario {k['SQ_THREAD_CYCLES_VALU'] / 1e5:.0f}")
PY
