"""Per-wave-step dynamic instruction counts of the rollout kernel from
tools/prof_insts.sh (SQ_INSTS_* summed over waves / SQ_WAVES / steps), and the
mean active lanes per VALU instruction (SQ_THREAD_CYCLES_VALU /
SQ_ACTIVE_INST_VALU, both in quad-cycle units)."""
import collections
import csv
import glob
import json
import sys

d = sys.argv[1]
T = int(sys.argv[2]) if len(sys.argv) > 2 else 1440
agg = collections.defaultdict(float)
for f in glob.glob(f"{d}/pmc/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "rollout_d1_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
w = agg["SQ_WAVES"]
out = {k: round(v / w / T, 2) for k, v in agg.items() if k.startswith("SQ_INSTS")}
out["waves"] = w
out["active_lanes_per_valu_inst"] = round(agg["SQ_THREAD_CYCLES_VALU"] / agg["SQ_ACTIVE_INST_VALU"], 2)
out["wave_cycles_per_step"] = round(agg["SQ_WAVE_CYCLES"] * 4 / w / T, 1)
print(json.dumps(out, indent=1))
