"""Summarise rocprofv3 PMC csv passes for the rollout kernel: per wave-step values."""
import collections, csv, glob, sys
d = sys.argv[1]
T = int(sys.argv[2]) if len(sys.argv) > 2 else 1440
KERNEL = sys.argv[3] if len(sys.argv) > 3 else "rollout_d1_kernel"
agg = collections.defaultdict(float)
for f in sorted(glob.glob(f"{d}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if KERNEL in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
w = agg.get("SQ_WAVES", 1564.0) or 1564.0
for k in sorted(agg):
    print(f"{k:28s} {agg[k]:16.0f} {agg[k] / w / T:10.1f} per wave-step")
