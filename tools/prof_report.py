"""Summarise tools/prof_round.sh output: per-kernel durations and per-launch
HBM traffic of the rollout kernel (bytes from the L2 memory-side request
counters). Writes <outdir>/summary.json."""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "rollout_kernel"
out = {}
stats = list(csv.DictReader(open(f"{d}/trace/run_kernel_stats.csv")))
out["kernels"] = [{k: r[k] for k in ("Name", "Calls", "AverageNs", "MinNs", "MaxNs", "Percentage")}
                  for r in stats]
per = collections.defaultdict(list)
durs = {}
for f in sorted(glob.glob(f"{d}/pmc*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            per[r["Counter_Name"]].append(float(r["Counter_Value"]))
            durs[r["Counter_Name"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
c = {k: sum(v) / len(v) for k, v in per.items()}
rd = c.get("TCC_EA0_RDREQ_32B", 0) * 32 + c.get("TCC_EA0_RDREQ_64B", 0) * 64 + c.get("TCC_EA0_RDREQ_128B", 0) * 128
wr64 = c.get("TCC_EA0_WRREQ_64B", 0)
wr = wr64 * 64 + (c.get("TCC_EA0_WRREQ", 0) - wr64) * 32
out["counters_per_launch"] = c
out["read_bytes_by_request_size"] = rd
out["write_bytes_by_request_size"] = wr
out["fetch_size_bytes"] = c.get("FETCH_SIZE", 0) * 1024
out["write_size_bytes"] = c.get("WRITE_SIZE", 0) * 1024
out["traffic_bytes"] = rd + wr
if "GRBM_GUI_ACTIVE" in c and "GRBM_GUI_ACTIVE" in durs:
    out["effective_clock_ghz"] = c["GRBM_GUI_ACTIVE"] / 8 / durs["GRBM_GUI_ACTIVE"] / 1e9
json.dump(out, open(f"{d}/summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
