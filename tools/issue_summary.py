"""Issue-side utilisation of the rollout kernel from tools/prof_issue.sh.

SQ *_CYCLES / ACTIVE_INST_* counters are summed over all waves in units of 4
shader cycles (one wave64 VALU instruction = 1 unit = 4 cycles of one wave's
issue); GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS
note), so GRBM_GUI_ACTIVE / 8 is the kernel length in shader cycles.
Fractions are of all SIMD (or CU) cycles of the kernel; waves of one SIMD
issue to different units in the same cycle, so the per-unit fractions can sum
past 1. wave_lifetime_frac = mean wave lifetime / kernel length (config 2 is
one resident round: 1 - this is the tail left by early-finishing waves)."""
import collections
import csv
import glob
import json
import sys

d = sys.argv[1]
SIMDS, CUS = 1024, 256
res = {}
for c in (2, 3, 4):
    agg = collections.defaultdict(float)
    for f in glob.glob(f"{d}/c{c}/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "rollout_d1_kernel" in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
    if not agg:
        continue
    bench = json.loads([ln for ln in open(f"{d}/c{c}.log").read().splitlines() if ln.startswith("{")][-1])
    res[c] = {"counters": dict(agg), "kernel_ms": bench["roofline"]["kernel_ms_avg"]}
unit = 4.0
out = {"sq_unit_cycles": unit}
for c, r in res.items():
    k = r["counters"]
    cyc = k["GRBM_GUI_ACTIVE"] / 8
    out[f"config{c}"] = {
        "kernel_ms_profiled": round(r["kernel_ms"], 3),
        "clock_ghz": round(cyc / (r["kernel_ms"] * 1e-3) / 1e9, 3),
        "simd_issue_frac": round(k["SQ_ACTIVE_INST_ANY"] * unit / (SIMDS * cyc), 4),
        "valu_issue_frac": round(k["SQ_ACTIVE_INST_VALU"] * unit / (SIMDS * cyc), 4),
        "salu_issue_frac": round(k["SQ_ACTIVE_INST_SCA"] * unit / (SIMDS * cyc), 4),
        "lds_issue_frac_per_cu": round(k["SQ_ACTIVE_INST_LDS"] * unit / (CUS * cyc), 5),
        "active_lanes_per_valu_inst": round(k["SQ_THREAD_CYCLES_VALU"] / k["SQ_INSTS_VALU"], 2),
        "wave_lifetime_frac": round(k["SQ_WAVE_CYCLES"] * unit / k["SQ_WAVES"] / cyc, 4),
        "waves": int(k["SQ_WAVES"]),
    }
print(json.dumps(out, indent=1))
