"""Summary of the config-5 MLP profile in profiles/<round>/: kernel-trace
average, achieved TFLOP/s, MFMA busy fraction of all SIMD cycles (one
profiled launch), effective clock (GRBM_GUI_ACTIVE / 8 / duration) and HBM
read bytes (FETCH_SIZE KiB x 2: the gfx950 correction, MI355X_MICROARCH.md).
usage: python3 tools/mlp_summary.py profiles/round1"""
import csv
import json
import sys

d = sys.argv[1]
FLOPS = 2 * (64 * 256 + 256 * 256 + 256 * 8) * 10_000_000
stats = [r for r in csv.DictReader(open(f"{d}/config5_mlp_kernel_stats.csv")) if "mlp_kernel" in r["Name"]][0]
c, dur = {}, {}
for name in ("config5_mlp_pmc_mfma.csv", "config5_mlp_pmc_fetch.csv"):
    for r in csv.DictReader(open(f"{d}/{name}")):
        if "mlp_kernel" in r["Kernel_Name"]:
            c[r["Counter_Name"]] = float(r["Counter_Value"])
            dur[r["Counter_Name"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
avg_ns = float(stats["AverageNs"])
cyc = c["GRBM_GUI_ACTIVE"] / 8
out = {
    "kernel": stats["Name"],
    "calls": int(stats["Calls"]),
    "avg_ns": avg_ns,
    "achieved_tflops": FLOPS / (avg_ns * 1e-9) / 1e12,
    "peak_tflops_dense_bf16": 2500.0,
    "mfma_busy_cycles": c.get("SQ_VALU_MFMA_BUSY_CYCLES"),
    "mfma_ops_bf16": c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16"),
    "effective_clock_ghz_profiled_launch": cyc / dur["GRBM_GUI_ACTIVE"] / 1e9,
    "mfma_busy_frac_of_simd_cycles": c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * cyc),
    "hbm_read_bytes_fetch_size_x2_gfx950": c.get("FETCH_SIZE", 0) * 1024 * 2,
    "x_bytes_algorithmic": 10_000_000 * 64 * 2,
    "y_bytes_algorithmic": 10_000_000 * 8 * 4,
}
json.dump(out, open(f"{d}/config5_mlp_summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
