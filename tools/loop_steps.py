"""Per-step durations of the closed loop's rollout_kernel launches from a
rocprofv3 kernel trace (analysis aid): launch k of a loop is step k - 1
(k = 0: the state initialisation). usage: python tools/loop_steps.py <trace dir>"""
import csv
import glob
import sys

rows = []
for f in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for name in ("rollout_kernel", "mlp_kernel", "policy"):
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows if name in r["Kernel_Name"]]
    print(name, len(d), "launches; ms:", " ".join(f"{x:.2f}" for x in d[:130]))
