#!/usr/bin/env bash
# Clock / issue counters of the config-2 rollout for the main build and variants.
# usage: tools/prof_clock.sh <outdir> [variant ...]
out="$1"; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$out"
for v in main "$@"; do
  arg=""; [ "$v" != main ] && arg="--variant=$v"
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU \
    -d "$out/$v" -o run --output-format csv -- python3 tools/one_rollout.py $arg > "$out/$v.log" 2>&1 || exit $?
  python3 - "$out/$v" <<'PY'
import csv, sys, collections
d = sys.argv[1]
rows = [r for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")) if "rollout_d1" in r["Kernel_Name"]]
c = collections.defaultdict(list); dur = {}
for r in rows:
    c[r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
m = {k: sum(v) / len(v) for k, v in c.items()}
t = sum(dur.values()) / len(dur)
print(d, f"kernel {t*1e3:.3f} ms  clock {m['GRBM_GUI_ACTIVE'] / 8 / t / 1e9:.2f} GHz(?)  VALU/wave {m['SQ_INSTS_VALU']/m['SQ_WAVES']:.0f}  SALU/wave {m['SQ_INSTS_SALU']/m['SQ_WAVES']:.0f}  lanes/VALU {m['SQ_THREAD_CYCLES_VALU']/m['SQ_ACTIVE_INST_VALU']:.1f}  busy {m['SQ_BUSY_CYCLES']:.4g}  gui {m['GRBM_GUI_ACTIVE']:.4g}")
PY
done
