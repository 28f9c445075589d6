"""Schedule counters of the general kernel's lane-skewed schedule (SK_STATS
variant: VARIANTS_NO_MAKE=1 python tools/build_variants.py "skstats=s@-DSK_STATS
-DCCKA_SK_ONE"), or with --stamps its phase cycles (GK_STAMPS variant "skgks=s@-DGK_STAMPS
-DCCKA_SK_ONE"), run with the diagnostic ablate bit 16 (the counter buffer;
results are the real ones). World: bench.py --deployments 2 (config 2, two HPA
deployments, 8 node slots). usage: python tools/sk_stats.py [--stamps] [N] [T]"""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd"))
from ccka import abi, configs  # noqa: E402
from ccka.engine import Engine  # noqa: E402

TRAJ = "--summary" not in sys.argv
if not TRAJ:
    sys.argv.remove("--summary")
STAMPS = "--stamps" in sys.argv
if STAMPS:
    sys.argv.remove("--stamps")
MODE = None  # --mode M: ccka_debug_engine(M) (3: the cooperative provisioning scans)
if "--mode" in sys.argv:
    k = sys.argv.index("--mode")
    MODE = int(sys.argv[k + 1])
    del sys.argv[k:k + 2]
VAR = None  # --lib NAME: another variant under csrc/build/variants (timing only); "main": the main build
if "--lib" in sys.argv:
    k = sys.argv.index("--lib")
    VAR = sys.argv[k + 1]
    del sys.argv[k:k + 2]
SLIB = None  # --slib NAME: the counter / stamp variant to read (default skstats / skgks)
if "--slib" in sys.argv:
    k = sys.argv.index("--slib")
    SLIB = sys.argv[k + 1]
    del sys.argv[k:k + 2]
N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
T = int(sys.argv[2]) if len(sys.argv) > 2 else 1440
lib = os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd", "csrc", "build", "variants", VAR or SLIB or ("skgks" if STAMPS else "skstats"),
                   "libccka.so")
if VAR == "main":
    lib = os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd", "csrc", "build", "libccka.so")
e = Engine(0, lib_path=lib)
e.lib.ccka_debug_ablate.argtypes = [C.c_void_p, C.c_int32]
e.lib.ccka_debug_stamps.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
spec = configs.config2_world(n_steps=T)
spec.deploys = [configs.deployment(abi.SCALER_HPA, replicas0=3, max_r=30, req_cpu=(200, 300)[d],
                                   target=(70, 60)[d]) for d in range(2)]
sc = configs.hpa_scenarios(N)
if MODE is not None:
    e.set_engine(MODE)
e.set_world(spec)
e.set_scenarios(sc)
e.gen_load(configs.trace_gen())
e.lib.ccka_debug_ablate(e.ctx, 16)
t0 = time.time()
e.rollout(trajectory=TRAJ)
print("engine", e.last_engine(), "kernel ms", e.kernel_ms(), "wall", time.time() - t0)
if VAR:
    ms = []
    for _ in range(3):
        e.rollout(trajectory=TRAJ)
        ms.append(e.kernel_ms())
    print(VAR, "kernel ms", sorted(ms))
    if not STAMPS:
        sys.exit(0)
    e.rollout(trajectory=TRAJ)
st = (C.c_ulonglong * 12)()
e._chk(e.lib.ccka_debug_stamps(e.ctx, st), "ccka_debug_stamps")
if STAMPS:
    ph = ["samples+hour", "readiness+profile", "scalers", "reconcile+sched", "provisioning", "disruption",
          "accounting+record", "SK: loop top + sample issue", "SK: quiet steps", "SK: caches", "SK: flush"]
    tot = sum(st[k] for k in range(11))
    for k, nm in enumerate(ph):
        print(f"{nm:30s} {st[k] / max(st[11], 1):14.0f} cycles/wave {100 * st[k] / max(tot, 1):6.1f} %")
    print("waves", st[11])
    sys.exit(0)
names = ["stall: disruption pending (g_dirty)", "stall: pods not placed", "stall: consolidation wake",
         "stall: node ready", "stall: hour / peak boundary", "stall: HPA outside thresholds",
         "live lane-passes", "lane full steps", "lane quiet steps", "wave full-step runs", "wave passes",
         "lanes served by provisioning"]
waves = (N + 63) // 64
for k, nm in enumerate(names):
    print(f"{nm:40s} {st[k]:14d}  per scenario {st[k] / N:10.2f}  per wave {st[k] / waves:10.2f}")
print("lanes per full-step run", st[7] / max(st[9], 1))
