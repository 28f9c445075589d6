"""Timing of kernel variants (tools/build_variants.py) on the config-2
trajectory rollout, interleaved rounds in one process; every variant's
results must equal the main build's bit for bit. Profiling aid only.
WORLD=defaults: the config-2 world with every upstream default of the path
(15 s HPA sync, drift, replacement and multi-node consolidation); WORLD=multi50:
drift, replacement and multi-node consolidation under 50 % budgets (G3).
usage: [WORLD=defaults] python tools/variant_bench.py [variant names...]"""
import glob
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd"))
from ccka import abi, configs  # noqa: E402
from ccka.engine import Engine  # noqa: E402

CSRC = os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd", "csrc", "build")
names = sys.argv[1:] or sorted(os.path.basename(os.path.dirname(p))
                               for p in glob.glob(os.path.join(CSRC, "variants", "*", "libccka.so")))
LPW = [int(x) for x in os.environ.get("LPW", "0").split(",")]  # scenarios per wave (0: automatic)
libs = [("main", abi.ENGINE_LIB)] + [(n, os.path.join(CSRC, "variants", n, "libccka.so")) for n in names]
libs = [(f"{n}@{lp}" if lp else n, path, lp) for n, path in libs for lp in LPW]
engs = {}
import ctypes as C  # noqa: E402
for n, path, lp in libs:
    e = Engine(0, lib_path=path)
    e.lib.ccka_debug_lpw.argtypes = [C.c_void_p, C.c_int32]
    e.lib.ccka_debug_lpw(e.ctx, lp)
    w = configs.config2_world()
    if os.environ.get("WORLD") == "defaults":
        w.hpa_sync_s, w.drift, w.replace, w.multi = 15, 1, 1, 1
    if os.environ.get("WORLD") == "multi50":  # multi-node consolidation acting (the G3 instantiation)
        w.drift, w.replace, w.multi = 1, 1, 1
        for pool in w.pools:
            pool.budget_pct = 50
    e.set_world(w)
    e.set_scenarios(configs.hpa_scenarios(100_000))
    e.gen_load(configs.trace_gen())
    engs[n] = e
times = {n: [] for n, _, _ in libs}
ref = None
for r in range(5):
    for n, _, _ in libs:
        engs[n].rollout(trajectory=True)
        times[n].append(engs[n].kernel_ms())
        if r == 0:
            res = engs[n].results()
            if ref is None:
                ref = res
            bad = [k for k in ref if not np.array_equal(res[k], ref[k])]
            assert not bad or os.environ.get("NOCHECK"), f"variant {n} differs from main in {bad}"
for n, _, _ in libs:
    v = sorted(times[n])
    print(f"{n:12s} median {v[2]:.3f} ms  min {v[0]:.3f} ms", flush=True)
