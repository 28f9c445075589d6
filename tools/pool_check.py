"""Pooled single-deployment kernel (rollout_pool.hip): parity with the oracle on
a ragged config-2 batch, then per-wave vs pooled on 1e5 x 1440 (results equal,
kernel times). Development aid."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pyoracle as po  # noqa: E402
from ccka import configs  # noqa: E402
from ccka.engine import Engine  # noqa: E402
from parity import compare  # noqa: E402

eng = Engine(0)
spec = configs.config2_world()
n = int(os.environ.get("NSMALL", "4099"))
sc = configs.hpa_scenarios(n)
load = po.gen_load(configs.trace_gen(), spec.n_steps, 1, sc.n)
eng.set_world(spec)
eng.set_scenarios(sc)
eng.set_load(load)
t0 = time.time()
eng.rollout(trajectory=True)
print("small rollout", time.time() - t0, "s, pooled", eng.debug_pool(), "kernel ms", eng.kernel_ms(), flush=True)
rg, tg = eng.results(), eng.trajectory()
rc, tc = po.rollout(spec, sc, load, traj=True, threads=16)
compare(rg, rc, tg, tc)
print("small parity OK", flush=True)
if os.environ.get("BIG", "1") == "1":
    sc = configs.hpa_scenarios(100_000)
    eng.set_scenarios(sc)
    eng.gen_load(configs.trace_gen())
    res = {}
    for mode in (0, 1, 0, 1):
        eng.debug_pool(mode)
        eng.rollout(trajectory=True)
        print("mode", mode, "pooled", eng.debug_pool(), "kernel ms", eng.kernel_ms(), flush=True)
        r = eng.results()
        if mode in res:
            continue
        res[mode] = (r, eng.trajectory())
    compare(res[1][0], res[0][0], res[1][1], res[0][1])
    print("1e5 pooled == per-wave", flush=True)
    import ctypes as C
    eng.lib.ccka_debug_ablate.argtypes = [C.c_void_p, C.c_int32]
    eng.lib.ccka_debug_stamps.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
    for q, age, idle in [(int(x.split(':')[0]), int(x.split(':')[1]), int(x.split(':')[2]))
                         for x in os.environ.get("POLICIES", "48:20000:1,64:20000:1,32:20000:1,64:100000:1").split(",")]:
        eng.debug_pool(1, q)
        eng.debug_pool_policy(age, idle)
        eng.lib.ccka_debug_ablate(eng.ctx, 16)
        eng.rollout(trajectory=True)
        eng.lib.ccka_debug_ablate(eng.ctx, 0)
        st = (C.c_ulonglong * 12)()
        eng.lib.ccka_debug_stamps(eng.ctx, st)
        v = list(st)
        waves = (sc.n + 391) // 392 * 8
        print(f"min {q} age {age} idle {idle}: {eng.kernel_ms():.3f} ms;  it max {v[0]} mean {v[1] / waves:.0f}; runs {v[2]} lanes/run {v[3] / max(v[2], 1):.1f} "
              f"events/scenario {v[3] / sc.n:.1f}; cycles/wave: serve {v[4] / waves:.0f} quiet {v[5] / waves:.0f} "
              f"idle {v[6] / waves:.0f} total {v[7] / waves:.0f} live/it {v[8] / max(v[1], 1):.1f} enq {v[9] / waves:.0f} srvchk {v[10] / waves:.0f} attach+pf {v[11] / waves:.0f}", flush=True)
