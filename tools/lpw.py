"""Timing of the single-deployment kernel vs scenarios per wave (config 2)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd"))
from ccka import configs  # noqa: E402
from ccka.engine import Engine  # noqa: E402

eng = Engine(0)
eng.lib.ccka_debug_lpw.argtypes = [C.c_void_p, C.c_int32]
eng.set_world(configs.config2_world())
eng.set_scenarios(configs.hpa_scenarios(100_000))
eng.gen_load(configs.trace_gen())
vals = [int(x) for x in (sys.argv[1:] or ["64", "56", "48", "40", "32"])]
res = {v: [] for v in vals}
ref = None
for r in range(3):
    for v in vals:
        eng.lib.ccka_debug_lpw(eng.ctx, v)
        eng.rollout(trajectory=True)
        res[v].append(eng.kernel_ms())
        out = eng.results()
        if ref is None:
            ref = out
        assert all((out[k] == ref[k]).all() for k in ref), f"lpw {v} changed results"
for v in vals:
    print(f"lpw {v:2d}: median {sorted(res[v])[1]:7.3f} ms")
