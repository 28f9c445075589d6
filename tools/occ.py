"""Timing of the single-deployment kernel vs its occupancy target, for the
config-2 (one round of waves) and config-3 / config-4 (multi-round) batches."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd"))
from ccka import configs  # noqa: E402
from ccka.engine import Engine  # noqa: E402

eng = Engine(0)
eng.lib.ccka_debug_occ.argtypes = [C.c_void_p, C.c_int32]
eng.lib.ccka_debug_lpw.argtypes = [C.c_void_p, C.c_int32]
# config 2 is one resident round at 2 waves/SIMD: refill the round for the
# occupancy being tested (lanes per wave = N / (occ * 4 SIMDs * CUs))
LPW2 = {2: 0, 3: 33}
cases = {
    "config2": (configs.config2_world(), configs.hpa_scenarios(100_000), configs.trace_gen(), True),
    "config3": (configs.config3_world(), configs.config3_scenarios(1_000_000), configs.trace_gen(), False),
    "config4/4": (configs.config2_world(), configs.config4_scenarios(0, 1024), configs.config4_trace_gen(), False),
}
for name, (spec, sc, gen, traj) in cases.items():
    eng.set_world(spec)
    eng.set_scenarios(sc)
    eng.gen_load(gen)
    ref = None
    res = {}
    for r in range(2):
        for occ in (2, 3):
            eng.lib.ccka_debug_occ(eng.ctx, occ)
            eng.lib.ccka_debug_lpw(eng.ctx, LPW2[occ] if name == "config2" else 0)
            eng.rollout(trajectory=traj)
            res.setdefault(occ, []).append(eng.kernel_ms())
            out = eng.results()
            if ref is None:
                ref = out
            assert all((out[k] == ref[k]).all() for k in ref), (name, occ)
    print(name, {o: f"{min(v):.2f} ms" for o, v in res.items()}, flush=True)
