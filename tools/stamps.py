"""Diagnostic: per-phase cycle attribution of the single-deployment rollout
kernel (s_memtime stamps, separate kernel instantiation; results of the
stamped run are the real results, timings are inflated by the stamps)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd"))
from ccka import configs  # noqa: E402
from ccka.engine import Engine  # noqa: E402

eng = Engine(0)
eng.lib.ccka_debug_ablate.argtypes = [C.c_void_p, C.c_int32]
eng.set_world(configs.config2_world())
eng.set_scenarios(configs.hpa_scenarios(100_000))
eng.gen_load(configs.trace_gen())
names = ["top(load,hour)", "readiness+profile", "hpa ring push (C3)", "reconcile+schedule",
         "provision", "disruption", "accounting", "tail", "hpa proposal (C1)", "hpa behavior (C2)"]
for mask in (16, 16 | 1):
    eng.lib.ccka_debug_ablate(eng.ctx, mask)
    eng.rollout(trajectory=True)
    buf = (C.c_ulonglong * 12)()
    assert eng.lib.ccka_debug_stamps(eng.ctx, buf) == 0
    tot = sum(buf)
    lpw = min(64, max(32, -(-100_000 // (2 * 4 * 256))))  # the engine's automatic lanes per wave
    waves = -(-100_000 // lpw)
    print(f"mask {mask}: kernel {eng.kernel_ms():.3f} ms; cycles per wave-step by phase:")
    tot = sum(list(buf)[:10])
    for n, v in zip(names, list(buf)[:10]):
        print(f"  {n:22s} {v / waves / 1440:9.1f}  {100.0 * v / tot:5.1f} %")
    print(f"  shader clock ~ {sum(list(buf)[:10]) / waves / (eng.kernel_ms() * 1e-3) / 1e9:.2f} GHz "
          f"(stamped cycles per wave / kernel time)")
    print(f"  wave-steps evaluating disruption {buf[10] / waves / 1440:.3f}, running HPA behavior {buf[11] / waves / 1440:.3f}")
