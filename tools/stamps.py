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

lib = None
for a in sys.argv[1:]:
    if a.startswith("--variant="):  # a tools/build_variants.py build
        lib = os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd", "csrc", "build", "variants",
                           a.split("=", 1)[1], "libccka.so")
eng = Engine(0, lib_path=lib) if lib else Engine(0)
eng.lib.ccka_debug_ablate.argtypes = [C.c_void_p, C.c_int32]
eng.set_world(configs.config2_world())
eng.set_scenarios(configs.hpa_scenarios(100_000))
eng.gen_load(configs.trace_gen())
names = ["-", "quiet steps", "top (row wait, refill) + event flush+hour", "event: readiness+profile",
         "event: hpa+reconcile+sched", "event: provision", "event: disruption", "event: accounting+nxt",
         "sample prefetch + loop"]
eng.lib.ccka_debug_ablate(eng.ctx, 16)
trajectory = "--summary" not in sys.argv
eng.rollout(trajectory=trajectory)
buf = (C.c_ulonglong * 12)()
assert eng.lib.ccka_debug_stamps(eng.ctx, buf) == 0
b = list(buf)
lpw = min(64, max(32, -(-100_000 // (2 * 4 * 256))))  # the engine's automatic lanes per wave
waves = -(-100_000 // lpw)
tot = sum(b[1:9])
print(f"{'trajectory' if trajectory else 'summary'} mode: kernel {eng.kernel_ms():.3f} ms (stamped); cycles per wave-step (1440 steps) by section:")
for n, v in list(zip(names, b[:9]))[1:]:
    print(f"  {n:28s} {v / waves / 1440:9.1f}  {100.0 * v / tot:5.1f} %")
print(f"  shader clock ~ {tot / waves / (eng.kernel_ms() * 1e-3) / 1e9:.2f} GHz (stamped cycles per wave / kernel time)")
print(f"  iterations per wave {b[9] / waves:.1f} ({b[9] / waves / 1440:.3f} per step); event runs per wave "
      f"{b[10] / waves:.1f}; lanes per event run {b[11] / max(b[10], 1):.2f}; event lane-steps "
      f"{b[11] / (waves * lpw * 1440):.4f} of all; longest wave {b[0]} iterations")
