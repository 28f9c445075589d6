"""Profiling aid: config-2 trajectory rollouts on the main build or a
tools/build_variants.py variant (--variant=name), for rocprofv3 passes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd"))
from ccka import configs  # noqa: E402
from ccka.engine import Engine  # noqa: E402

lib = None
for a in sys.argv[1:]:
    if a.startswith("--variant="):
        lib = os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd", "csrc", "build", "variants",
                           a.split("=", 1)[1], "libccka.so")
eng = Engine(0, lib_path=lib) if lib else Engine(0)
eng.set_world(configs.config2_world())
eng.set_scenarios(configs.hpa_scenarios(100_000))
eng.gen_load(configs.trace_gen())
for _ in range(3):
    eng.rollout(trajectory=True)
    print(f"kernel {eng.kernel_ms():.3f} ms", flush=True)
