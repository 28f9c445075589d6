"""Phase-ablation timing of the rollout kernel (profiling aid; ablated results
are meaningless). Interleaved rounds in one process (guide §5.4 rule 24).
The switches exist only in a variant build: python tools/build_variants.py
abl=-DCCKA_ABLATE_BUILD=1, then LIB=<its libccka.so> python tools/ablate.py."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd"))
from ccka import configs  # noqa: E402
from ccka.engine import Engine  # noqa: E402

masks = [int(x) for x in (sys.argv[1:] or ["0", "1", "2", "4", "8", "15"])]
eng = Engine(0, lib_path=os.environ.get("LIB"))
eng.lib.ccka_debug_ablate.argtypes = [C.c_void_p, C.c_int32]
eng.set_world(configs.config2_world())
eng.set_scenarios(configs.hpa_scenarios(100_000))
eng.gen_load(configs.trace_gen())
res = {m: [] for m in masks}
for r in range(4):
    for m in masks:
        eng.lib.ccka_debug_ablate(eng.ctx, m)
        eng.rollout(trajectory=True)
        if r:
            res[m].append(eng.kernel_ms())
for m in masks:
    v = sorted(res[m])
    print(f"mask {m:2d}: median {v[len(v) // 2]:8.3f} ms  min {v[0]:8.3f}")
