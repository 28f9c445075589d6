"""Phase attribution of the general kernel (rollout_kernel) from s_memtime
stamps: the GK_STAMPS variant (python tools/build_variants.py
gks="r@rollout.hip:-DGK_STAMPS"), run with the diagnostic ablate bit 16 (the
stamp buffer; results are the real ones, timings inflated by the stamps).
Worlds: tools/multi_bench.py's, plus "loop" (the fused closed loop, config-2
world, N x 60). usage: python tools/gk_stamps.py [N] [world names...]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from ccka import configs  # noqa: E402
from ccka.engine import Engine  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
names = sys.argv[2:] or ["hpa1_8_general", "hpa2_8", "hpa4_16", "loop"]
sys.argv = sys.argv[:1]
import multi_bench as mb  # noqa: E402  (its world builders; its own run is skipped by __name__)

PHASES = ["samples+hour", "readiness+profile", "scalers", "reconcile+sched", "provisioning", "disruption",
          "accounting+record", "policy: features", "policy: MLP tile a", "policy: MLP tile b", "policy: action"]
lib = os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd", "csrc", "build", "variants", "gks",
                   "libccka.so")
e = Engine(0, lib_path=lib)
e.lib.ccka_debug_engine.argtypes = [C.c_void_p, C.c_int32]
e.lib.ccka_debug_ablate.argtypes = [C.c_void_p, C.c_int32]
e.lib.ccka_debug_stamps.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
for name in names:
    if name == "loop":
        T = 60
        w = configs.config2_world(n_steps=T)
        ws, bs = configs.mlp_weights(11)
        e.mlp_set_weights([configs.to_bf16_bits(x) for x in ws], bs)
    else:
        w = mb.worlds[name]()
        T = w.n_steps
    e.lib.ccka_debug_engine(e.ctx, 1)
    e.set_world(w)
    e.set_scenarios(configs.hpa_scenarios(N))
    e.gen_load(configs.trace_gen())
    e.lib.ccka_debug_ablate(e.ctx, 16)
    if name == "loop":
        e.policy_rollout(trajectory=False)
    else:
        e.rollout(trajectory=False)
    ms = e.kernel_ms()
    buf = (C.c_ulonglong * 12)()
    assert e.lib.ccka_debug_stamps(e.ctx, buf) == 0
    e.lib.ccka_debug_ablate(e.ctx, 0)
    waves = max(buf[11], 1)
    tot = sum(buf[k] for k in range(11)) or 1
    print(f"{name}: kernel {ms:.2f} ms (stamped), {waves} waves x {T} steps; cycles per wave-step by phase:")
    for k in range(11):
        if buf[k]:
            print(f"  {PHASES[k]:22s} {buf[k] / waves / T:9.1f}  {100 * buf[k] / tot:5.1f} %")
