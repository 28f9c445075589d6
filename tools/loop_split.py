"""Time split of the fused closed loop (profiling aid): the config-5 loop at
N scenarios x T steps as shipped, without its MLP (ablate bit 32: actions from
zero outputs, the rollout logic and features alone), with the catalog scans
instead of the argmin tables for its launches, phase ablations, and the
launched loop
(general kernel + mlp_kernel + policy_act_kernel per step, hipGraph).
usage: python tools/loop_split.py [N] [T]"""
import ctypes as C
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd"))
from ccka import configs  # noqa: E402
from ccka.engine import Engine  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
T = int(sys.argv[2]) if len(sys.argv) > 2 else 60
eng = Engine(0)
ws, bs = configs.mlp_weights(11)
eng.mlp_set_weights([configs.to_bf16_bits(w) for w in ws], bs)
eng.set_world(configs.config2_world(n_steps=T))
eng.set_scenarios(configs.hpa_scenarios(N))
eng.gen_load(configs.trace_gen())
eng.lib.ccka_debug_ablate.argtypes = [C.c_void_p, C.c_int32]
eng.lib.ccka_debug_policy_fused.argtypes = [C.c_void_p, C.c_int32]
eng.lib.ccka_debug_policy_table.argtypes = [C.c_void_p, C.c_int32]
# ablations (bits of ccka_debug_ablate; they change the dynamics, so they bound
# a phase's share rather than measure it): 32 no MLP, 1 no disruption, 2 no
# provisioning, 8 no HPA behavior
MODES = (("fused", 1, 0), ("fused, catalog scans", 2, 0), ("fused, no MLP", 1, 32), ("  - disruption", 1, 33),
         ("  - provisioning", 1, 34), ("  - both", 1, 35), ("  - HPA behavior", 1, 40), ("launched (graph)", 0, 0))
for name, fused, abl in MODES:
    eng.lib.ccka_debug_policy_fused(eng.ctx, 1 if fused else 0)
    eng.lib.ccka_debug_policy_table(eng.ctx, 0 if fused == 2 else 1)  # 2: launches by catalog scans
    eng.lib.ccka_debug_ablate(eng.ctx, abl)
    ms = []
    for _ in range(3):
        eng.policy_rollout()
        ms.append(eng.kernel_ms())
    print(f"{name:18s} {min(ms):9.3f} ms per loop  {min(ms) / T:7.3f} ms per step", flush=True)
eng.lib.ccka_debug_ablate(eng.ctx, 0)
