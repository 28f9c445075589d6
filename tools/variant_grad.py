"""Wall time of ccka_policy_grad (config-5 world, N scenarios x 60 steps) for
pg.hip variants (tools/build_variants.py NAME=p@file.hip), interleaved in one
process; gradients must equal the main build's unless NOCHECK is set (timing
ablations). Profiling aid only.
usage: [NOCHECK=1] python tools/variant_grad.py [N] [variant names...]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd"))
from ccka import abi, configs  # noqa: E402
from ccka.engine import Engine  # noqa: E402

CSRC = os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd", "csrc", "build")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 250_000
libs = [("main", abi.ENGINE_LIB)] + [(n, os.path.join(CSRC, "variants", n, "libccka.so")) for n in sys.argv[2:]]
ws, bs = configs.mlp_weights(11)
engs = {}
for n, path in libs:
    e = Engine(0, lib_path=path)
    e.mlp_set_weights([configs.to_bf16_bits(w) for w in ws], bs)
    e.set_world(configs.config2_world(n_steps=60))
    e.set_scenarios(configs.hpa_scenarios(N))
    e.gen_load(configs.trace_gen())
    e.policy_grad(seed=1, w_carbon=0.05, w_slo=0.01)  # warm-up (allocations)
    engs[n] = e
times = {n: [] for n, _ in libs}
ref = None
for r in range(5):
    for n, _ in libs:
        t0 = time.perf_counter()
        g, _ = engs[n].policy_grad(seed=2, w_carbon=0.05, w_slo=0.01)
        times[n].append((time.perf_counter() - t0) * 1e3)
        if r == 0 and not os.environ.get("NOCHECK"):
            if ref is None:
                ref = g
            assert all(np.array_equal(g[k], ref[k]) for k in ref), f"{n}: gradients differ"
for n, _ in libs:
    v = sorted(times[n])
    print(f"{n:12s} median {v[2]:.2f} ms  min {v[0]:.2f} ms per gradient ({N} x 60)", flush=True)
