"""Timing of general-kernel variants (tools/build_variants.py NAME=r@file.hip)
on the fused closed loop (config 5 world, N scenarios x T steps), interleaved
rounds in one process; every variant's results, recorded actions and sampled
policy-gradient loop must equal the main build's bit for bit. Profiling aid.
usage: python tools/variant_loop.py [N] [variant names...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd"))
from ccka import abi, configs  # noqa: E402
from ccka.engine import Engine  # noqa: E402

CSRC = os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd", "csrc", "build")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
T = 60
names = sys.argv[2:]
libs = [("main", abi.ENGINE_LIB)] + [(n, os.path.join(CSRC, "variants", n, "libccka.so")) for n in names]
ws, bs = configs.mlp_weights(11)
engs = {}
for n, path in libs:
    e = Engine(0, lib_path=path)
    e.mlp_set_weights([configs.to_bf16_bits(w) for w in ws], bs)
    e.set_world(configs.config2_world(n_steps=T))
    e.set_scenarios(configs.hpa_scenarios(N))
    e.gen_load(configs.trace_gen())
    engs[n] = e
times = {n: [] for n, _ in libs}
ref = None
for r in range(4):
    for n, _ in libs:
        e = engs[n]
        e.policy_rollout(trajectory=False, record=r == 0)
        times[n].append(e.kernel_ms())
        if r == 0:
            got = (e.results(), e.policy_actions())
            e.policy_grad(seed=7, w_carbon=0.05, w_slo=0.01)
            got = got + (e.results(),)
            if ref is None:
                ref = got
            for k in ref[0]:
                assert np.array_equal(got[0][k], ref[0][k]), f"{n}: results {k}"
                assert np.array_equal(got[2][k], ref[2][k]), f"{n}: sampled-loop results {k}"
            assert all(np.array_equal(a, b) for a, b in zip(got[1], ref[1])), f"{n}: actions"
for n, _ in libs:
    v = sorted(times[n])
    print(f"{n:12s} median {v[1]:.3f} ms  min {v[0]:.3f} ms per loop ({N} x {T})", flush=True)
