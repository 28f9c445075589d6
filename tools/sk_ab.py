"""A/B of the skewed schedule's provisioning paths (ccka_debug_engine 0: lane-local
NodeClaims where they fit in LDS, 3: the wave-cooperative scans) and of the lockstep
kernel (2) on bench.py's --deployments worlds (1e5 x 1440, trajectory mode).
Results must be identical across modes. SK_AB_LIBS=main,NAME,...: the main build and
variant builds (csrc/build/variants/NAME), mode 0 only, results compared with the main
build's. usage: python tools/sk_ab.py [N]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd"))
from ccka import abi, configs  # noqa: E402
from ccka.engine import Engine  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
LIBS = [x for x in os.environ.get("SK_AB_LIBS", "").split(",") if x]
VDIR = os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd", "csrc", "build", "variants")
engs = [(n, Engine(0, lib_path=None if n == "main" else os.path.join(VDIR, n, "libccka.so"))) for n in LIBS]
e = Engine(0) if not engs else engs[0][1]
for nd, slots in ((2, 8), (2, 16), (4, 8), (4, 16)):
    spec = configs.config2_world()
    spec.deploys = [configs.deployment(abi.SCALER_HPA, replicas0=3, max_r=30, req_cpu=(200, 300, 250, 400)[d % 4],
                                       target=(70, 60, 80, 50)[d % 4]) for d in range(nd)]
    spec.max_nodes = slots
    e.set_world(spec)
    e.set_scenarios(configs.hpa_scenarios(N))
    e.gen_load(configs.trace_gen())
    ref = None
    if engs:
        for n, en in engs:
            en.set_world(spec)
            en.set_scenarios(configs.hpa_scenarios(N))
            en.gen_load(configs.trace_gen())
            ms = []
            for _ in range(3):
                en.rollout(trajectory=True)
                ms.append(en.kernel_ms())
            r = en.results()
            ref = r if ref is None else ref
            same = all(np.array_equal(r[k], ref[k]) for k in ref)
            print(f"{nd} deployments x {slots} slots {n}: engine {en.last_engine()[0]} kernel ms "
                  f"{sorted(ms)[1]:.2f} same={same}", flush=True)
        continue
    for mode in (0, 3, 2):
        e.set_engine(mode)
        ms = []
        for _ in range(3):
            e.rollout(trajectory=True)
            ms.append(e.kernel_ms())
        r = e.results()
        if ref is None:
            ref = r
        same = all(np.array_equal(r[k], ref[k]) for k in ref)
        print(f"{nd} deployments x {slots} slots mode {mode}: engine {e.last_engine()[0]} kernel ms "
              f"{sorted(ms)[1]:.2f} same={same}", flush=True)
    e.set_engine(0)
