"""Throughput of the general kernel on multi-deployment worlds (profiling aid):
the config-1 burst (12 static deployments, 16 node slots) and HPA mixes of
2 / 4 / 12 deployments at N scenarios x 1440 steps, summary mode.
usage: python tools/multi_bench.py [N]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd"))
from ccka import abi, configs  # noqa: E402
from ccka.engine import Engine  # noqa: E402
from ccka.world import deployment  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 and __name__ == "__main__" else 100_000


def hpa_mix(d, max_nodes):
    w = configs.config2_world(max_nodes=max_nodes)
    w.deploys = [deployment(abi.SCALER_HPA, replicas0=3, max_r=30, target=(50, 60, 70, 80)[i % 4],
                            cap_sel=abi.CAP_SPOT if i % 2 == 0 else abi.CAP_OD) for i in range(d)]
    return w


def hpa1(max_nodes, inert=0):
    w = configs.config2_world(max_nodes=max_nodes)
    w.deploys = w.deploys + [deployment(abi.SCALER_STATIC, 0, 0, 0) for _ in range(inert)]
    return w


worlds = {
    "hpa1_8_general": lambda: hpa1(8),
    "hpa1_16_general": lambda: hpa1(16),
    "hpa1+static0_16": lambda: hpa1(16, 1),
    "burst12_static_16": lambda: configs.config1_world(),
    "hpa2_8": lambda: hpa_mix(2, 8),
    "hpa4_16": lambda: hpa_mix(4, 16),
    "hpa12_16": lambda: hpa_mix(12, 16),
}



def main():
    names = sys.argv[2:] or list(worlds)
    LIB = os.environ.get("VARIANT")  # a tools/build_variants.py variant instead of the main build
    e = Engine(0, lib_path=os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd", "csrc", "build",
                                        "variants", LIB, "libccka.so") if LIB else None)
    import ctypes as C  # noqa: E402
    e.lib.ccka_debug_engine.argtypes = [C.c_void_p, C.c_int32]
    e.lib.ccka_debug_engine(e.ctx, 1)  # the general kernel for every world
    ABL = [int(x) for x in os.environ.get("ABLATE", "0").split(",")]  # profiling: ccka_debug_ablate masks
    e.lib.ccka_debug_ablate.argtypes = [C.c_void_p, C.c_int32]
    for name, abl in [(n, a) for n in names for a in ABL]:
        e.lib.ccka_debug_ablate(e.ctx, abl)
        w = worlds[name]()
        e.set_world(w)
        e.set_scenarios(configs.hpa_scenarios(N))
        e.gen_load(configs.trace_gen())
        t0 = time.time()
        e.rollout(trajectory=False)
        first = time.time() - t0
        ms = []
        for _ in range(3):
            e.rollout(trajectory=False)
            ms.append(e.kernel_ms())
        eng = e.last_engine()[0]
        m = sorted(ms)[1]
        print(f"{name:20s} ablate={abl:2d} D={len(w.deploys):2d} slots={w.max_nodes:2d} engine={eng} kernel {m:9.2f} ms "
              f"{N * w.n_steps / m * 1e3:.3e} cluster-steps/s (first call {first:.1f} s)", flush=True)


if __name__ == "__main__":
    main()
