"""KEDA ScaledObject worlds on the single-deployment kernel (its KEDA
instantiation, SEMANTICS 3.C: activation, scale from zero, scale to zero after
the cooldown, proposal ceil(metric / threshold) outside the tolerance band,
default behavior): results and trajectories bit-exact against the CPU oracle,
and the engine that ran them is the single-deployment one (last_engine 2).
Worlds the instantiation does not cover (drift, pool limits, 15 s sync) run on
the general kernel with the same results. Reference side: the queue-worker
path the reference stubs (.env:10-12; SURVEY a15, Appendix A.2 defaults)."""
import numpy as np
import pytest

import pyoracle as po
from ccka import abi, configs
from ccka.world import deployment, default_down
from parity import compare, oracle, run_engine

pytestmark = pytest.mark.gpu
THREADS = 16


def keda_world(T=1440, **kw):
    spec = configs.config2_world(n_steps=T)
    args = dict(replicas0=0, keda_threshold=500, keda_activation=0, keda_cooldown=300, keda_min=0, keda_max=100)
    args.update(kw)
    spec.deploys = [deployment(abi.SCALER_KEDA, **args)]
    return spec


CASES = {
    # SURVEY A.2 defaults: scale from / to zero, cooldown 300 s
    "defaults": dict(),
    # an activation threshold the trace crosses: long idle stretches at zero
    "activation": dict(keda_activation=1800, keda_threshold=700),
    # minReplicaCount 1: no scale to zero, no cooldown
    "min1": dict(keda_min=1, replicas0=3),
    # cooldown 0 (scale to zero at the first inactive step) and a low maximum
    "cool0_max": dict(keda_cooldown=0, keda_activation=2500, keda_max=6),
    # a 10-minute cooldown and a 480 s down window (the 8-record ring)
    "long_windows": dict(keda_cooldown=600, keda_activation=1200, down=default_down(480)),
    # a large threshold: the tolerance band around every count is wide
    "big_threshold": dict(keda_threshold=4000, keda_activation=100, replicas0=2),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_keda_single_deployment_parity(engine, case):
    spec = keda_world(**CASES[case])
    sc = configs.hpa_scenarios(2113, first_id=17)  # ragged; cap_sel alternates spot / on-demand
    load = po.gen_load(configs.trace_gen(21), spec.n_steps, 1, sc.n, first_id=17)
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    assert engine.last_engine()[0] == 2, "the KEDA world should run on the single-deployment kernel"
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    assert rc["launches"].sum() > 0
    compare(rg, rc, tg, tc)
    reps = tc["replicas"]
    if case in ("activation", "cool0_max", "long_windows"):
        assert (reps[1:] == 0).any() and (reps > 0).any()  # scaled to zero and back


@pytest.mark.parametrize("lpw", [1, 33, 64])
def test_keda_lane_schedules(engine, lpw):
    """Any scenarios per wave (the lane-skewed schedule) on the KEDA instantiation."""
    import ctypes as C
    spec = keda_world(T=700, keda_activation=1500)
    sc = configs.hpa_scenarios(777, first_id=5)
    load = po.gen_load(configs.trace_gen(3), spec.n_steps, 1, sc.n, first_id=5)
    lp = engine.lib.ccka_debug_lpw
    lp.argtypes = [C.c_void_p, C.c_int32]
    assert lp(engine.ctx, lpw) == 0
    try:
        rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
        assert engine.last_engine()[0] == 2
    finally:
        lp(engine.ctx, 0)
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    compare(rg, rc, tg, tc)


@pytest.mark.parametrize("variant", ["drift", "pool_limit", "sync15"])
def test_keda_general_kernel_fallback(engine, variant):
    spec = keda_world(T=600, keda_activation=1500)
    if variant == "drift":
        spec.drift = 1
    elif variant == "pool_limit":
        for p in spec.pools:
            p.limit_cpu_m = 9000
    else:
        spec.hpa_sync_s = 15
    sc = configs.hpa_scenarios(640, first_id=9)
    load = po.gen_load(configs.trace_gen(4), spec.n_steps, 1, sc.n, first_id=9)
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    assert engine.last_engine()[0] == 1
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    compare(rg, rc, tg, tc)


def test_keda_negative_and_edge_metrics(engine):
    """Metric samples at the activation threshold, zero, negative and very
    large (beyond the quiet steps' 2^20 range): every step the exact path
    decides matches the oracle."""
    spec = keda_world(T=240, keda_activation=1000, keda_threshold=333, keda_cooldown=120)
    n = 300
    sc = configs.hpa_scenarios(n, first_id=1)
    rng = np.random.default_rng(5)
    load = po.gen_load(configs.trace_gen(8), spec.n_steps, 1, n, first_id=1).copy()
    mask = rng.random(load.shape) < 0.05
    special = rng.choice(np.array([0, 1000, 1001, -1, -5000, 1 << 21, 2_000_000_000, 999], np.int32),
                         size=load.shape)
    load[mask] = special[mask]
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    assert engine.last_engine()[0] == 2
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    compare(rg, rc, tg, tc)
