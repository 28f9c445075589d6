"""The pooled single-deployment engine (rollout_pool.hip: scenario state in LDS,
a workgroup event queue served by any wave; an A/B engine, off by default,
DESIGN.md "Pooled event steps, built and measured") against the CPU oracle:
results and trajectories bit-exact, the pooled kernel asserted to have run."""
import numpy as np
import pytest

import pyoracle as po
from ccka import abi, configs
from ccka.world import ScenarioSet, deployment
from parity import compare, oracle, run_engine

pytestmark = pytest.mark.gpu


def _pooled(engine, spec, sc, load, min_queue=48):
    engine.debug_pool(1, min_queue)
    try:
        rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
        assert engine.last_engine()[0] == 2 and engine.debug_pool() == 1
    finally:
        engine.debug_pool(0)
    return rg, tg


@pytest.mark.parametrize("min_queue", [16, 64])
def test_pooled_config2_parity(engine, min_queue):
    spec = configs.config2_world()
    sc = configs.hpa_scenarios(4099)  # ragged: a partial last workgroup and wave
    load = po.gen_load(configs.trace_gen(), spec.n_steps, 1, sc.n)
    rg, tg = _pooled(engine, spec, sc, load, min_queue)
    rc, tc = oracle(spec, sc, load, traj=True, threads=16)
    compare(rg, rc, tg, tc)


def test_pooled_keda_parity(engine):
    spec = configs.config2_world(n_steps=720)
    spec.deploys = [deployment(abi.SCALER_KEDA, replicas0=0, keda_threshold=700, keda_activation=300,
                               keda_cooldown=180, keda_min=0, keda_max=40)]
    sc = ScenarioSet(2113, 5)
    load = po.gen_load(configs.trace_gen(9), spec.n_steps, 1, sc.n, first_id=5)
    rg, tg = _pooled(engine, spec, sc, load)
    rc, tc = oracle(spec, sc, load, traj=True, threads=16)
    assert rc["launches"].sum() > 0
    compare(rg, rc, tg, tc)


def test_pooled_cheap_large_types(engine):
    spec = configs.cheap_large_world()
    sc = configs.hpa_scenarios(1500, first_id=31)
    load = po.gen_load(configs.trace_gen(), spec.n_steps, 1, sc.n, first_id=31)
    rg, tg = _pooled(engine, spec, sc, load)
    rc, tc = oracle(spec, sc, load, traj=True, threads=16)
    compare(rg, rc, tg, tc)
