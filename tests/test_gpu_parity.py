"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle on the
same seeded inputs. Integers, instance choices and trajectories bit-exact;
fp64 energy/gCO2 within 1e-9 relative (observed bit-exact)."""
import numpy as np
import pytest

import pyoracle as po
from ccka import abi, configs
from ccka.world import ScenarioSet, deployment
from parity import compare, oracle, run_engine

pytestmark = pytest.mark.gpu
THREADS = 16


def test_engine_abi(engine):
    assert engine.lib.ccka_abi_version() == abi.ABI_VERSION
    name, cus = engine.device_info()
    assert "gfx950" in name and cus >= 200


def test_gen_load_matches_oracle(engine):
    spec = configs.config2_world(n_steps=1440)
    sc = configs.hpa_scenarios(3000, first_id=123457)
    engine.set_world(spec)
    engine.set_scenarios(sc)
    engine.gen_load(configs.trace_gen())
    got = engine.get_load()
    want = po.gen_load(configs.trace_gen(), 1440, 1, 3000, first_id=123457)
    assert np.array_equal(got, want)


def test_config2_parity_trajectory(engine):
    spec = configs.config2_world()
    sc = configs.hpa_scenarios(4099)  # ragged: not a multiple of 64/256
    load = po.gen_load(configs.trace_gen(), spec.n_steps, 1, sc.n)
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    assert rc["launches"].sum() > 0 and rc["deletions"].sum() > 0
    compare(rg, rc, tg, tc)


def test_config2_totals(engine):
    spec = configs.config2_world()
    sc = configs.hpa_scenarios(5000, first_id=77)
    load = po.gen_load(configs.trace_gen(), spec.n_steps, 1, sc.n, first_id=77)
    run_engine(engine, spec, sc, load=load)
    tg = engine.totals()
    rc, _ = oracle(spec, sc, load, threads=THREADS)
    tc = po.totals(rc, sc.n)
    for f in ["scenarios", "cost_uphmin", "slo_minutes", "pending_pod_minutes", "node_min_spot",
              "node_min_od", "launches", "deletions"]:
        assert getattr(tg, f) == getattr(tc, f), f
    for f in ["energy_wmin", "gco2"]:
        assert abs(getattr(tg, f) - getattr(tc, f)) <= 1e-9 * abs(getattr(tc, f)), f


def test_config3_catalog800_regions(engine):
    """~800-type catalog in LDS, 8 regions with region blocks small enough that
    workgroups straddle regions (2 price tiles staged), carbon-weighted argmin,
    10 % of spot offerings unavailable."""
    spec = configs.config3_world()
    n = 3000
    sc = configs.hpa_scenarios(n, 0, 8, 350, configs.CONFIG3_CARBON)
    load = po.gen_load(configs.trace_gen(), spec.n_steps, 1, n)
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    assert len(set(rc["last_choice"] & 0xFFF)) > 5  # several instance types chosen
    compare(rg, rc, tg, tc)


def test_config1_replay_12_deployments(engine):
    spec = configs.config1_world()
    sc = ScenarioSet(1)
    load = np.zeros((spec.n_steps, 12, 1), np.int32) + 100
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    rc, tc = oracle(spec, sc, load, traj=True)
    assert rc["final_replicas"][0] == 60
    compare(rg, rc, tg, tc)


def test_multi_deployment_hpa_keda(engine):
    """3 deployments (HPA spot, HPA on-demand with bigger pods, KEDA) sharing nodes."""
    spec = configs.config2_world(max_nodes=12)
    spec.deploys = [
        deployment(abi.SCALER_HPA, cap_sel=abi.CAP_SPOT),
        deployment(abi.SCALER_HPA, req_cpu=500, req_mem=512, limit_cpu=1000, cap_sel=abi.CAP_OD, target=60),
        deployment(abi.SCALER_KEDA, replicas0=0, keda_threshold=800, keda_activation=1500,
                   keda_cooldown=300, cap_sel=abi.CAP_SPOT | abi.CAP_OD),
    ]
    n = 700
    sc = ScenarioSet(n)
    load = po.gen_load(configs.trace_gen(9), spec.n_steps, 3, n)
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    compare(rg, rc, tg, tc)


@pytest.mark.parametrize("variant", ["one_slot", "pool_limit", "no_pdb", "wrap_peak", "delay3",
                                     "zero_load", "single", "no_switch"])
def test_edge_cases(engine, variant):
    spec = configs.config2_world(n_steps=600)
    n = 513
    sc = configs.hpa_scenarios(n)
    gen = configs.trace_gen(5)
    if variant == "one_slot":
        spec.max_nodes = 1
    elif variant == "pool_limit":
        for p in spec.pools:
            p.limit_cpu_m = 8000
    elif variant == "no_pdb":
        spec.pdb_pct = -1
    elif variant == "wrap_peak":
        spec.peak_start, spec.peak_end, spec.start_minute = 1300, 200, 1200
    elif variant == "delay3":
        spec.provision_delay_steps = 3
    elif variant == "single":
        n = 1
        sc = configs.hpa_scenarios(1, first_id=41)
    elif variant == "no_switch":
        sc.peak_switch = np.zeros(n, np.uint8)
    load = po.gen_load(gen, spec.n_steps, 1, n, first_id=sc.first_id)
    if variant == "zero_load":
        load[:] = 0
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    compare(rg, rc, tg, tc)


def test_sharding_invariance(engine):
    """Scenarios are independent: two shards (with their global ids) reproduce
    the unsharded run exactly, including device-generated traces."""
    spec = configs.config2_world(n_steps=720)
    n = 2000
    full = configs.hpa_scenarios(n)
    rf, _ = run_engine(engine, spec, full, gen=configs.trace_gen())
    parts = []
    for lo, hi in [(0, 1234), (1234, n)]:
        r, _ = run_engine(engine, spec, full.slice(lo, hi), gen=configs.trace_gen())
        parts.append(r)
    for f in rf:
        assert np.array_equal(rf[f], np.concatenate([parts[0][f], parts[1][f]])), f


def test_deterministic_rerun(engine):
    spec = configs.config2_world(n_steps=720)
    sc = configs.hpa_scenarios(1500)
    r1, t1 = run_engine(engine, spec, sc, gen=configs.trace_gen(), traj=True)
    engine.rollout(trajectory=True)
    r2, t2 = engine.results(), engine.trajectory()
    for f in r1:
        assert np.array_equal(r1[f], r2[f]), f
    assert np.array_equal(t1, t2)
