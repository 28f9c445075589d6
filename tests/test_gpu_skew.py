"""The general kernel's lane-skewed schedule (rollout_kernel<DMAX, MAXN, 0, 1>,
rollout_sk.hip): worlds of several HPA / static deployments run quiet steps per
lane and full steps in per-wave batches of stalled lanes. Each world runs on
the skewed schedule (engine 5), on the lockstep general kernel (engine 1,
ccka_debug_engine(2)) and on the CPU oracle: results, instance choices and
every trajectory record bit-exact. Reference side: the burst Deployments
sharing the Karpenter pools (demo_30_burst_configure.sh:57-151)
under HPA, the pool patches (demo_20_offpeak_configure.sh:59-81,
demo_21_peak_configure.sh:56-77) and the PDB (demo_10_setup_configure.sh:47-56)."""
import numpy as np
import pytest

import pyoracle as po
from ccka import abi, configs
from ccka.world import ScenarioSet, deployment, hpa_rules
from parity import compare, oracle, run_engine

pytestmark = pytest.mark.gpu
THREADS = 16
SPOT, OD = abi.CAP_SPOT, abi.CAP_OD


def hpa(cap, **kw):
    return deployment(abi.SCALER_HPA, cap_sel=cap, **kw)


def static(n, cap):
    return deployment(abi.SCALER_STATIC, n, n, n, cap_sel=cap)


def custom_rules():
    # a scale-up stabilisation window, rate limits with 60-240 s periods (the
    # register rings hold them: one decision per step, windows <= 8 steps)
    up = hpa_rules(abi.SELECT_MIN, [(abi.HPA_PERCENT, 50, 60), (abi.HPA_PODS, 3, 120)], 120)
    dn = hpa_rules(abi.SELECT_MAX, [(abi.HPA_PODS, 2, 240)], 180)
    return up, dn


def world(name):
    """(spec, scenarios) of each skewed-schedule world."""
    spec = configs.config2_world(n_steps=720)
    n = 1200
    sc = ScenarioSet(n, 5)
    if name == "d2_n8":
        spec.deploys = [hpa(SPOT), hpa(OD, req_cpu=400, target=60)]
    elif name == "d2_n8_overrides":  # per-scenario target / max / cap / peak switch / down window
        spec.deploys = [hpa(SPOT, replicas0=3, max_r=30, req_cpu=300),
                        hpa(SPOT | OD, replicas0=2, max_r=30, req_cpu=250, target=60)]
        sc = configs.hpa_scenarios(n, first_id=11)
        ids = np.arange(n)
        sc.peak_switch = (ids % 3 != 0).astype(np.uint8)
        sc.down_stab_s = (60 * (ids % 6)).astype(np.int16)
        sc.reset_ca_s = np.array([0, 30, 120, 300], np.int16)[ids % 4]
    elif name == "d2_n16_limits":  # CPU limits, memory requests, pool CPU limit, tolerance 0.05
        spec.max_nodes = 16
        spec.deploys = [hpa(SPOT, req_cpu=500, req_mem=900, limit_cpu=700, tol=0.05),
                        hpa(OD, req_cpu=350, limit_cpu=0, target=50, max_r=60)]
        spec.pools[0].limit_cpu_m = 24000
    elif name == "d3_n8_static":  # <4, 8>: two HPA + one static
        spec.deploys = [hpa(SPOT), static(4, SPOT | OD), hpa(OD, req_cpu=300, target=80)]
    elif name == "d4_n16_rules":  # non-default behavior rules, PDB 80 %, budget 50 %
        spec.max_nodes = 16
        up, dn = custom_rules()
        spec.deploys = [hpa(SPOT, up=up, down=dn), hpa(OD, req_cpu=300, target=60),
                        hpa(SPOT | OD, req_cpu=250, max_r=25, up=up, down=dn), static(3, OD)]
        spec.pdb_pct = 80
        for p in spec.pools:
            p.budget_pct = 50
    elif name == "d4_n8_delay0":  # nodes ready in the step they launch; wrapped peak window
        spec.deploys = [hpa(SPOT), hpa(OD, target=60), hpa(SPOT, req_cpu=150), hpa(OD, req_cpu=450, target=80)]
        spec.provision_delay_steps = 0
        spec.peak_start, spec.peak_end, spec.start_minute = 1380, 120, 1200
    elif name == "d4_n16_delay3":
        spec.max_nodes = 16
        spec.deploys = [hpa(SPOT), hpa(OD, target=60), hpa(SPOT, req_cpu=150), hpa(OD, req_cpu=450, target=80)]
        spec.provision_delay_steps = 3
        spec.carbon_weight = 1.0
    elif name == "d8_n16":
        spec.max_nodes = 16
        spec.deploys = [hpa(SPOT if d % 2 else OD, target=(50, 60, 70, 80)[d % 4], max_r=12, replicas0=2,
                            req_cpu=(200, 300, 250, 400)[d % 4]) for d in range(8)]
        n = 600
        sc = ScenarioSet(n, 9)
    elif name == "d12_n16":  # the bench's --deployments 12 shape (demo_30: alternating spot / on-demand)
        spec.max_nodes = 16
        spec.deploys = [hpa(SPOT if d % 2 == 0 else OD, replicas0=5, max_r=10,
                            req_cpu=(200, 300, 250, 400)[d % 4], target=(70, 60, 80, 50)[d % 4])
                        for d in range(12)]
        n = 400
        sc = ScenarioSet(n, 13)
    elif name == "config1_static12":  # the reference's own burst: 12 static Deployments x 5 replicas
        spec = configs.config1_world()
        spec.n_steps = 720
        n = 256
        sc = ScenarioSet(n, 0)
    else:
        raise KeyError(name)
    return spec, sc


NAMES = ["d2_n8", "d2_n8_overrides", "d2_n16_limits", "d3_n8_static", "d4_n16_rules", "d4_n8_delay0",
         "d4_n16_delay3", "d8_n16", "d12_n16", "config1_static12"]
# more than four deployments keep the lockstep kernel (its state would spill: slower, sk_eligible)
SKEWED = {n for n in NAMES if n not in ("d8_n16", "d12_n16", "config1_static12")}


@pytest.mark.parametrize("name", NAMES)
def test_skewed_schedule_matches_oracle_and_lockstep(engine, name):
    spec, sc = world(name)
    load = po.gen_load(configs.trace_gen(23), spec.n_steps, len(spec.deploys), sc.n, first_id=sc.first_id)
    try:
        rs, ts = run_engine(engine, spec, sc, load=load, traj=True)
        assert engine.last_engine()[0] == (5 if name in SKEWED else 1), "engine choice"
        engine.set_engine(2)
        rl, tl = run_engine(engine, spec, sc, load=load, traj=True)
        assert engine.last_engine()[0] == 1
    finally:
        engine.set_engine(0)
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    assert rc["launches"].sum() > 0
    compare(rs, rc, ts, tc)
    compare(rl, rc, tl, tc)


def test_skewed_schedule_summary_mode(engine):
    """Without a trajectory (the records' buffer absent) the results are the same."""
    spec, sc = world("d2_n8_overrides")
    load = po.gen_load(configs.trace_gen(29), spec.n_steps, len(spec.deploys), sc.n, first_id=sc.first_id)
    rs, _ = run_engine(engine, spec, sc, load=load, traj=False)
    assert engine.last_engine()[0] == 5
    rc, _ = oracle(spec, sc, load, traj=False, threads=THREADS)
    compare(rs, rc)


def test_skewed_schedule_not_used_where_it_does_not_hold(engine):
    """KEDA, drift and 15 s sync worlds keep the lockstep kernel."""
    spec, sc = world("d2_n8")
    load = po.gen_load(configs.trace_gen(31), spec.n_steps, 2, sc.n, first_id=sc.first_id)
    for mut in ("keda", "drift", "sync15"):
        s2, _ = world("d2_n8")
        if mut == "keda":
            s2.deploys[1] = deployment(abi.SCALER_KEDA, replicas0=0, keda_threshold=800, cap_sel=OD)
        elif mut == "drift":
            s2.drift = 1
        else:
            s2.hpa_sync_s = 15
        rg, tg = run_engine(engine, s2, sc, load=load, traj=True)
        assert engine.last_engine()[0] == 1, mut
        rc, tc = oracle(s2, sc, load, traj=True, threads=THREADS)
        compare(rg, rc, tg, tc)
    del spec


@pytest.mark.parametrize("name", ["d2_n8_overrides", "d2_n16_limits", "d4_n8_delay0"])
def test_skewed_schedule_cooperative_provisioning(engine, name):
    """ccka_debug_engine(3) (the skewed schedule with the wave-cooperative scans
    forced; builds with SK_LANE_F2 otherwise provision lane-locally for small
    catalogs) and the default give the oracle's launches, bit for bit."""
    spec, sc = world(name)
    load = po.gen_load(configs.trace_gen(37), spec.n_steps, len(spec.deploys), sc.n, first_id=sc.first_id)
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    for mode in (0, 3):
        try:
            engine.set_engine(mode)
            rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
            assert engine.last_engine()[0] == 5
        finally:
            engine.set_engine(0)
        compare(rg, rc, tg, tc)
