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
    # int64 sums (energy / gCO2 in fixed point) and the doubles derived from
    # them: bit-identical to the oracle's serial totals
    for f, _ in abi.Totals._fields_:
        assert getattr(tg, f) == getattr(tc, f), f
    # and within the north star's 1e-9 of the plain fp64 sums
    assert abs(tg.gco2 - rc["gco2"].sum()) <= 1e-9 * rc["gco2"].sum()
    assert abs(tg.energy_wmin - rc["energy_wmin"].sum()) <= 1e-9 * rc["energy_wmin"].sum()


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


def test_larger_type_wins_small_claim(engine):
    """A claim of a few pods won by a much larger type: the launched node holds
    its type's pod capacity, not the claim's capacity bracket (the argmin
    tables carry the winner's capacity). Both engines against the oracle."""
    spec = configs.cheap_large_world()
    sc = configs.hpa_scenarios(2000)
    load = po.gen_load(configs.trace_gen(), spec.n_steps, 1, sc.n)
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    kinds = set((rc["last_choice"] & 0xFFF).tolist())
    assert kinds and kinds <= {3, 7, 11, 15}  # only 4xlarge types launch
    for mode in (0, 1):  # automatic (single-deployment engine), general kernel
        engine.set_engine(mode)
        try:
            rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
            assert engine.last_engine()[0] == (2 if mode == 0 else 1)
        finally:
            engine.set_engine(0)
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


# ---------------------------------------------------------------------------
# single-deployment engine (rollout_d1.hip) vs general kernel vs oracle
# ---------------------------------------------------------------------------
def test_engine_selection(engine):
    spec = configs.config2_world(n_steps=60)
    sc = configs.hpa_scenarios(300)
    load = po.gen_load(configs.trace_gen(), spec.n_steps, 1, sc.n)
    run_engine(engine, spec, sc, load=load)
    assert engine.last_engine()[0] == 2  # config 2 runs on the single-deployment kernel
    for p in spec.pools:
        p.limit_cpu_m = 8000  # pool limits: launch choice depends on pool usage
    run_engine(engine, spec, sc, load=load)
    assert engine.last_engine()[0] == 1


def _sweep_scenarios(n, first_id=0):
    """config-4-style per-scenario policy parameters (targets, down-stabilisation
    windows, consolidateAfter, peak switch, carbon weights, capacity types)."""
    ids = np.arange(first_id, first_id + n, dtype=np.uint64)
    sc = configs.hpa_scenarios(n, first_id, 1, None, (0.0, 0.5, 1.0, 2.0))
    sc.target_util_pct = (40 + 3 * (configs.splitmix32(ids, 11) % 16)).astype(np.int16)
    sc.down_stab_s = (60 * (configs.splitmix32(ids, 12) % 8)).astype(np.int16)
    sc.reset_ca_s = np.array([30, 60, 120, 300], np.int16)[configs.splitmix32(ids, 13) % 4]
    sc.peak_switch = (configs.splitmix32(ids, 14) % 2).astype(np.uint8)
    sc.cap_sel = (1 + configs.splitmix32(ids, 15) % 3).astype(np.uint8)
    return sc


def test_d1_policy_sweep_parity(engine):
    spec = configs.config2_world(n_steps=720)
    n = 2500
    sc = _sweep_scenarios(n, 99)
    load = po.gen_load(configs.trace_gen(3), spec.n_steps, 1, n, first_id=99)
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    assert engine.last_engine()[0] == 2
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    assert rc["deletions"].sum() > 0 and len(set(rc["last_choice"] & 0xFFF)) > 3
    compare(rg, rc, tg, tc)


@pytest.mark.parametrize("variant", ["slots16", "delay0", "tol0", "big_load", "neg_load",
                                     "no_limit_cpu", "behavior", "budget50", "one_pool",
                                     "pdb100", "pdb0", "long_ca", "up_stab", "rules_reordered",
                                     "min0", "t1", "heavy_delay0"])
def test_d1_edge_cases(engine, variant):
    spec = configs.config2_world(n_steps=480)
    n = 700
    sc = configs.hpa_scenarios(n, 5)
    load = po.gen_load(configs.trace_gen(8), spec.n_steps, 1, n, first_id=5)
    if variant == "slots16":
        spec.max_nodes = 16
        load = load * 6
    elif variant == "delay0":
        spec.provision_delay_steps = 0
    elif variant == "tol0":
        spec.deploys = [deployment(abi.SCALER_HPA, tol=0.0)]
    elif variant == "big_load":  # usage*100 beyond 32 bits: int64 utilisation path
        load[::7] = np.int32(2_000_000_000)
    elif variant == "neg_load":
        load[::5] = -load[::5]
    elif variant == "no_limit_cpu":
        spec.deploys = [deployment(abi.SCALER_HPA, limit_cpu=0)]
    elif variant == "behavior":
        from ccka.world import hpa_rules
        up = hpa_rules(abi.SELECT_MIN, [(abi.HPA_PODS, 2, 120), (abi.HPA_PERCENT, 50, 240)], 120)
        dn = hpa_rules(abi.SELECT_MAX, [(abi.HPA_PODS, 1, 180), (abi.HPA_PERCENT, 30, 60)], 240)
        spec.deploys = [deployment(abi.SCALER_HPA, up=up, down=dn, min_r=2, max_r=60)]
    elif variant == "budget50":
        spec.max_nodes = 16
        for p in spec.pools:
            p.budget_pct = 50
        load = load * 5
    elif variant == "one_pool":
        spec.pools = spec.pools[1:]
    elif variant == "pdb100":  # no voluntary eviction ever allowed: empty nodes only
        spec.pdb_pct = 100
        load = load * 4
    elif variant == "pdb0":
        spec.pdb_pct = 0
        load = load * 4
    elif variant == "long_ca":  # consolidateAfter beyond the 16-bit per-slot field (clamped)
        for p in spec.pools:
            p.profile[abi.PROFILE_OFFPEAK].consolidate_after_s = 5_000_000
        sc.reset_ca_s = np.full(n, 30000, np.int16)
    elif variant in ("up_stab", "rules_reordered"):  # the generic-behaviour instantiation
        from ccka.world import default_down, hpa_rules
        pol = [(abi.HPA_PERCENT, 100, 15), (abi.HPA_PODS, 4, 15)]
        up = hpa_rules(abi.SELECT_MAX, pol, 120) if variant == "up_stab" else \
            hpa_rules(abi.SELECT_MAX, pol[::-1], 0)
        spec.deploys = [deployment(abi.SCALER_HPA, up=up, down=default_down(300))]
    elif variant == "min0":
        spec.deploys = [deployment(abi.SCALER_HPA, min_r=0, replicas0=0)]
        load[(np.arange(spec.n_steps) // 37) % 3 == 0] = 0
    elif variant == "t1":
        spec.n_steps = 1
        load = np.ascontiguousarray(load[:1])
    elif variant == "heavy_delay0":  # saturated nodes and zero-delay launches together
        spec.provision_delay_steps = 0
        load = load * 7
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    assert engine.last_engine()[0] == 2, variant
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    compare(rg, rc, tg, tc)


def test_d1_trace_layouts(engine):
    """The single-deployment kernel reads its wave-tiled trace copy
    ([wave][T][lanes], built by the first rollout of a trace); the [T][N] trace
    (ccka_debug_trace_flat) and a re-tiling after the lanes-per-wave value
    changes under a resident trace give the same bit-exact results and
    trajectories as the oracle."""
    import ctypes as C

    spec = configs.config2_world(n_steps=301)
    n = 3001
    sc = configs.hpa_scenarios(n, 5)
    load = po.gen_load(configs.trace_gen(9), spec.n_steps, 1, n, first_id=5)
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    fl = engine.lib.ccka_debug_trace_flat
    fl.argtypes = [C.c_void_p, C.c_int32]
    lp = engine.lib.ccka_debug_lpw
    lp.argtypes = [C.c_void_p, C.c_int32]
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    assert engine.last_engine()[0] == 2
    compare(rg, rc, tg, tc)
    try:
        assert fl(engine.ctx, 1) == 0
        engine.rollout(trajectory=True)
        compare(engine.results(), rc, engine.trajectory(), tc)
        assert fl(engine.ctx, 0) == 0
        assert lp(engine.ctx, 23) == 0  # the copy was tiled for the automatic value: re-tiled at the rollout
        engine.rollout(trajectory=True)
        compare(engine.results(), rc, engine.trajectory(), tc)
    finally:
        fl(engine.ctx, 0)
        lp(engine.ctx, 0)


@pytest.mark.parametrize("lpw,steps", [(1, 97), (7, 5), (17, 29), (33, 1440), (64, 300), (49, 61)])
def test_d1_lane_skew_schedule(engine, lpw, steps):
    """The lane-skewed schedule of rollout_d1_kernel (quiet steps per lane,
    batched event steps, LDS-DMA trace ring, scenario-major records): any
    scenarios per wave (one lane to a full wave, partial last waves) and
    horizons shorter than the ring prologue, not a multiple of the quiet
    steps per iteration, or the full day, bit-exact against the oracle."""
    import ctypes as C

    spec = configs.config2_world(n_steps=steps)
    n = 997
    sc = configs.hpa_scenarios(n, 11)
    load = po.gen_load(configs.trace_gen(3), spec.n_steps, 1, n, first_id=11)
    engine.lib.ccka_debug_lpw.argtypes = [C.c_void_p, C.c_int32]
    assert engine.lib.ccka_debug_lpw(engine.ctx, lpw) == 0
    try:
        rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    finally:
        engine.lib.ccka_debug_lpw(engine.ctx, 0)
    assert engine.last_engine()[0] == 2
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    compare(rg, rc, tg, tc)


@pytest.mark.parametrize("variant", ["start_37", "peak_odd_wrap", "peak_empty", "no_switch"])
def test_d1_boundaries_off_the_hour(engine, variant):
    """Hour and peak-window boundaries that do not coincide (the next-event
    step of a lane is the minimum of both), a wrapped window, an empty one."""
    spec = configs.config2_world(n_steps=700)
    n = 600
    sc = configs.hpa_scenarios(n, 3)
    load = po.gen_load(configs.trace_gen(5), spec.n_steps, 1, n, first_id=3)
    if variant == "start_37":
        spec.start_minute = 37
        spec.peak_start, spec.peak_end = 300, 420
    elif variant == "peak_odd_wrap":
        spec.start_minute = 1200
        spec.peak_start, spec.peak_end = 1301, 97
    elif variant == "peak_empty":
        spec.peak_start = spec.peak_end = 611
    elif variant == "no_switch":
        spec.peak_switch = 0
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    assert engine.last_engine()[0] == 2, variant
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    assert (tc["flags"] & 1).any() == (variant != "peak_empty" and variant != "no_switch")
    compare(rg, rc, tg, tc)


def test_d1_matches_general_kernel(engine):
    spec = configs.config3_world(n_steps=360)
    n = 1500
    sc = configs.hpa_scenarios(n, 0, 8, 190, configs.CONFIG3_CARBON)
    load = po.gen_load(configs.trace_gen(), spec.n_steps, 1, n)
    r2, t2 = run_engine(engine, spec, sc, load=load, traj=True)
    assert engine.last_engine()[0] == 2
    engine.set_engine(1)
    try:
        engine.rollout(trajectory=True)
        assert engine.last_engine()[0] == 1
        r1, t1 = engine.results(), engine.trajectory()
    finally:
        engine.set_engine(0)
    compare(r2, r1, t2, t1)


def test_d1_replacement_large_catalog(engine):
    """Replacement consolidation on the 800-type, 8-region catalog with
    carbon weights: the single-deployment kernel's price-only offer table
    (multi-chunk prefix scan) against the general kernel's per-lane offer
    search and the oracle, bit for bit."""
    spec = configs.config3_world(n_steps=720)
    spec.replace = 1
    spec.pdb_pct = -1
    spec.deploys[0].cap_sel = abi.CAP_OD
    spec.pools[0].profile[abi.PROFILE_OFFPEAK].policy = abi.WHEN_EMPTY_OR_UNDERUTILIZED
    n = 1200
    sc = configs.hpa_scenarios(n, 0, 8, 150, configs.CONFIG3_CARBON)
    load = po.gen_load(configs.trace_gen(6), spec.n_steps, 1, n)
    r2, t2 = run_engine(engine, spec, sc, load=load, traj=True)
    assert engine.last_engine()[0] == 2
    engine.set_engine(1)
    try:
        engine.rollout(trajectory=True)
        assert engine.last_engine()[0] == 1
        r1, t1 = engine.results(), engine.trajectory()
    finally:
        engine.set_engine(0)
    compare(r2, r1, t2, t1)
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    assert ((tc["flags"] & 32) != 0).any()  # replacements happened
    compare(r2, rc, t2, tc)


@pytest.mark.parametrize("variant", ["drift", "drift_pdb_budget", "drift_delay0_bdef"])
def test_d1_drift_matches_general_kernel(engine, variant):
    """The single-deployment kernel's drift (pre-spun replacements, takeovers,
    taint) against the general kernel on the same inputs, bit for bit."""
    spec = configs.config2_world(n_steps=1440)
    spec.drift = 1
    n = 2222
    sc = configs.hpa_scenarios(n, first_id=7)
    if variant == "drift_pdb_budget":
        spec.pdb_pct = 80
        for p in spec.pools:
            p.budget_pct = 40
    elif variant == "drift_delay0_bdef":
        spec.provision_delay_steps = 0
        spec.pdb_pct = -1
        sc.down_stab_s = np.full(n, 120, np.int16)
    load = po.gen_load(configs.trace_gen(2), spec.n_steps, 1, n, first_id=7)
    r2, t2 = run_engine(engine, spec, sc, load=load, traj=True)
    assert engine.last_engine()[0] == 2
    engine.set_engine(1)
    try:
        engine.rollout(trajectory=True)
        assert engine.last_engine()[0] == 1
        r1, t1 = engine.results(), engine.trajectory()
    finally:
        engine.set_engine(0)
    assert ((t1["flags"] & 48) == 48).any() and ((t1["flags"] & 20) == 20).any()
    compare(r2, r1, t2, t1)


# ---------------------------------------------------------------------------
# Karpenter drift on the peak/off-peak zone switch (SEMANTICS 3.G0)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("variant", ["pdb50", "no_pdb", "budget50", "wrap_peak", "pool_limit", "delay0",
                                     "delay3", "one_slot", "slots16"])
def test_drift_parity_single_deployment(engine, variant):
    spec = configs.config2_world(n_steps=1440)
    spec.drift = 1
    n = 1537
    sc = configs.hpa_scenarios(n, first_id=901)
    if variant == "no_pdb":
        spec.pdb_pct = -1
    elif variant == "budget50":
        for p in spec.pools:
            p.budget_pct = 50
    elif variant == "wrap_peak":
        spec.peak_start, spec.peak_end, spec.start_minute = 1300, 200, 1200
        spec.pdb_pct = -1
    elif variant == "pool_limit":
        for p in spec.pools:
            p.limit_cpu_m = 12000
    elif variant in ("delay0", "delay3"):
        spec.provision_delay_steps = int(variant[-1])
        spec.pdb_pct = -1
    elif variant == "one_slot":
        spec.max_nodes = 1
        spec.pdb_pct = -1
    elif variant == "slots16":
        spec.max_nodes = 16
        spec.pdb_pct = -1
    load = po.gen_load(configs.trace_gen(3), spec.n_steps, 1, n, first_id=sc.first_id)
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    # drift runs inside the single-deployment kernel (8 slots, no pool limits),
    # otherwise on the general kernel
    assert engine.last_engine()[0] == (1 if variant in ("pool_limit", "slots16") else 2), variant
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    f = tc["flags"]
    # both drift branches are covered: a pre-spun replacement (flags 16|32) where
    # a slot is free, and the eviction fallback (flags 16|4)
    if variant != "one_slot":
        assert ((f & 48) == 48).any()
    else:
        assert not ((f & 48) == 48).any()
    assert ((f & 20) == 20).any()
    compare(rg, rc, tg, tc)


def test_drift_parity_multi_deployment(engine):
    spec = configs.config2_world(max_nodes=12)
    spec.drift = 1
    spec.pdb_pct = -1
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
    assert ((tc["flags"] & 48) == 48).any() and ((tc["flags"] & 20) == 20).any()
    compare(rg, rc, tg, tc)


# ---------------------------------------------------------------------------
# multi-trigger KEDA ScaledObjects (SEMANTICS 3.C)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("drift", [0, 1])
def test_keda_multi_trigger_parity(engine, drift):
    """HPA on spot + a 3-trigger KEDA worker (own column + 2 KEDA_TRIGGER
    columns with their own thresholds / activations) + a 2-trigger KEDA worker."""
    from ccka.world import keda_trigger
    spec = configs.config2_world(max_nodes=12)
    spec.drift = drift
    spec.deploys = [
        deployment(abi.SCALER_HPA, cap_sel=abi.CAP_SPOT),
        deployment(abi.SCALER_KEDA, replicas0=0, keda_threshold=900, keda_activation=2500,
                   keda_cooldown=240, cap_sel=abi.CAP_SPOT | abi.CAP_OD, keda_max=40),
        keda_trigger(1200, 3000),
        keda_trigger(2500, 6000),
        deployment(abi.SCALER_KEDA, replicas0=1, keda_threshold=1500, keda_activation=1000,
                   keda_cooldown=300, keda_min=1, keda_max=20, req_cpu=300, cap_sel=abi.CAP_OD),
        keda_trigger(700, 4000),
    ]
    n = 600
    sc = ScenarioSet(n)
    load = po.gen_load(configs.trace_gen(13), spec.n_steps, len(spec.deploys), n)
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    compare(rg, rc, tg, tc)


def test_keda_trigger_validation(engine):
    from ccka.world import keda_trigger
    spec = configs.config2_world(n_steps=60)
    spec.deploys = [deployment(abi.SCALER_HPA), keda_trigger(500)]  # trigger after an HPA
    with pytest.raises(abi.CckaError):
        engine.set_world(spec)


# ---------------------------------------------------------------------------
# single-node replacement consolidation (SEMANTICS 3.G2)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("variant", ["spot_pool_only", "od_pool_weou", "drift_replace", "pdb50", "delay0",
                                     "pool_limit", "one_pool_budget50"])
def test_replacement_parity_single_deployment(engine, variant):
    spec = configs.config2_world(n_steps=1440)
    spec.replace = 1
    spec.pdb_pct = -1
    spec.deploys[0].cap_sel = abi.CAP_OD  # on-demand nodes in a WhenEmptyOrUnderutilized pool
    n = 1537
    sc = configs.hpa_scenarios(n, first_id=901)
    if variant == "spot_pool_only":
        spec.pools = [spec.pools[1]]
    else:
        spec.pools[0].profile[abi.PROFILE_OFFPEAK].policy = abi.WHEN_EMPTY_OR_UNDERUTILIZED
    if variant == "drift_replace":
        spec.drift = 1
    elif variant == "pdb50":
        spec.pdb_pct = 50
    elif variant == "delay0":
        spec.provision_delay_steps = 0
    elif variant == "pool_limit":
        for p in spec.pools:
            p.limit_cpu_m = 12000
    elif variant == "one_pool_budget50":  # the on-demand pool alone, half its nodes per step
        spec.pools = [spec.pools[0]]
        spec.pools[0].budget_pct = 50
        spec.drift = 1
    load = po.gen_load(configs.trace_gen(3), spec.n_steps, 1, n, first_id=sc.first_id)
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    # replacement runs inside the single-deployment kernel (8 slots, <= 2 pools,
    # no pool limits); pool limits take the general kernel
    assert engine.last_engine()[0] == (1 if variant == "pool_limit" else 2), variant
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    if variant != "pdb50":
        assert ((tc["flags"] & 32) != 0).any()  # replacements happened
    compare(rg, rc, tg, tc)


@pytest.mark.parametrize("lpw,steps,max_nodes,start", [(5, 300, 8, 0), (64, 1440, 8, 37), (23, 700, 3, 11),
                                                     (40, 900, 2, 0)])
def test_d1_replacement_schedule(engine, lpw, steps, max_nodes, start):
    """Replacement consolidation (+ drift) inside the single-deployment kernel
    under the lane-skewed schedule: offers re-evaluated only at event steps
    (hour boundaries off the clock hour, readiness, scheduling), few or no
    free slots for the replacement, bit-exact against the oracle."""
    import ctypes as C

    spec = configs.config2_world(n_steps=steps, max_nodes=max_nodes)
    spec.replace = 1
    spec.drift = 1
    spec.pdb_pct = -1
    spec.start_minute = start
    spec.deploys[0].cap_sel = abi.CAP_OD
    spec.pools[0].profile[abi.PROFILE_OFFPEAK].policy = abi.WHEN_EMPTY_OR_UNDERUTILIZED
    n = 1100
    sc = configs.hpa_scenarios(n, first_id=77)
    load = po.gen_load(configs.trace_gen(4), spec.n_steps, 1, n, first_id=sc.first_id)
    engine.lib.ccka_debug_lpw.argtypes = [C.c_void_p, C.c_int32]
    assert engine.lib.ccka_debug_lpw(engine.ctx, lpw) == 0
    try:
        rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    finally:
        engine.lib.ccka_debug_lpw(engine.ctx, 0)
    assert engine.last_engine()[0] == 2
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    if max_nodes > 2:
        assert ((tc["flags"] & 32) != 0).any()  # replacements happened
    compare(rg, rc, tg, tc)


def test_replacement_parity_multi_deployment(engine):
    spec = configs.config2_world(max_nodes=12)
    spec.replace = 1
    spec.drift = 1
    spec.pdb_pct = -1
    spec.pools[0].profile[abi.PROFILE_OFFPEAK].policy = abi.WHEN_EMPTY_OR_UNDERUTILIZED
    spec.deploys = [
        deployment(abi.SCALER_HPA, cap_sel=abi.CAP_OD),
        deployment(abi.SCALER_HPA, req_cpu=500, req_mem=512, limit_cpu=1000, cap_sel=abi.CAP_OD, target=60),
        deployment(abi.SCALER_KEDA, replicas0=0, keda_threshold=800, keda_activation=1500,
                   keda_cooldown=300, cap_sel=abi.CAP_SPOT | abi.CAP_OD),
    ]
    n = 700
    sc = ScenarioSet(n)
    load = po.gen_load(configs.trace_gen(9), spec.n_steps, 3, n)
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    assert ((tc["flags"] & 32) != 0).any()
    compare(rg, rc, tg, tc)


def test_inert_disruption_runs_on_d1(engine):
    """Worlds that enable drift / replacement run on the single-deployment
    kernel within its 8 slots and 2 pools (inert or not) and match the oracle
    (which runs the phases); beyond them they run on the general kernel."""
    spec = configs.config2_world(n_steps=1440)
    spec.replace = 1
    sc = configs.hpa_scenarios(1200)
    load = po.gen_load(configs.trace_gen(), spec.n_steps, 1, sc.n)
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    assert engine.last_engine()[0] == 2  # half the scenarios select on-demand: replacement can act
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    compare(rg, rc, tg, tc)
    sc.cap_sel = np.full(sc.n, abi.CAP_SPOT, np.uint8)  # spot-only: no on-demand node can exist
    load = po.gen_load(configs.trace_gen(), spec.n_steps, 1, sc.n)
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    assert engine.last_engine()[0] == 2
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    compare(rg, rc, tg, tc)
    spec.drift = 1  # zones move at the switch: drift acts, inside the single-deployment kernel
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    assert engine.last_engine()[0] == 2
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    assert (tc["flags"] & 16).any()
    compare(rg, rc, tg, tc)
    spec.max_nodes = 12  # beyond its 8 slots: the general kernel
    run_engine(engine, spec, sc, load=po.gen_load(configs.trace_gen(), spec.n_steps, 1, sc.n))
    assert engine.last_engine()[0] == 1
    spec.max_nodes = 8
    sc.peak_switch = np.zeros(sc.n, np.uint8)  # no scenario switches: drift is inert
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    assert engine.last_engine()[0] == 2
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    compare(rg, rc, tg, tc)
