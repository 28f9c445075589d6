"""The C oracle against an independent pure-Python restatement of
docs/SEMANTICS.md (tests/spec_model.py) on random small worlds (hypothesis):
every result field and every trajectory record equal, fp64 included.

The two were written separately from the same normative text; a misreading
of phase order, PDB or budget interplay, the consolidation candidate order,
the claim packing or the HPA behavior shows up here as a mismatch (SURVEY.md
§4 test plan 3, §8(c)). Worlds: 1-5 instance types, 1-2 regions, 1-3 zones,
1-2 NodePools with random profile patches, disruption budgets and CPU /
memory limits, 1-2 deployments (HPA with random behavior rules, one-trigger
KEDA, static), 1-4 node slots, 20-120 steps, HPA sync 60/30/15 s, drift and
replacement consolidation on or off, per-scenario overrides."""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import pyoracle as po
import spec_model as sm
from ccka import abi
from ccka.world import Catalog, ScenarioSet, WorldSpec, deployment, hpa_rules

FIELDS = ["cost_uphmin", "energy_wmin", "gco2", "slo_minutes", "pending_pod_minutes", "node_min_spot",
          "node_min_od", "launches", "deletions", "peak_nodes", "final_replicas", "final_nodes",
          "last_choice", "choice_hash"]


def _patch(draw, Z, base):
    x = abi.PoolPatch()
    x.policy = draw(st.sampled_from([1, 2] if base else [0, 1, 2]))
    x.consolidate_after_s = draw(st.sampled_from([0, 30, 60, 120, 300] if base else [-1, 0, 30, 60, 120, 300]))
    zm = draw(st.integers(1 if base else 0, (1 << Z) - 1))
    x.zone_mask = zm
    x.cap_mask = draw(st.integers(1 if base else 0, 3))
    return x


def _rules(draw, up):
    choice = draw(st.integers(0, 3))
    if choice == 0:  # the autoscaling/v2 defaults
        return (hpa_rules(abi.SELECT_MAX, [(abi.HPA_PERCENT, 100, 15), (abi.HPA_PODS, 4, 15)], 0) if up else
                hpa_rules(abi.SELECT_MAX, [(abi.HPA_PERCENT, 100, 15)], draw(st.sampled_from([0, 60, 300]))))
    sel = draw(st.sampled_from([abi.SELECT_MAX, abi.SELECT_MIN, abi.SELECT_DISABLED]))
    n = draw(st.integers(1, 3))
    pols = [(draw(st.sampled_from([abi.HPA_PODS, abi.HPA_PERCENT])), draw(st.integers(1, 150)),
             draw(st.sampled_from([15, 30, 60, 120, 240, 420]))) for _ in range(n)]
    return hpa_rules(sel, pols, draw(st.sampled_from([0, 45, 60, 120, 300, 450])))


@st.composite
def worlds(draw):
    K = draw(st.integers(1, 5))
    R = draw(st.integers(1, 2))
    Z = draw(st.integers(1, 3))
    vcpu = np.array([draw(st.sampled_from([1, 2, 4, 8])) for _ in range(K)], np.int32)
    mem = np.array([float(v * draw(st.sampled_from([2, 4, 8]))) for v in vcpu])
    pods = np.array([draw(st.sampled_from([4, 8, 17, 29, 58])) for _ in range(K)], np.int32)
    od = np.array([draw(st.integers(20000, 400000)) for _ in range(K)], np.int64)
    names = ["m6i.large"] + [f"t{k}.x" for k in range(1, K)]
    cat = Catalog(names, vcpu, mem, pods, od)
    rng = np.random.default_rng(draw(st.integers(0, 2**31)))
    price = rng.integers(1000, 300000, size=(R, 24, K, Z, 2)).astype(np.int32)
    price[rng.random(price.shape) < draw(st.sampled_from([0.0, 0.2, 0.5]))] = 0  # offerings missing
    ci = rng.uniform(50.0, 700.0, size=(R, 24))
    pools = []
    for _ in range(draw(st.integers(1, 2))):
        p = abi.Pool()
        p.limit_cpu_m = draw(st.sampled_from([-1, -1, 4000, 12000]))
        p.limit_mem_mi = draw(st.sampled_from([-1, -1, 16384]))
        p.budget_pct = draw(st.sampled_from([0, 10, 34, 50, 100]))
        p.base = _patch(draw, Z, True)
        for prof in range(3):
            p.profile[prof] = _patch(draw, Z, False)
        pools.append(p)
    deps = []
    for _ in range(draw(st.integers(1, 2))):
        kind = draw(st.sampled_from([abi.SCALER_HPA, abi.SCALER_HPA, abi.SCALER_KEDA, abi.SCALER_STATIC]))
        d = deployment(kind, replicas0=draw(st.integers(0, 6)), min_r=draw(st.integers(0, 2)),
                       max_r=draw(st.integers(3, 14)), target=draw(st.integers(30, 95)),
                       req_cpu=draw(st.sampled_from([100, 200, 250, 500, 900])),
                       req_mem=draw(st.sampled_from([64, 128, 512, 2048])),
                       limit_cpu=draw(st.sampled_from([0, 500, 1000])), cap_sel=draw(st.integers(1, 3)),
                       pdb=draw(st.integers(0, 1)), keda_threshold=draw(st.sampled_from([300, 700, 2000])),
                       keda_activation=draw(st.sampled_from([0, 200, 1000])),
                       keda_cooldown=draw(st.sampled_from([0, 60, 300])), keda_min=draw(st.integers(0, 1)),
                       keda_max=draw(st.integers(2, 12)), tol=draw(st.sampled_from([0.1, 0.0, 0.25])),
                       up=_rules(draw, True), down=_rules(draw, False))
        deps.append(d)
    spec = WorldSpec(catalog=cat, ci=ci, price=price, pools=pools, deploys=deps,
                     n_steps=draw(st.integers(20, 120)), start_minute=draw(st.integers(0, 1439)),
                     provision_delay_steps=draw(st.integers(0, 2)), max_nodes=draw(st.integers(1, 4)),
                     base_nodes=draw(st.integers(0, 3)), base_util=draw(st.sampled_from([0.0, 0.25])),
                     slo_util_pct=draw(st.sampled_from([60, 100, 150])), pdb_pct=draw(st.sampled_from([-1, 0, 50, 100])),
                     peak_start=draw(st.integers(0, 1439)), peak_end=draw(st.integers(0, 1439)),
                     peak_switch=draw(st.integers(0, 1)), reset_ca_s=draw(st.sampled_from([0, 30, 90])),
                     carbon_weight=draw(st.sampled_from([0.0, 0.5, 2.0])), drift=draw(st.integers(0, 1)),
                     replace=draw(st.integers(0, 1)), hpa_sync_s=draw(st.sampled_from([0, 60, 30, 15])))
    n = 3
    kw = {}
    if draw(st.booleans()):
        kw["target_util_pct"] = np.array([draw(st.integers(30, 95)) for _ in range(n)], np.int16)
    if draw(st.booleans()):
        kw["max_replicas"] = np.array([draw(st.integers(2, 14)) for _ in range(n)], np.int16)
    if draw(st.booleans()):
        kw["cap_sel"] = np.array([draw(st.integers(1, 3)) for _ in range(n)], np.uint8)
    if draw(st.booleans()):
        kw["down_stab_s"] = np.array([draw(st.sampled_from([0, 60, 300, 450])) for _ in range(n)], np.int16)
    if draw(st.booleans()):
        kw["region"] = np.array([draw(st.integers(0, R - 1)) for _ in range(n)], np.uint8)
    if draw(st.booleans()):
        kw["carbon_weight"] = np.array([draw(st.sampled_from([0.0, 1.0, 3.0])) for _ in range(n)])
    if draw(st.booleans()):
        kw["reset_ca_s"] = np.array([draw(st.sampled_from([0, 60, 200])) for _ in range(n)], np.int16)
    if draw(st.booleans()):
        kw["peak_switch"] = np.array([draw(st.integers(0, 1)) for _ in range(n)], np.uint8)
    sc = ScenarioSet(n, draw(st.integers(0, 1000)), **kw)
    hi = draw(st.sampled_from([800, 3000, 9000]))
    load = rng.integers(0, hi, size=(spec.n_steps, len(deps), n)).astype(np.int32)
    return spec, sc, load


def compare_model(spec, sc, load):
    rc, tc = po.rollout(spec, sc, load, traj=True)
    rm, tm = sm.rollout(spec, sc, load)
    for f in FIELDS:
        got = np.asarray(rm[f]).astype(rc[f].dtype)
        assert np.array_equal(got, rc[f]), f"{f}: model {got} oracle {rc[f]}"
    names = tc.dtype.names
    for s in range(sc.n):
        for t in range(spec.n_steps):
            want = tuple(int(tc[t][s][x]) for x in names)
            assert tuple(tm[s][t]) == want, f"scenario {s} step {t}: model {tm[s][t]} oracle {want}"


@settings(max_examples=320, deadline=None, suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
@given(worlds())
def test_oracle_equals_independent_model(case):
    compare_model(*case)


def test_model_config2_reference_world():
    """The reference's own world (config 2 pools, patches and burst-shaped
    load) through both, 240 steps (peak window inside via start_minute)."""
    from ccka import configs
    spec = configs.config2_world(n_steps=240)
    spec.start_minute = 900
    sc = configs.hpa_scenarios(12)
    load = po.gen_load(configs.trace_gen(), spec.n_steps, 1, sc.n)
    compare_model(spec, sc, load)


def test_model_config1_burst_replay():
    """demo_30's 12 burst Deployments x 5 replicas (alternating spot / on-demand
    nodeSelectors) on the reference pools, a day of one-minute steps through
    the off-peak -> peak -> off-peak switch (config 1): both restatements agree
    on every record, claim packing across deployments included."""
    from ccka import configs
    spec = configs.config1_world()
    sc = ScenarioSet(1)
    load = np.zeros((spec.n_steps, 12, 1), np.int32) + 100
    compare_model(spec, sc, load)
