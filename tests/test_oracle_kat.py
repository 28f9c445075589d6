"""Known-answer tests pinning the CPU oracle (the GPU engine's checker).

HPA replica-calculator cases are restated from upstream Kubernetes'
pkg/controller/podautoscaler/replica_calculator_test.go (k8s 1.34 is the
version the reference deploys, .env:4); the upstream tree is not available
offline, so the cases are reproduced from its documented expectations and
re-derived by hand below. Behavior/KEDA/Karpenter cases are hand-computed
from docs/SEMANTICS.md. Philox vectors are the published Random123 KATs.
"""
import ctypes as C

import numpy as np
import pytest

import pyoracle as po
from ccka import abi, configs
from ccka.world import (ScenarioSet, WorldSpec, catalog_small, default_down, default_up,
                        deployment, hpa_rules, price_tiles, reference_pools)

L = po.lib()


def hpa(cur, ready, usages_m, req_m, target, tol=0.1):
    u = C.c_int32()
    p = L.ccka_oracle_hpa_resource_proposal(cur, ready, int(sum(usages_m)), req_m, target, tol, C.byref(u))
    return p, u.value


# ---------------------------------------------------------------- HPA calculator
def test_hpa_scale_up():  # upstream TestReplicaCalcScaleUp
    assert hpa(3, 3, [300, 500, 700], 1000, 30) == (5, 50)


def test_hpa_scale_down():  # upstream TestReplicaCalcScaleDown
    assert hpa(5, 5, [100, 300, 500, 250, 250], 1000, 50) == (3, 28)


def test_hpa_tolerance():  # upstream TestReplicaCalcToleranceCPU
    assert hpa(3, 3, [1010, 1030, 1020], 1000, 100) == (3, 102)


def test_hpa_unready_less_scale():  # upstream TestReplicaCalcScaleUpUnreadyLessScale
    # 3 pods, 1 unready; ready usage 500+700 of 2x1000 -> 60 %; unready counted at 0
    assert hpa(3, 2, [500, 700], 1000, 30) == (4, 60)


def test_hpa_unready_no_scale():  # upstream TestReplicaCalcScaleUpUnreadyNoScale
    assert hpa(3, 1, [400], 1000, 30) == (3, 40)


def test_hpa_tolerance_edges():
    # ratio exactly 1.1 and 0.9 are inside the (inclusive) band
    assert hpa(4, 4, [4 * 110], 100, 100)[0] == 4
    assert hpa(4, 4, [4 * 90], 100, 100)[0] == 4
    assert hpa(4, 4, [4 * 111], 100, 100)[0] == 5   # ceil(1.11*4)=ceil(4.44)
    assert hpa(10, 10, [10 * 89], 100, 100)[0] == 9  # ceil(8.9)


def test_hpa_no_ready_pods():
    assert hpa(5, 0, [0], 200, 70) == (5, -1)


def test_keda_proposal():
    assert L.ccka_oracle_keda_proposal(2, 1000, 500, 0.1) == 2   # r = 1.0
    assert L.ccka_oracle_keda_proposal(2, 1500, 500, 0.1) == 3
    assert L.ccka_oracle_keda_proposal(4, 1000, 500, 0.1) == 2
    assert L.ccka_oracle_keda_proposal(2, 1050, 500, 0.1) == 2   # within 10 %


# ---------------------------------------------------------------- HPA behavior
def behavior(cur, prop, mn, mx, up, down, recs=(), valid=(), deltas=()):
    r = (C.c_int32 * 8)(*([*recs] + [0] * (8 - len(recs))))
    v = (C.c_uint8 * 8)(*([*valid] + [0] * (8 - len(valid))))
    d = (C.c_int32 * 8)(*([*deltas] + [0] * (8 - len(deltas))))
    return L.ccka_oracle_hpa_behavior(cur, prop, mn, mx, C.byref(up), C.byref(down), r, v, d)


def test_behavior_down_stabilisation():
    # recs of the last 4 steps are inside the 300 s window: highest (12) caps the drop
    assert behavior(10, 5, 1, 100, default_up(), default_down(300), [10, 8, 12, 6], [1, 1, 1, 1]) == 10
    # outside the window (k=4 is 300 s old: not strictly newer) only k<4 count
    assert behavior(10, 5, 1, 100, default_up(), default_down(300), [6, 6, 6, 6, 20], [1] * 5) == 6
    assert behavior(10, 5, 1, 100, default_up(), default_down(0), [10, 8, 12], [1, 1, 1]) == 5


def test_behavior_up_rate_limit():
    # default up: max(+4 pods, +100 %) per 15 s
    assert behavior(3, 20, 1, 100, default_up(), default_down()) == 7
    assert behavior(10, 50, 1, 100, default_up(), default_down()) == 20
    mn = hpa_rules(abi.SELECT_MIN, [(abi.HPA_PERCENT, 100, 15), (abi.HPA_PODS, 4, 15)], 0)
    assert behavior(10, 50, 1, 100, mn, default_down()) == 14
    assert behavior(3, 20, 1, 5, default_up(), default_down()) == 5  # maxReplicas


def test_behavior_period_history():
    # Pods policy +2 per 180 s; +3 scaled 60 s ago counts (periodStart = cur-3)
    up = hpa_rules(abi.SELECT_MAX, [(abi.HPA_PODS, 2, 180)], 0)
    assert behavior(8, 20, 1, 100, up, default_down(), deltas=[3]) == 8   # limit 7 < cur -> cur
    assert behavior(8, 20, 1, 100, up, default_down(), deltas=[0, 0, 3]) == 10  # 180 s old: out
    dn = hpa_rules(abi.SELECT_MAX, [(abi.HPA_PODS, 2, 120)], 0)
    assert behavior(10, 1, 1, 100, default_up(), dn, deltas=[-1]) == 9   # ps=11 -> 9
    dis = hpa_rules(abi.SELECT_DISABLED, [], 0)
    assert behavior(10, 1, 1, 100, default_up(), dis) == 10


# ---------------------------------------------------------------- Philox KATs
@pytest.mark.parametrize("ctr,key,want", [
    ([0, 0, 0, 0], [0, 0], [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
    ([0xffffffff] * 4, [0xffffffff] * 2, [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
    ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
     [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]),
])
def test_philox_random123_kat(ctr, key, want):
    out = (C.c_uint32 * 4)()
    L.ccka_oracle_philox(*ctr, *key, out)
    assert list(out) == want


def test_trace_generator_properties():
    g = configs.trace_gen()
    a = po.gen_load(g, 1440, 1, 500)
    assert a.min() >= 0 and a.dtype == np.int32
    # shard invariance: ids 200..499 generated alone equal the slice
    b = po.gen_load(g, 1440, 1, 300, first_id=200)
    assert np.array_equal(a[:, :, 200:], b)
    # diurnal + burst shape: per-scenario max/mean within the configured envelope
    assert (a.max(axis=0) <= 3 * 5000 * 1.8 * 1.3).all()


# ---------------------------------------------------------------- full rollouts
def tiny_world(deploys, T=120, **kw):
    cat = catalog_small()
    price = price_tiles(cat, 1, 3)
    return WorldSpec(catalog=cat, ci=np.full((1, 24), 400.0), price=price, pools=reference_pools(),
                     deploys=deploys, n_steps=T, **kw)


def run(spec, load, n=1, **sc):
    scen = ScenarioSet(n, **sc)
    return po.rollout(spec, scen, load, traj=True)


def test_static_deployment_single_launch_and_cost():
    """5 static pods (1 vCPU) on the spot pool: one launch at t=0 of the cheapest
    feasible spot offering in us-east-2a, ready at t=1; cost = base + node price
    every step."""
    spec = tiny_world([deployment(abi.SCALER_STATIC, replicas0=5, min_r=5, max_r=5)], T=60,
                      peak_switch=0)
    load = np.full((60, 1, 1), 500, np.int32)
    r, tr = run(spec, load)
    assert r["launches"][0] == 1 and r["deletions"][0] == 0
    k = r["last_choice"][0] & 0xFFF
    z = (r["last_choice"][0] >> 12) & 3
    c = (r["last_choice"][0] >> 14) & 3
    pool = r["last_choice"][0] >> 16
    assert (z, c, pool) == (0, 0, 1)  # zone a (off-peak), spot, spot-preferred
    # argmin over spot types in zone 0 that fit 5 x 200m pods (all do)
    spot = spec.price[0, 0, :, 0, 0]
    assert k == int(np.argmin(spot))
    base = 3 * spec.price[0, 0, spec.catalog.index("m6i.large"), 0, 1]
    assert r["cost_uphmin"][0] == 60 * (base + spot[k])
    assert tr["pending"][0, 0] == 5 and (tr["pending"][1:, 0] == 0).all()


def test_argmin_tie_break_lowest_index():
    spec = tiny_world([deployment(abi.SCALER_STATIC, replicas0=2, min_r=2, max_r=2)], T=3,
                      peak_switch=0)
    spec.price[:] = 100000
    load = np.zeros((3, 1, 1), np.int32)
    r, _ = run(spec, load)
    assert r["last_choice"][0] == (0 | 0 << 12 | 0 << 14 | 1 << 16)


def test_spot_first_even_if_od_cheaper():
    spec = tiny_world([deployment(abi.SCALER_STATIC, replicas0=2, min_r=2, max_r=2,
                                  cap_sel=abi.CAP_SPOT | abi.CAP_OD)], T=3, peak_switch=0)
    # no selector: pods are compatible with on-demand-slo first (name order) -> OD pool
    r, _ = run(spec, np.zeros((3, 1, 1), np.int32))
    assert r["last_choice"][0] >> 16 == 0 and ((r["last_choice"][0] >> 14) & 3) == 1
    # spot-only pool order: make the spot pool the only one
    spec.pools = [reference_pools()[1]]
    spec.price[..., 1] = 1          # on-demand absurdly cheap
    r, _ = run(spec, np.zeros((3, 1, 1), np.int32))
    assert ((r["last_choice"][0] >> 14) & 3) == 0  # still spot


def test_claim_skips_a_pool_its_limits_exhaust():
    """SEMANTICS 3.F: new claims go to the first pool (Karpenter order) that
    admits the pods' capacity types AND can hold one of them under its limits
    (found by the independent restatement, tests/spec_model.py: Karpenter then
    tries the next NodePool). on-demand-slo comes first for selector-less pods;
    with its CPU limit at 0 every claim lands in spot-preferred instead."""
    dep = [deployment(abi.SCALER_STATIC, replicas0=4, min_r=4, max_r=4, cap_sel=abi.CAP_SPOT | abi.CAP_OD)]
    spec = tiny_world(dep, T=3, peak_switch=0)
    r, _ = run(spec, np.zeros((3, 1, 1), np.int32))
    assert r["last_choice"][0] >> 16 == 0  # unlimited: the on-demand pool
    spec.pools[0].limit_cpu_m = 0
    r, tr = run(spec, np.zeros((3, 1, 1), np.int32))
    assert r["launches"][0] >= 1 and r["last_choice"][0] >> 16 == 1  # the spot pool
    assert tr["pending"][1, 0] == 0


def test_keda_scale_to_zero_and_when_empty_timing():
    """KEDA: active for 10 steps then idle. Scale 1->0 after the 300 s cooldown
    (5 steps after the last active step), node then empty; WhenEmpty/30 s in
    RESET... the OFFPEAK spot pool is WhenEmptyOrUnderutilized with inherited
    30 s -> the empty node is deleted one step after it empties."""
    d = deployment(abi.SCALER_KEDA, replicas0=0, keda_threshold=1000, keda_activation=0,
                   keda_cooldown=300, keda_min=0, keda_max=10)
    spec = tiny_world([d], T=40, peak_switch=0)
    load = np.zeros((40, 1, 1), np.int32)
    load[:10] = 1500
    r, tr = run(spec, load)
    reps = tr["replicas"][:, 0]
    assert reps[0] == 1                 # activation 0 -> 1
    assert reps[1] == 2                 # ceil(1500/1000)
    last_active = 9
    assert reps[last_active + 4] > 0 and reps[last_active + 5] == 0   # 60*(t-9) >= 300
    n_nodes = tr["nodes_spot"][:, 0].astype(int) + tr["nodes_od"][:, 0]
    t0 = last_active + 5
    # pods removed at t0 (last_event = t0); 60*(t - t0) >= 30 first at t0+1
    assert n_nodes[t0] == 1 and n_nodes[t0 + 1] == 0
    assert r["deletions"][0] == 1


def test_peak_flag_window():
    spec = tiny_world([deployment(abi.SCALER_STATIC, replicas0=1, min_r=1, max_r=1)], T=1440)
    r, tr = run(spec, np.zeros((1440, 1, 1), np.int32))
    peak = (tr["flags"][:, 0] & 1) == 1
    assert peak.sum() == 300 and peak[960:1260].all()


def test_underutilized_consolidation_and_pdb():
    """Hour 0 offers only 2-vCPU spot types: 3 x 500m KEDA pods fill node A.
    From minute 60 only 8-vCPU spot types exist and the 4th pod lands on a new
    node B. At t=61 (B ready): B (1 pod) cannot move to the full A -> rejected;
    A (3 pods) fits on B -> deleted under WhenEmptyOrUnderutilized, unless a
    100 % minAvailable PDB forbids the evictions."""
    d = deployment(abi.SCALER_KEDA, replicas0=3, req_cpu=500, keda_threshold=1000,
                   keda_activation=0, keda_min=0, keda_max=10)
    for pdb, want in ((-1, 1), (100, 0)):
        spec = tiny_world([d], T=90, peak_switch=0, pdb_pct=pdb)
        v = spec.catalog.vcpu
        spec.price[0, 0, :, :, 0] = np.where(v[:, None] == 2, spec.price[0, 0, :, :, 0], 0)
        spec.price[0, 1:, :, :, 0] = np.where(v[None, :, None] == 8, spec.price[0, 1:, :, :, 0], 0)
        load = np.full((90, 1, 1), 3000, np.int32)
        load[60:] = 4000
        r, tr = run(spec, load)
        assert r["launches"][0] == 2
        assert r["deletions"][0] == want
        n = tr["nodes_spot"][:, 0]
        assert n[59] == 1 and n[60] == 2
        assert n[61] == (1 if want else 2)


def test_oracle_deterministic_and_thread_invariant():
    spec = configs.config2_world(n_steps=300)
    sc = configs.hpa_scenarios(400)
    load = po.gen_load(configs.trace_gen(), 300, 1, 400)
    a, ta = po.rollout(spec, sc, load, traj=True, threads=1)
    b, tb = po.rollout(spec, sc, load, traj=True, threads=7)
    for k in a:
        assert np.array_equal(a[k], b[k]), k
    assert np.array_equal(ta, tb)


# ---------------------------------------------------------------- energy (SEMANTICS §3.H)
def test_energy_integer_nanowatt_minutes():
    """One scenario, constant load, no scaling: the step energy is exactly
    base + idle + dyn_per_m * min(pods * upp, alloc) in nW (hand-derived)."""
    spec = configs.config2_world(n_steps=3)
    spec.deploys = [deployment(abi.SCALER_STATIC, replicas0=2, min_r=2, max_r=2, limit_cpu=0)]
    spec.peak_switch = 0
    spec.provision_delay_steps = 0
    sc = ScenarioSet(1)
    load = np.full((3, 1, 1), 301, np.int32)
    res, tr = po.rollout(spec, sc, load, traj=True)
    types = spec.catalog.itypes()
    bt = types[spec.catalog.index("m6i.large")]
    base = spec.base_nodes * (bt.idle_nw + bt.dyn_nw_per_m * int(spec.base_util * bt.alloc_cpu_m))
    k = res["last_choice"][0] & 0xFFF
    ty = types[int(k)]
    upp = 301 // 2
    step = base + ty.idle_nw + ty.dyn_nw_per_m * min(2 * upp, ty.alloc_cpu_m)
    assert res["energy_wmin"][0] == float(3 * step) * 1e-9
    ci = spec.ci[0, 0] / 60000.0
    assert res["gco2"][0] == float(3 * step) * (ci * 1e-9)


def test_shared_traces_equal_expanded_traces():
    """n_traces > 0 reads trace (first_id + i) % n_traces: identical to giving
    every scenario a copy of its trace."""
    spec = configs.config2_world(n_steps=120)
    sc = configs.config4_scenarios(3, 4, 16)
    shared = po.gen_load(configs.config4_trace_gen(), 120, 1, 16)
    r1, _ = po.rollout(spec, sc, shared, threads=4)
    sc2 = configs.config4_scenarios(3, 4, 16)
    sc2.n_traces = 0
    cols = (sc.first_id + np.arange(sc.n)) % 16
    r2, _ = po.rollout(spec, sc2, np.ascontiguousarray(shared[:, :, cols]), threads=4)
    for f in r1:
        assert np.array_equal(r1[f], r2[f]), f


def test_pareto_known_answer():
    st = {"cost_uphmin": np.array([5, 3, 4, 3, 6]), "gco2": np.array([1.0, 2.0, 2.0, 2.0, 0.5]),
          "slo_minutes": np.array([0, 0, 0, 1, 9])}
    # 2 is dominated by 1 (equal carbon/SLO, cheaper); 3 by 1; 1 == itself kept
    assert po.pareto(st).tolist() == [0, 1, 4]


# ---------------------------------------------------------------- drift (SEMANTICS §3.G0)
def test_drift_prespun_replacement_in_peak_zone():
    """5 static spot pods launch in us-east-2a (off-peak) at t=0. At t=10 the
    clock reaches 16:00 and PEAK narrows the zones to us-east-2c: with drift on
    the pods have no other node, so a replacement launches in zone c at t=10
    (no consolidateAfter wait), takes the pods when ready at t=11 and the
    drifted node is deleted; no pod is ever Pending after t=0. With a single
    node slot there is no room for the replacement: the pods are evicted at
    t=10, re-provisioned at t=11 and running at t=12. Without drift the node
    stays in zone a."""
    d = deployment(abi.SCALER_STATIC, replicas0=5, min_r=5, max_r=5)
    spec = tiny_world([d], T=40, start_minute=950, pdb_pct=-1, drift=1)
    load = np.zeros((40, 1, 1), np.int32)
    r, tr = run(spec, load)
    assert r["launches"][0] == 2 and r["deletions"][0] == 1
    assert (r["last_choice"][0] >> 12) & 3 == 2              # us-east-2c
    flags = tr["flags"][:, 0]
    assert (flags[10] & 16) and (flags[10] & 32) and (flags[10] & 2) and not (flags[10] & 4)
    assert (flags[11] & 4) and not (flags[:10] & 16).any()
    n = tr["nodes_spot"][:, 0]
    assert n[9] == 1 and n[10] == 2 and n[11] == 1
    assert (tr["pending"][1:, 0] == 0).all()
    spec.max_nodes = 1
    r1, tr1 = run(spec, load)
    assert r1["launches"][0] == 2 and r1["deletions"][0] == 1
    assert (tr1["flags"][10, 0] & 16) and (tr1["flags"][10, 0] & 4)
    assert list(tr1["pending"][9:13, 0]) == [0, 5, 5, 0]
    spec.max_nodes, spec.drift = 8, 0
    r0, tr0 = run(spec, load)
    assert r0["launches"][0] == 1 and r0["deletions"][0] == 0
    assert (r0["last_choice"][0] >> 12) & 3 == 0 and (tr0["pending"][1:, 0] == 0).all()


def test_drift_blocked_by_pdb_and_budget():
    """minAvailable 50 % of 5 ready pods allows 2 evictions < 5 on the node:
    the drifted node is kept. A 0 % budget also blocks drift."""
    d = deployment(abi.SCALER_STATIC, replicas0=5, min_r=5, max_r=5)
    spec = tiny_world([d], T=30, start_minute=950, pdb_pct=50, drift=1)
    r, tr = run(spec, np.zeros((30, 1, 1), np.int32))
    assert r["deletions"][0] == 0 and (tr["pending"][1:, 0] == 0).all()
    spec = tiny_world([d], T=30, start_minute=950, pdb_pct=-1, drift=1)
    for p in spec.pools:
        p.budget_pct = 0
    r, _ = run(spec, np.zeros((30, 1, 1), np.int32))
    assert r["deletions"][0] == 0 and r["launches"][0] == 1


# ---------------------------------------------------------------- multi-trigger KEDA (SEMANTICS §3.C)
def test_keda_multi_trigger_any_active_max_proposal():
    """Trigger 0 (own column) never fires; trigger 1 (threshold 500,
    activation 100) carries 1500 for 10 steps: active via trigger 1, 0 -> 1 at
    t=0, then max(ceil(0/1000)=0, ceil(1500/500)=3) = 3; idle from t=10, back
    to 0 once 60*(t-9) >= 300. Without the trigger nothing ever activates."""
    from ccka.world import keda_trigger
    d = deployment(abi.SCALER_KEDA, replicas0=0, keda_threshold=1000, keda_activation=0,
                   keda_cooldown=300, keda_min=0, keda_max=10)
    spec = tiny_world([d, keda_trigger(500, 100)], T=30, peak_switch=0)
    load = np.zeros((30, 2, 1), np.int32)
    load[:10, 1] = 1500
    r, tr = run(spec, load)
    reps = tr["replicas"][:, 0]
    assert reps[0] == 1 and reps[1] == 3 and reps[9] == 3
    assert reps[13] > 0 and reps[14] == 0
    assert r["launches"][0] >= 1
    # the trigger alone decides: drop it and the deployment stays at zero
    spec1 = tiny_world([d], T=30, peak_switch=0)
    r1, tr1 = run(spec1, np.ascontiguousarray(load[:, :1]))
    assert (tr1["replicas"][:, 0] == 0).all() and r1["launches"][0] == 0
    # both triggers active: the larger proposal wins (own: ceil(4000/1000) = 4)
    load2 = load.copy()
    load2[:10, 0] = 4000
    _, tr2 = run(spec, load2)
    assert tr2["replicas"][1, 0] == 4


# ---------------------------------------------------------------- replacement consolidation (SEMANTICS §3.G2)
def test_replacement_consolidation_on_demand_to_cheaper():
    """Spot pool only (WhenEmptyOrUnderutilized off-peak), 5 on-demand pods.
    Hour 0 offers only 8-vCPU on-demand types, so an 8-vCPU node launches at
    t=0. From minute 60 smaller types are back: the node cannot be deleted
    (no other node) but a strictly cheaper single offering exists, so a
    replacement launches at t=60, takes the pods when ready at t=61 and the
    8-vCPU node is deleted. Pods never go Pending after t=0."""
    d = deployment(abi.SCALER_STATIC, replicas0=5, min_r=5, max_r=5, cap_sel=abi.CAP_OD)
    spec = tiny_world([d], T=90, peak_switch=0, replace=1, pdb_pct=-1)
    spec.pools = [reference_pools()[1]]
    v = spec.catalog.vcpu
    spec.price[0, 0, :, :, 1] = np.where(v[:, None] == 8, spec.price[0, 0, :, :, 1], 0)
    load = np.zeros((90, 1, 1), np.int32)
    r, tr = run(spec, load)
    n = tr["nodes_od"][:, 0].astype(int) + tr["nodes_spot"][:, 0]
    assert r["launches"][0] == 2 and r["deletions"][0] == 1
    assert tr["flags"][60, 0] & 32 and not (tr["flags"][:60, 0] & 32).any()
    assert n[59] == 1 and n[60] == 2 and n[61] == 1 and n[89] == 1
    assert (tr["pending"][1:, 0] == 0).all()
    k_new = r["last_choice"][0] & 0xFFF
    assert v[k_new] < 8
    spec.replace = 0
    r0, _ = run(spec, load)
    assert r0["launches"][0] == 1 and r0["deletions"][0] == 0
    assert r["cost_uphmin"][0] < r0["cost_uphmin"][0]
    # a 50 % PDB allows 2 of the 5 evictions: no replacement
    spec.replace, spec.pdb_pct = 1, 50
    r1, _ = run(spec, load)
    assert r1["launches"][0] == 1 and r1["deletions"][0] == 0
    spec.pdb_pct = -1
    # spot nodes are never replaced (no spot-to-spot single-node replacement)
    spec.replace = 1
    spec.deploys = [deployment(abi.SCALER_STATIC, replicas0=5, min_r=5, max_r=5, cap_sel=abi.CAP_SPOT)]
    spec.price[0, 0, :, :, 0] = np.where(v[:, None] == 8, spec.price[0, 0, :, :, 0], 0)
    r2, _ = run(spec, load)
    assert r2["launches"][0] == 1 and r2["deletions"][0] == 0


def test_drift_replacement_in_flight_is_tainted():
    """karpenter.sh/disrupted (SEMANTICS 3.G0): 5 HPA pods run
    on one spot node in us-east-2a; PEAK at t=10 drifts it and a replacement
    sized for those 5 pods launches in us-east-2c (ready at t=12, delay 2). At
    t=11 the HPA doubles the deployment. The 5 new pods must not land on the
    tainted source nor be nominated onto the in-flight replacement: they form
    a claim of their own, and the takeover at t=12 moves exactly the 5 source
    pods, evicting none (running = replicas from t=13 on)."""
    d = deployment(abi.SCALER_HPA, replicas0=5, min_r=1, max_r=20, target=50, limit_cpu=0)
    spec = tiny_world([d], T=30, start_minute=950, pdb_pct=-1, drift=1, provision_delay_steps=2)
    load = np.full((30, 1, 1), 500, np.int32)  # 5 pods x 200m at 50 %: in band
    load[11:, 0, 0] = 1000                      # 100 %: ratio 2 -> 10 replicas at t=11
    r, tr = run(spec, load)
    reps, pend, fl = tr["replicas"][:, 0], tr["pending"][:, 0], tr["flags"][:, 0]
    assert reps[10] == 5 and reps[11] == 10
    assert (fl[10] & 16) and (fl[10] & 32)          # drift at t=10: pre-spun replacement
    assert fl[11] & 2                               # the new pods get a claim of their own
    assert fl[12] & 4 and not (fl[12] & 16)         # takeover: the source goes
    assert pend[11] == 5 and pend[12] == 5          # only the new pods wait (claim ready at t=13)
    assert (pend[13:] == 0).all()
    assert r["launches"][0] == 3 and r["deletions"][0] == 1
