"""Karpenter multi-node consolidation (SEMANTICS 3.G3):
>= 2 nodes of a WhenEmptyOrUnderutilized pool leave together when their pods
fit on the remaining nodes plus at most one new node that is strictly cheaper
than the set (firstN binary search over the consolidation order). The
hand-computed 2 -> 1 case runs on the oracle (CPU); the GPU parity variants
(PDB, budget, delay 0, spot sets, multi-deployment) are marked gpu."""
import numpy as np
import pytest

import pyoracle as po
from ccka import abi, configs
from ccka.world import ScenarioSet, deployment, hpa_rules
from parity import compare, run_engine
from test_oracle_kat import tiny_world

THREADS = 16


def _two_to_one_world(multi=1, delay=1, budget=100, p_xl=150):
    """Two c6i.large on-demand nodes (one 1500m pod each, placed 5 minutes
    apart) that cannot absorb each other's pod; a c6i.xlarge holds both. Only
    zone-a on-demand offerings of c6i.large (100), c6i.xlarge (p_xl) and
    c6i.2xlarge (400) exist."""
    a = deployment(abi.SCALER_STATIC, replicas0=1, min_r=1, max_r=1, req_cpu=1500, req_mem=256, limit_cpu=0,
                   cap_sel=abi.CAP_OD, pdb=0)
    b = deployment(abi.SCALER_KEDA, replicas0=0, req_cpu=1500, req_mem=256, limit_cpu=0, cap_sel=abi.CAP_OD, pdb=0,
                   keda_threshold=1000, keda_activation=100, keda_cooldown=300, keda_min=0, keda_max=10)
    spec = tiny_world([a, b], T=12, peak_switch=0, pdb_pct=-1, multi=multi, provision_delay_steps=delay)
    od = spec.pools[0]
    od.budget_pct = budget
    for pr in (abi.PROFILE_RESET, abi.PROFILE_OFFPEAK, abi.PROFILE_PEAK):
        od.profile[pr].policy = abi.WHEN_EMPTY_OR_UNDERUTILIZED
        od.profile[pr].consolidate_after_s = 0
    price = np.zeros_like(spec.price)
    k = {n: spec.catalog.index(n) for n in ("c6i.large", "c6i.xlarge", "c6i.2xlarge")}
    price[:, :, k["c6i.large"], 0, 1] = 100
    price[:, :, k["c6i.xlarge"], 0, 1] = p_xl
    price[:, :, k["c6i.2xlarge"], 0, 1] = 400
    spec.price = price
    load = np.zeros((12, 2, 1), np.int32)
    load[5:, 1] = 500  # B's KEDA trigger active from t = 5
    return spec, load, k


def test_two_to_one_hand_computed():
    spec, load, k = _two_to_one_world()
    r, tr = po.rollout(spec, ScenarioSet(1), load, traj=True)
    f = tr["flags"][:, 0]
    # t=0: node 0 = c6i.large for A; t=5: node 1 = c6i.large for B (ready t=6);
    # t=6: neither single delete fits (430m free each); the pair leaves for one
    # c6i.xlarge (150 < 100 + 100) launched into slot 2; t=7: it takes both pods
    assert (f[6] & 64) and (f[6] & 2) and (f[6] & 32)
    assert (f[7] & 4) and not (f[7] & 2)
    assert r["launches"][0] == 3 and r["deletions"][0] == 2 and r["final_nodes"][0] == 1
    assert r["last_choice"][0] & 0xFFF == k["c6i.xlarge"]
    base = 3 * int(spec.price[0, 0, spec.catalog.index("m6i.large"), 0, 1])  # 0: not offered here
    want = 5 * 100 + 1 * 200 + 1 * 350 + 5 * 150  # t0-4, t5, t6, t7-11
    assert r["cost_uphmin"][0] == want + 12 * base
    assert tr["pending"][6:, 0].tolist() == [0] * 6 and tr["nodes_od"][:, 0].tolist() == [1] * 5 + [2, 3] + [1] * 5


def test_two_to_one_needs_a_cheaper_replacement_and_budget():
    # 200 is not strictly cheaper than 100 + 100: nothing happens
    spec, load, _ = _two_to_one_world(p_xl=200)
    r, tr = po.rollout(spec, ScenarioSet(1), load, traj=True)
    assert r["launches"][0] == 2 and r["deletions"][0] == 0 and not (tr["flags"] & 64).any()
    # a 10 % budget of 2 nodes allows one disruption: no set of two
    spec, load, _ = _two_to_one_world(budget=10)
    r, tr = po.rollout(spec, ScenarioSet(1), load, traj=True)
    assert r["launches"][0] == 2 and not (tr["flags"] & 64).any()
    # off: single-node consolidation alone cannot do it
    spec, load, _ = _two_to_one_world(multi=0)
    r, tr = po.rollout(spec, ScenarioSet(1), load, traj=True)
    assert r["launches"][0] == 2 and r["final_nodes"][0] == 2


def test_two_to_one_delay0_takes_over_next_step():
    spec, load, _ = _two_to_one_world(delay=0)
    r, tr = po.rollout(spec, ScenarioSet(1), load, traj=True)
    f = tr["flags"][:, 0]
    # delay 0: B's node is ready at t=5 already, so the pair leaves at t=5 and
    # the ready replacement takes over at t=6
    assert (f[5] & 64) and (f[6] & 4)
    assert r["launches"][0] == 3 and r["deletions"][0] == 2 and r["final_nodes"][0] == 1


# ---------------------------------------------------------------- GPU parity
def _gpu_variant(name):
    spec = configs.config2_world(max_nodes=12)
    spec.multi = 1
    for p in spec.pools:
        p.budget_pct = 100
    # on-demand nodes consolidate under WhenEmptyOrUnderutilized too (spot sets
    # may not be replaced by spot: SpotToSpotConsolidation off)
    for pr in (abi.PROFILE_RESET, abi.PROFILE_OFFPEAK, abi.PROFILE_PEAK):
        spec.pools[0].profile[pr].policy = abi.WHEN_EMPTY_OR_UNDERUTILIZED
    n = 900
    sc = configs.hpa_scenarios(n, first_id=31)
    if name == "pdb":
        spec.pdb_pct = 50
    elif name == "budget50":
        for p in spec.pools:
            p.budget_pct = 50
    elif name == "delay0":
        spec.provision_delay_steps = 0
        spec.pdb_pct = -1
    elif name == "with_replace_drift":
        spec.replace = 1
        spec.drift = 1
        spec.pdb_pct = -1
    elif name == "no_pdb":
        spec.pdb_pct = -1
    elif name == "multi_deploy":
        spec.pdb_pct = -1
        spec.deploys = [
            deployment(abi.SCALER_HPA, cap_sel=abi.CAP_SPOT | abi.CAP_OD),
            deployment(abi.SCALER_HPA, req_cpu=700, req_mem=900, limit_cpu=1400,
                       cap_sel=abi.CAP_SPOT | abi.CAP_OD, target=55),
            deployment(abi.SCALER_KEDA, replicas0=0, keda_threshold=800, keda_activation=1500,
                       keda_cooldown=300, cap_sel=abi.CAP_SPOT | abi.CAP_OD),
        ]
        sc = ScenarioSet(n)
    return spec, sc


GPU_VARIANTS = ["pdb", "budget50", "delay0", "with_replace_drift", "no_pdb", "multi_deploy"]


@pytest.mark.parametrize("variant", GPU_VARIANTS)
def test_oracle_multi_consolidation_acts(variant):
    spec, sc = _gpu_variant(variant)
    load = po.gen_load(configs.trace_gen(13), spec.n_steps, len(spec.deploys), sc.n)
    _, tc = po.rollout(spec, sc, load, traj=True, threads=8)
    assert ((tc["flags"] & 64) != 0).any(), "no multi-node consolidation happened"


@pytest.mark.gpu
@pytest.mark.parametrize("variant", GPU_VARIANTS)
def test_gpu_multi_consolidation_parity(engine, variant):
    spec, sc = _gpu_variant(variant)
    load = po.gen_load(configs.trace_gen(13), spec.n_steps, len(spec.deploys), sc.n)
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    rc, tc = po.rollout(spec, sc, load, traj=True, threads=THREADS)
    assert engine.last_engine()[0] == 1
    compare(rg, rc, tg, tc)


@pytest.mark.gpu
def test_gpu_two_to_one(engine):
    spec, load, k = _two_to_one_world()
    rg, tg = run_engine(engine, spec, ScenarioSet(1), load=load, traj=True)
    rc, tc = po.rollout(spec, ScenarioSet(1), load, traj=True)
    compare(rg, rc, tg, tc)
    assert rg["final_nodes"][0] == 1 and rg["last_choice"][0] & 0xFFF == k["c6i.xlarge"]


@pytest.mark.gpu
@pytest.mark.parametrize("budget", [10, 12, 13, 25])
def test_gpu_multi_under_reference_budgets(engine, budget):
    """The reference's upstream defaults together (15 s HPA sync, drift and
    replacement at the zone switch, multi-node consolidation for the
    WhenEmptyOrUnderutilized pool, demo_20_offpeak_configure.sh:59) at the
    config-2 node count, on the single-deployment kernel: with a budget of <= 1
    node per step for any pool size (ceil(pct * 8 / 100) <= 1, the reference's
    10 %) the firstN search has no prefix of >= 2 nodes to try (no G3 at all),
    from 2 nodes on its G3 instantiation runs it. Bit-exact either way."""
    spec = configs.config2_world()
    spec.multi = 1
    spec.drift = 1
    spec.replace = 1
    spec.hpa_sync_s = 15
    for p in spec.pools:
        p.budget_pct = budget
    sc = configs.hpa_scenarios(1500, first_id=555)
    load = po.gen_load(configs.trace_gen(13), spec.n_steps, 1, sc.n, first_id=sc.first_id)
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    assert engine.last_engine()[0] == 2
    rc, tc = po.rollout(spec, sc, load, traj=True, threads=THREADS)
    compare(rg, rc, tg, tc)
    if budget <= 12:
        assert not ((tc["flags"] & 64) != 0).any()


def _d1_multi_world(name):
    """8 slots, both pools WhenEmptyOrUnderutilized, budgets admitting >= 2
    nodes: multi-node consolidation in the single-deployment kernel."""
    spec = configs.config2_world()
    spec.multi = 1
    for p in spec.pools:
        p.budget_pct = 100
    for pr in (abi.PROFILE_RESET, abi.PROFILE_OFFPEAK, abi.PROFILE_PEAK):
        spec.pools[0].profile[pr].policy = abi.WHEN_EMPTY_OR_UNDERUTILIZED
        spec.pools[1].profile[pr].policy = abi.WHEN_EMPTY_OR_UNDERUTILIZED
    sc = configs.hpa_scenarios(1200, first_id=77)
    if name == "pdb":
        spec.pdb_pct = 50
    elif name == "budget50":
        for p in spec.pools:
            p.budget_pct = 50
    elif name == "delay0":
        spec.provision_delay_steps = 0
        spec.pdb_pct = -1
    elif name == "drift_replace":
        spec.drift = 1
        spec.replace = 1
        spec.pdb_pct = -1
    elif name == "sync15":
        spec.hpa_sync_s = 15
        spec.pdb_pct = -1
    elif name == "no_pdb":
        spec.pdb_pct = -1
    elif name == "custom_rules":
        spec.pdb_pct = -1
        spec.deploys = [deployment(abi.SCALER_HPA, down=hpa_rules(abi.SELECT_MAX, [(abi.HPA_PODS, 2, 60)], 120))]
    return spec, sc


D1_VARIANTS = ["pdb", "budget50", "delay0", "drift_replace", "sync15", "no_pdb", "custom_rules"]


@pytest.mark.parametrize("variant", D1_VARIANTS)
def test_oracle_d1_multi_worlds_act(variant):
    spec, sc = _d1_multi_world(variant)
    load = po.gen_load(configs.trace_gen(17), spec.n_steps, 1, sc.n, first_id=sc.first_id)
    _, tc = po.rollout(spec, sc, load, traj=True, threads=8)
    assert ((tc["flags"] & 64) != 0).any(), "no multi-node consolidation happened"


@pytest.mark.gpu
@pytest.mark.parametrize("variant", D1_VARIANTS)
def test_gpu_multi_single_deployment_kernel(engine, variant):
    spec, sc = _d1_multi_world(variant)
    load = po.gen_load(configs.trace_gen(17), spec.n_steps, 1, sc.n, first_id=sc.first_id)
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    assert engine.last_engine()[0] == 2
    rc, tc = po.rollout(spec, sc, load, traj=True, threads=THREADS)
    compare(rg, rc, tg, tc)
