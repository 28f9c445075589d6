"""GPU parity for the widened HPA / Karpenter range (SEMANTICS 3.C, 3.F):
windows up to 3600 s and periods up to 1800 s, four policies per direction,
`hpa_sync_s` sub-steps (the HBM decision history of the general kernel), and
NodePool spec.limits.memory; the engine against the CPU oracle, bit-exact.
Known answers for the same rules are in tests/test_hpa_range.py."""
import numpy as np
import pytest

import pyoracle as po
from ccka import abi, configs
from ccka.world import ScenarioSet, default_down, deployment, hpa_rules, keda_trigger
from parity import compare, oracle, run_engine

pytestmark = pytest.mark.gpu
THREADS = 16

UP4 = [(abi.HPA_PODS, 2, 60), (abi.HPA_PERCENT, 50, 300), (abi.HPA_PODS, 6, 1800), (abi.HPA_PERCENT, 10, 900)]
DN4 = [(abi.HPA_PODS, 1, 120), (abi.HPA_PERCENT, 20, 600), (abi.HPA_PODS, 3, 1800), (abi.HPA_PERCENT, 5, 60)]


def _variant(name):
    spec = configs.config2_world()
    n = 1111
    sc = configs.hpa_scenarios(n, first_id=4242)
    if name == "window3600":
        spec.deploys = [deployment(abi.SCALER_HPA, down=default_down(3600))]
    elif name == "scenario_windows":
        rng = np.random.default_rng(5)
        sc.down_stab_s = rng.choice([0, 300, 900, 1800, 3600], n).astype(np.int16)
    elif name == "policies4_max":
        spec.deploys = [deployment(abi.SCALER_HPA, up=hpa_rules(abi.SELECT_MAX, UP4, 120),
                                   down=hpa_rules(abi.SELECT_MAX, DN4, 1200))]
    elif name == "policies4_min":
        spec.deploys = [deployment(abi.SCALER_HPA, up=hpa_rules(abi.SELECT_MIN, UP4, 0),
                                   down=hpa_rules(abi.SELECT_MIN, DN4, 600))]
    elif name == "sync15_window3600":
        spec.hpa_sync_s = 15
        spec.deploys = [deployment(abi.SCALER_HPA, down=default_down(3600),
                                   up=hpa_rules(abi.SELECT_MAX, UP4, 60))]
    elif name.startswith("sync"):
        spec.hpa_sync_s = int(name[4:])
    elif name == "mem_limit":
        for p in spec.pools:
            p.limit_mem_mi = 48 * 1024
    elif name == "mem_cpu_limit_drift":
        for p in spec.pools:
            p.limit_mem_mi = 40 * 1024
            p.limit_cpu_m = 24000
        spec.drift = 1
        spec.replace = 1
    return spec, sc


VARIANTS = ["window3600", "scenario_windows", "policies4_max", "policies4_min", "sync10", "sync15", "sync20",
            "sync30", "sync15_window3600", "mem_limit", "mem_cpu_limit_drift"]


@pytest.mark.parametrize("variant", VARIANTS)
def test_hpa_range_parity(engine, variant):
    spec, sc = _variant(variant)
    load = po.gen_load(configs.trace_gen(7), spec.n_steps, 1, sc.n, first_id=sc.first_id)
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    # beyond the register rings / limits: the general kernel; the Kubernetes
    # default 15 s sync with the default behavior runs on the single-deployment
    # kernel (tests/test_gpu_sync15.py)
    assert engine.last_engine()[0] == (2 if variant == "sync15" else 1)
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    compare(rg, rc, tg, tc)
    if variant.startswith("mem"):
        # the memory limit binds: the launches differ from the unlimited world's
        spec0, _ = _variant("none")
        r0, _ = oracle(spec0, sc, load, threads=THREADS)
        assert (rc["choice_hash"] != r0["choice_hash"]).mean() > 0.05


def test_multi_deployment_keda_substeps(engine):
    """HPA + KEDA (two triggers) + a static deployment at a 15-s sync with four
    policies, a 1-hour window and a memory limit, drift on."""
    spec = configs.config2_world(max_nodes=12)
    spec.hpa_sync_s = 15
    spec.drift = 1
    spec.pdb_pct = -1
    for p in spec.pools:
        p.limit_mem_mi = 96 * 1024
    spec.deploys = [
        deployment(abi.SCALER_HPA, cap_sel=abi.CAP_SPOT, up=hpa_rules(abi.SELECT_MAX, UP4, 0),
                   down=hpa_rules(abi.SELECT_MAX, DN4, 3600)),
        deployment(abi.SCALER_KEDA, replicas0=0, keda_threshold=800, keda_activation=1500, keda_cooldown=300,
                   cap_sel=abi.CAP_SPOT | abi.CAP_OD),
        keda_trigger(400, 900),
        deployment(abi.SCALER_STATIC, replicas0=3, min_r=3, max_r=3, cap_sel=abi.CAP_OD),
    ]
    n = 300
    sc = ScenarioSet(n)
    load = po.gen_load(configs.trace_gen(11), spec.n_steps, 4, n)
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    compare(rg, rc, tg, tc)


def test_register_path_unchanged_by_sync60(engine):
    """hpa_sync_s 60 is the one-decision-per-step default: the single-deployment
    engine still runs it, with the same results as hpa_sync_s 0."""
    spec = configs.config2_world()
    sc = configs.hpa_scenarios(777)
    load = po.gen_load(configs.trace_gen(), spec.n_steps, 1, sc.n)
    r0, t0 = run_engine(engine, spec, sc, load=load, traj=True)
    spec.hpa_sync_s = 60
    r1, t1 = run_engine(engine, spec, sc, load=load, traj=True)
    assert engine.last_engine()[0] == 2
    compare(r1, r0, t1, t0)
