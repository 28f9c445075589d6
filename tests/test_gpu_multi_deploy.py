"""Multi-deployment worlds on every general-kernel instantiation
(rollout_kernel<DMAX, MAXN>: 2 / 4 / 8 / 16 deployment and 8 / 16 node-slot
register layouts; kernel_dims picks the smallest one that holds the world):
results and trajectories bit-exact against the CPU oracle. Reference side:
the burst's deployments sharing the Karpenter pools
(demo_30_burst_configure.sh:57-151) under HPA and KEDA scalers
(SURVEY a14, a15)."""
import numpy as np
import pytest

import pyoracle as po
from ccka import abi, configs
from ccka.world import ScenarioSet, deployment, keda_trigger
from parity import compare, oracle, run_engine

pytestmark = pytest.mark.gpu
THREADS = 16


def hpa(cap, **kw):
    return deployment(abi.SCALER_HPA, cap_sel=cap, **kw)


def keda(**kw):
    args = dict(replicas0=0, keda_threshold=800, keda_activation=1500, keda_cooldown=300,
                cap_sel=abi.CAP_SPOT | abi.CAP_OD)
    args.update(kw)
    return deployment(abi.SCALER_KEDA, **args)


SPOT, OD = abi.CAP_SPOT, abi.CAP_OD
WORLDS = {
    # (deployments, node slots, drift)
    "d2_n8": ([hpa(SPOT), hpa(OD, req_cpu=400, target=60)], 8, 0),
    "d2_n12_keda": ([hpa(SPOT, max_r=40), keda(keda_max=30)], 12, 0),
    "d4_n8": ([hpa(SPOT), hpa(OD, req_cpu=300, target=80), keda(keda_max=12),
               deployment(abi.SCALER_STATIC, 4, 4, 4, cap_sel=SPOT | OD)], 8, 0),
    "d4_n16_drift": ([hpa(SPOT), hpa(OD, req_cpu=500, req_mem=512, limit_cpu=1000),
                      hpa(SPOT | OD, target=50, max_r=25), keda(keda_min=1, replicas0=2)], 16, 1),
    "d7_n16": ([hpa(SPOT), hpa(OD, target=60), keda(keda_threshold=900), keda_trigger(1200, 3000),
                hpa(SPOT | OD, req_cpu=250, max_r=20),
                deployment(abi.SCALER_STATIC, 6, 6, 6, cap_sel=OD),
                deployment(abi.SCALER_STATIC, 3, 3, 3, cap_sel=SPOT)], 16, 0),
    "d12_n16_hpa": ([hpa(SPOT if d % 2 else OD, target=(50, 60, 70, 80)[d % 4], max_r=15, replicas0=2)
                     for d in range(12)], 16, 0),
}


SKEWED = {"d2_n8"}  # (d12_n16_hpa: more than four deployments keep the lockstep kernel)


@pytest.mark.parametrize("name", list(WORLDS))
def test_multi_deployment_instantiations(engine, name):
    deps, slots, drift = WORLDS[name]
    spec = configs.config2_world(n_steps=720, max_nodes=slots)
    spec.deploys = deps
    spec.drift = drift
    n = 400 if len(deps) > 4 else 900
    sc = ScenarioSet(n, 3)  # no per-scenario overrides: each deployment keeps its own settings
    load = po.gen_load(configs.trace_gen(17), spec.n_steps, len(deps), n, first_id=3)
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    # HPA / static worlds without drift run on the lane-skewed schedule (engine 5,
    # tests/test_gpu_skew.py), the others on the lockstep general kernel
    assert engine.last_engine()[0] == (5 if name in SKEWED else 1)
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    assert rc["launches"].sum() > 0 and rc["deletions"].sum() > 0
    compare(rg, rc, tg, tc)
