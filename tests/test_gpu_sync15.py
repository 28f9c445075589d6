"""GPU parity of the Kubernetes default HPA sync period on the single-
deployment kernel: `hpa_sync_s` 15 (kube-controller-manager
--horizontal-pod-autoscaler-sync-period default; k8s 1.34, /root/reference/
.env:4) with the default behavior runs four decisions per one-minute step
(SEMANTICS 3.C sub-steps) in rollout_d1_kernel<..., NSUB = 4>, whose down-
stabilisation records cover 20 decisions. Every variant asserts that engine
(last_engine == 2) and compares results and trajectories bit-exactly with the
CPU oracle, which evaluates the sub-steps one by one."""
import numpy as np
import pytest

import pyoracle as po
from ccka import abi, configs
from ccka.world import default_down, deployment
from parity import compare, oracle, run_engine

pytestmark = pytest.mark.gpu
THREADS = 16


def _world(name):
    spec = configs.config2_world()
    spec.hpa_sync_s = 15
    n = 2222
    sc = configs.hpa_scenarios(n, first_id=9000)
    if name.startswith("down"):  # default behavior with another down window
        spec.deploys = [deployment(abi.SCALER_HPA, down=default_down(int(name[4:])))]
    elif name == "scenario_windows":
        rng = np.random.default_rng(15)
        sc.down_stab_s = rng.choice([0, 15, 30, 45, 60, 120, 165, 240, 300, 315], n).astype(np.int16)
    elif name == "drift_replace":
        spec.drift = 1
        spec.replace = 1
    elif name == "pdb_delay0":
        spec.pdb_pct = 100
        spec.provision_delay_steps = 0
    elif name == "off_hour_start":
        spec.start_minute = 1437
        spec.n_steps = 777
    return spec, sc


VARIANTS = ["default", "down0", "down30", "down60", "down180", "down315", "scenario_windows", "drift_replace",
            "pdb_delay0", "off_hour_start"]


@pytest.mark.parametrize("variant", VARIANTS)
def test_sync15_single_deployment_parity(engine, variant):
    spec, sc = _world(variant)
    load = po.gen_load(configs.trace_gen(3), spec.n_steps, 1, sc.n, first_id=sc.first_id)
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    assert engine.last_engine()[0] == 2
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    compare(rg, rc, tg, tc)


def test_sync15_differs_from_one_decision_per_step(engine):
    """The sub-steps matter: the same world at one decision per step gives
    other trajectories (scale-ups compound within a minute), so the parity
    above is not the 60 s path in disguise."""
    spec, sc = _world("default")
    load = po.gen_load(configs.trace_gen(3), spec.n_steps, 1, sc.n, first_id=sc.first_id)
    r15, _ = run_engine(engine, spec, sc, load=load)
    spec.hpa_sync_s = 0
    r60, _ = run_engine(engine, spec, sc, load=load)
    assert (r15["slo_minutes"] != r60["slo_minutes"]).mean() > 0.05


def test_sync15_long_window_falls_back(engine):
    """A down window beyond the 20-record ring (> 315 s at 15 s) runs on the
    general kernel, still bit-exact."""
    spec, sc = _world("down600")
    load = po.gen_load(configs.trace_gen(3), spec.n_steps, 1, sc.n, first_id=sc.first_id)
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    assert engine.last_engine()[0] == 1
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    compare(rg, rc, tg, tc)
