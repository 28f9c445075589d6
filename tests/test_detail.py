"""The per-scenario breakdown behind the demo_41 summary (ccka_detail,
ccka_set_detail / ccka_get_detail): per NodePool cost / energy / gCO2 /
node-minutes / launches / final and peak nodes, the base managed node group,
and per Deployment the final DESIRED / READY / pending
(demo_30_burst_observe.sh:10-11).

CPU: the oracle's breakdown adds up to its own run totals (integer fields
exactly, gCO2 to rounding) and matches the trajectory's last step.
GPU: the engine's breakdown equals the oracle's bit for bit, and recording it
leaves the results unchanged (the detail run takes the general kernel)."""
import numpy as np
import pytest

import pyoracle as po
from ccka import abi, configs
from ccka.world import ScenarioSet, deployment
from parity import compare, run_engine

THREADS = 16
INT_DETAIL = ["pool_cost_uphmin", "pool_energy_nwmin", "pool_node_min_spot", "pool_node_min_od",
              "pool_final_nodes", "pool_peak_nodes", "pool_launches", "desired", "ready", "pending",
              "base_cost_uphmin", "base_energy_nwmin"]
FP_DETAIL = ["pool_gco2", "base_gco2"]


def _multi_world():
    spec = configs.config2_world(max_nodes=12)
    spec.drift = 1
    spec.replace = 1
    spec.pdb_pct = -1
    spec.deploys = [
        deployment(abi.SCALER_HPA, cap_sel=abi.CAP_SPOT),
        deployment(abi.SCALER_HPA, req_cpu=500, req_mem=512, limit_cpu=1000, cap_sel=abi.CAP_OD, target=60),
        deployment(abi.SCALER_KEDA, replicas0=0, keda_threshold=800, keda_activation=1500,
                   keda_cooldown=300, cap_sel=abi.CAP_SPOT | abi.CAP_OD),
    ]
    return spec


def _cases():
    out = []
    spec = configs.config2_world()
    sc = configs.hpa_scenarios(333, first_id=41)
    out.append(("config2", spec, sc, po.gen_load(configs.trace_gen(), spec.n_steps, 1, sc.n, first_id=41)))
    spec = _multi_world()
    sc = ScenarioSet(97)
    out.append(("multi_drift_replace", spec, sc, po.gen_load(configs.trace_gen(9), spec.n_steps, 3, sc.n)))
    spec = configs.config1_world()
    sc = ScenarioSet(1)
    out.append(("config1_replay", spec, sc, np.zeros((spec.n_steps, 12, 1), np.int32) + 100))
    return out


def _check_consistent(spec, res, traj, det):
    P, D = len(spec.pools), len(spec.deploys)
    assert np.array_equal(det["pool_cost_uphmin"][:, :P].sum(1) + det["base_cost_uphmin"], res["cost_uphmin"])
    e = det["pool_energy_nwmin"][:, :P].sum(1) + det["base_energy_nwmin"]
    assert np.array_equal(e * 1e-9, res["energy_wmin"]) or np.allclose(e * 1e-9, res["energy_wmin"], rtol=1e-15)
    g = det["pool_gco2"][:, :P].sum(1) + det["base_gco2"]
    assert np.allclose(g, res["gco2"], rtol=1e-12)
    assert np.array_equal(det["pool_node_min_spot"][:, :P].sum(1), res["node_min_spot"])
    assert np.array_equal(det["pool_node_min_od"][:, :P].sum(1), res["node_min_od"])
    assert np.array_equal(det["pool_launches"][:, :P].sum(1), res["launches"])
    assert np.array_equal(det["pool_final_nodes"][:, :P].sum(1), res["final_nodes"])
    assert (det["pool_peak_nodes"][:, :P].sum(1) >= res["peak_nodes"]).all()
    assert np.array_equal(det["desired"][:, :D].sum(1), res["final_replicas"])
    assert np.array_equal(det["pending"][:, :D].sum(1), traj["pending"][-1])
    assert np.array_equal(det["desired"] - det["ready"], det["pending"])
    assert (det["ready"] >= 0).all()
    # unused pool / deployment slots stay zero
    assert not det["pool_cost_uphmin"][:, P:].any() and not det["desired"][:, D:].any()


@pytest.mark.parametrize("case", [c[0] for c in _cases()])
def test_oracle_detail_adds_up(case):
    name, spec, sc, load = next(c for c in _cases() if c[0] == case)
    res, traj, det = po.rollout(spec, sc, load, traj=True, threads=8, detail=True)
    res2, traj2 = po.rollout(spec, sc, load, traj=True, threads=8)
    for f in res:  # recording the breakdown changes nothing
        assert np.array_equal(res[f], res2[f]), f
    _check_consistent(spec, res, traj, det)
    assert det["pool_cost_uphmin"].sum() > 0
    if name == "config1_replay":
        # demo_30: 12 Deployments x 5 replicas, odd -> spot, even -> on-demand
        assert list(det["desired"][0, :12]) == [5] * 12


def test_detail_dtype_matches_header():
    assert abi.detail_dtype().itemsize == 392


@pytest.mark.gpu
@pytest.mark.parametrize("case", [c[0] for c in _cases()])
def test_gpu_detail_parity(engine, case):
    name, spec, sc, load = next(c for c in _cases() if c[0] == case)
    engine.set_detail(True)
    try:
        rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
        assert engine.last_engine()[0] == 1  # the summary path runs the general kernel
        dg = engine.detail()
    finally:
        engine.set_detail(False)
    rc, tc, dc = po.rollout(spec, sc, load, traj=True, threads=THREADS, detail=True)
    compare(rg, rc, tg, tc)
    for f in INT_DETAIL:
        bad = np.argwhere(dg[f] != dc[f])
        assert bad.size == 0, f"{f}: first mismatches {bad[:5].tolist()}"
    for f in FP_DETAIL:
        assert np.array_equal(dg[f], dc[f]), f
    # a rollout without detail leaves nothing to read
    run_engine(engine, spec, sc, load=load)
    with pytest.raises(abi.CckaError):
        engine.detail()
