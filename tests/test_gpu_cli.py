"""GPU: the drop-in CLI (`ccka replay`, manifests in -> summary out) against the
oracle on the world the host library builds from the same manifests
(BASELINE config 1: demo_20/21/30 replay, 12 burst Deployments, 3 base nodes)."""
import json
import os
import subprocess

import numpy as np
import pytest

import pyoracle as po
from ccka import abi
from ccka.host import CLI, Host
from ccka.world import ScenarioSet
from parity import INT_FIELDS

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("load_m,catalog,drift,sync", [(100, "tiny", 0, 0), (450, "small", 0, 0), (450, "small", 1, 0),
                                                        (450, "small", 3, 0), (450, "small", 1, 15)])
def test_cli_replay_matches_oracle(tmp_path, load_m, catalog, drift, sync):
    out = tmp_path / "r.json"
    env = {k: v for k, v in os.environ.items() if k not in ("COUNT", "REPLICAS", "NP_SPOT", "NP_OD")}
    prom = tmp_path / "r.prom"
    txt = subprocess.run([CLI, "replay", "--catalog", catalog, "--load-m", str(load_m), "--json", str(out),
                          "--prom", str(prom)] + (["--drift"] if drift & 1 else [])
                         + (["--replace"] if drift & 2 else []) + (["--hpa-sync", str(sync)] if sync else []),
                         env=env, check=True, capture_output=True, text=True, timeout=120).stdout
    assert "cost=$" in txt and "spot-preferred" in txt
    got = json.load(open(out))
    h = Host()
    h.apply(h.manifest(-1))
    for i in range(1, 13):
        h.apply(h.manifest(i))
    h.apply(h.manifest(0))
    h.label("NodePool", "spot-preferred", "autoscale.strategy=cost carbon.simulated=low")
    h.label("NodePool", "on-demand-slo", "autoscale.strategy=slo carbon.simulated=medium")
    w = h.build_world(catalog, 1440, 16)
    w.disrupt_ext = drift
    w.hpa_sync_s = sync
    load = np.full((1440, 12, 1), load_m, np.int32)
    want, traj, det = po.rollout_world(w, ScenarioSet(1), load, traj=True, detail=True)
    for f in INT_FIELDS:
        assert got[f] == int(want[f][0]), f
    for f in ("energy_wmin", "gco2"):
        assert got[f] == float(want[f][0]), f
    # the engine's per-pool / per-deployment breakdown (ccka_get_detail) == the oracle's
    P, D = w.n_pools, w.n_deploy
    gd = got["detail"]
    for f in ("pool_cost_uphmin", "pool_energy_nwmin", "pool_node_min_spot", "pool_node_min_od",
              "pool_final_nodes", "pool_peak_nodes", "pool_launches"):
        assert gd[f] == det[f][0, :P].tolist(), f
    for f in ("desired", "ready", "pending"):
        assert gd[f] == det[f][0, :D].tolist(), f
    assert gd["pool_gco2"] == det["pool_gco2"][0, :P].tolist()
    for f in ("base_cost_uphmin", "base_energy_nwmin", "base_gco2"):
        assert gd[f] == det[f][0], f
    # the summary prints the reference's columns from it, identically to the
    # host library fed with the oracle's records
    r = abi.Results()
    keep = []
    for name, ct, dt in abi.RESULT_FIELDS:
        a = np.ascontiguousarray(want[name], dt)
        keep.append(a)
        setattr(r, name, a.ctypes.data_as(abi.C.POINTER(ct)))
    assert txt == h.summary(w, r, traj, det)
    lines = txt.splitlines()
    hdr = next(i for i, ln in enumerate(lines) if ln.split()[:4] == ["NAME", "READY", "DESIRED", "CAPACITY"])
    assert [ln.split()[0] for ln in lines[hdr + 1:hdr + 13]] == [f"burst-web-{i}" for i in range(1, 13)]
    assert "consolidationPolicy=" in txt and "carbon.simulated=low" in txt and "NODEPOOL" in txt
    assert 'ccka_nodepool_cost_dollars_total{scenario="0",nodepool="spot-preferred",carbon_simulated="low"' in open(prom).read()
    # the exported run totals are the same results
    lines = [ln for ln in open(prom).read().splitlines() if ln.startswith("ccka_launches_total{")]
    assert len(lines) == 1 and float(lines[0].split()[1]) == got["launches"]
