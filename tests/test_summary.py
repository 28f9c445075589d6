"""The demo_41 summary surface (host side, CPU): `kubectl label` emulation
(demo_10_setup_configure.sh:61-62), the summary's reference columns
(demo_30_burst_observe.sh:10-11 NAME/READY/DESIRED/CAPACITY,
demo_20_offpeak_observe.sh:11 consolidationPolicy=... consolidateAfter=...,
zones by name), the per-pool / carbon.simulated breakdown, and its
Prometheus export, fed by the oracle's ccka_detail records (the GPU CLI test
checks the engine's against these)."""
import json
import re

import numpy as np
import pytest

import pyoracle as po
from ccka import abi
from ccka.host import Host
from ccka.world import ScenarioSet


def _demo_host(labels=True):
    h = Host()
    h.apply(h.manifest(-1))
    for i in range(1, 13):
        h.apply(h.manifest(i))
    h.apply(h.manifest(0))
    if labels:  # demo_10_setup_configure.sh:61-62
        h.label("NodePool", "spot-preferred", "autoscale.strategy=cost carbon.simulated=low")
        h.label("NodePool", "on-demand-slo", "autoscale.strategy=slo carbon.simulated=medium")
    return h


def test_kubectl_label_semantics():
    h = _demo_host(labels=False)
    h.label("NodePool", "spot-preferred", "carbon.simulated=low", overwrite=False)
    got = json.loads(h.get_json("NodePool", "spot-preferred"))["metadata"]["labels"]
    assert got == {"carbon.simulated": "low"}
    # same value again: fine without --overwrite; a different one is kubectl's error
    h.label("NodePool", "spot-preferred", "carbon.simulated=low", overwrite=False)
    with pytest.raises(abi.CckaError, match="already has a value \\(low\\), and --overwrite is false"):
        h.label("NodePool", "spot-preferred", "carbon.simulated=high", overwrite=False)
    h.label("NodePool", "spot-preferred", "carbon.simulated=high a=b")
    h.label("NodePool", "spot-preferred", "a-")
    got = json.loads(h.get_json("NodePool", "spot-preferred"))["metadata"]["labels"]
    assert got == {"carbon.simulated": "high"}
    with pytest.raises(abi.CckaError, match="NotFound"):
        h.label("NodePool", "nope", "x=y")
    with pytest.raises(abi.CckaError, match="at least one label"):
        h.label("NodePool", "spot-preferred", "   ")


def _run(h, load_m=450, catalog="small", steps=1440):
    w = h.build_world(catalog, steps, 16)
    load = np.full((steps, 12, 1), load_m, np.int32)
    res, traj, det = po.rollout_world(w, ScenarioSet(1), load, traj=True, detail=True)
    r = abi.Results()
    keep = []
    for name, ct, dt in abi.RESULT_FIELDS:
        a = np.ascontiguousarray(res[name], dt)
        keep.append(a)
        setattr(r, name, a.ctypes.data_as(abi.C.POINTER(ct)))
    return w, r, res, traj, det, keep


def test_summary_reference_columns():
    h = _demo_host()
    w, r, res, traj, det, _keep = _run(h)
    txt = h.summary(w, r, traj, det)
    # demo_20_offpeak_observe.sh:9-20 views, per pool, with zones by name
    assert "== spot-preferred ==" in txt and "== on-demand-slo ==" in txt
    assert re.search(r"consolidationPolicy=WhenEmpty(OrUnderutilized)?  consolidateAfter=\d+[smh]", txt)
    assert "topology.kubernetes.io/zone=In: us-east-2" in txt
    assert "karpenter.sh/capacity-type=In: " in txt
    assert "carbon.simulated=low" in txt and "carbon.simulated=medium" in txt
    # demo_30_burst_observe.sh:10-11 custom columns, the rollout's final values
    lines = txt.splitlines()
    hdr = next(i for i, ln in enumerate(lines) if ln.split()[:4] == ["NAME", "READY", "DESIRED", "CAPACITY"])
    rows = [ln.split() for ln in lines[hdr + 1:hdr + 13]]
    assert [x[0] for x in rows] == [f"burst-web-{i}" for i in range(1, 13)]
    for d, row in enumerate(rows):
        ready = int(det["ready"][0, d])
        assert row[1] == (str(ready) if ready else "<none>")
        assert row[2] == str(int(det["desired"][0, d]))
        assert row[3] == ("spot" if d % 2 == 0 else "on-demand")  # odd burst-web-N -> spot
    # per pool and per carbon.simulated group, summing to the run totals
    pools = {ln.split()[0]: ln.split() for ln in lines if ln.startswith(("spot-preferred ", "on-demand-slo "))}
    assert pools["spot-preferred"][1] == "low" and pools["on-demand-slo"][1] == "medium"
    assert "(base managed nodes)" in txt
    grp = {ln.split()[0]: float(ln.split()[1]) for ln in lines[lines.index(next(x for x in lines if x.startswith("GROUP"))) + 1:]
           if ln and ln.split()[0] in ("low", "medium", "<none>")}
    assert set(grp) == {"low", "medium", "<none>"}
    assert abs(sum(grp.values()) - res["cost_uphmin"][0] / 6e7) < 1e-3
    # without the breakdown the summary still renders (manifest replicas, marked)
    txt2 = h.summary(w, r, None, None)
    assert "(* manifest replicas" in txt2 and "NODEPOOL" not in txt2


def test_summary_final_profile_and_unlabelled_pools():
    h = _demo_host(labels=False)
    w, r, res, traj, det, _keep = _run(h, steps=300)
    txt = h.summary(w, r, traj, det)
    assert "carbon.simulated=<none>" in txt
    assert "(last step, off-peak profile)" in txt or "(last step, peak profile)" in txt


def test_export_detail_series():
    h = _demo_host()
    w, r, res, traj, det, _keep = _run(h)
    prom = h.export_detail(w, det, first_id=7, start_unix_ms=1_700_000_000_000)
    vals = {}
    for ln in prom.splitlines():
        if ln.startswith("ccka_nodepool_cost_dollars_total{"):
            lab = dict(re.findall(r'(\w+)="([^"]*)"', ln))
            vals[lab["nodepool"]] = (lab["carbon_simulated"], float(ln.split()[1]), int(ln.split()[2]))
    assert vals["spot-preferred"][0] == "low" and vals["on-demand-slo"][0] == "medium"
    assert vals["base-managed"][0] == ""
    assert abs(sum(v[1] for v in vals.values()) - res["cost_uphmin"][0] / 6e7) < 1e-9
    assert all(v[2] == 1_700_000_000_000 + 1439 * 60000 for v in vals.values())
    ready = [ln for ln in prom.splitlines() if ln.startswith("kube_deployment_status_replicas_ready{")]
    assert len(ready) == 12 and 'scenario="7"' in ready[0]
    assert sum(int(ln.split()[1]) for ln in ready) == int(det["ready"][0, :12].sum())


def test_label_syntax_validated_like_kubectl():
    """apimachinery label rules (IsQualifiedName / IsValidLabelValue): kubectl
    rejects these before they reach the object."""
    h = _demo_host(labels=False)
    for bad in ("carbon.simulated=" + "x" * 64, "carbon.simulated=-low", "carbon.simulated=lo_",
                'carbon.simulated=a"b', "b@d=1", "Example.com/x=1", "/x=1", "x/=1"):
        with pytest.raises(abi.CckaError, match="invalid label spec"):
            h.label("NodePool", "spot-preferred", bad)
    h.label("NodePool", "spot-preferred", "example.com/strategy=cost carbon.simulated=")
    got = json.loads(h.get_json("NodePool", "spot-preferred"))["metadata"]["labels"]
    assert got == {"example.com/strategy": "cost", "carbon.simulated": ""}


def test_export_detail_long_labels_not_truncated():
    """A 63-character label value (the kubectl maximum) reaches every
    Prometheus line whole; no line is cut short or loses its newline."""
    h = _demo_host(labels=False)
    v = "c" + "a" * 61 + "z"
    h.label("NodePool", "spot-preferred", f"carbon.simulated={v} autoscale.strategy={v}")
    w, r, res, traj, det, _keep = _run(h, steps=120)
    prom = h.export_detail(w, det)
    assert prom.endswith("\n")
    lines = [ln for ln in prom.splitlines() if ln.startswith("ccka_nodepool_cost_dollars_total{")]
    spot = [ln for ln in lines if 'nodepool="spot-preferred"' in ln]
    assert spot and f'carbon_simulated="{v}",autoscale_strategy="{v}"}}' in spot[0]
    for ln in prom.splitlines():
        if ln and not ln.startswith("#"):
            assert re.fullmatch(r'[a-z_]+\{[^}]*\} \S+ \d+', ln), ln
