"""Trajectory export: ccka_host_export renders a rollout's
trajectory and results as Prometheus text exposition (the kube-state-metrics /
OpenCost series the reference's observe path scrapes: 06_opencost.sh:318-341,
404-432; demo_40_watch_config.sh:51-72) or CSV. Host code only: the rollout
feeding it here is the oracle's (the GPU trajectory is bit-identical to it,
tests/test_gpu_parity.py), so these tests run on CPU."""
import re

import numpy as np
import pytest

import pyoracle as po
from ccka import abi, configs
from ccka.host import EXPORT_CSV, EXPORT_PROMETHEUS, Host

SAMPLE = re.compile(r'^([a-zA-Z_:][a-zA-Z0-9_:]*)\{([^}]*)\} (\S+) (\d+)$')
T0 = 1_764_892_800_000  # 2025-12-05T00:00:00Z


@pytest.fixture(scope="module")
def run():
    spec = configs.config2_world(n_steps=180)
    sc = configs.hpa_scenarios(24)
    load = po.gen_load(configs.trace_gen(), spec.n_steps, 1, sc.n)
    res, tr = po.rollout(spec, sc, load, traj=True, threads=2)
    return spec, res, tr


def parse(text):
    fam, out = {}, {}
    for line in text.splitlines():
        if line.startswith("# TYPE "):
            _, _, name, typ = line.split(" ")
            assert name not in fam, f"family {name} declared twice"
            fam[name] = typ
            continue
        if line.startswith("# HELP "):
            continue
        m = SAMPLE.match(line)
        assert m, f"not exposition format: {line!r}"
        name, labels, val, ts = m.groups()
        assert name in fam, f"sample before its TYPE line: {name}"
        lab = dict(re.findall(r'(\w+)="([^"]*)"', labels))
        key = (name, tuple(sorted((k, v) for k, v in lab.items())), int(ts))
        assert key not in out, f"duplicate series sample {key}"
        out[key] = float(val)
    return fam, out


def series(samples, name, **lab):
    want = {k: str(v) for k, v in lab.items()}
    return {ts: v for (n, labs, ts), v in samples.items()
            if n == name and all(dict(labs).get(k) == x for k, x in want.items())}


def test_prometheus_matches_trajectory_and_results(run):
    spec, res, tr = run
    w = spec.to_c()
    h = Host()
    fam, s = parse(h.export(w, res, tr, EXPORT_PROMETHEUS, first_id=100, start_unix_ms=T0))
    assert fam["kube_deployment_spec_replicas"] == "gauge"
    assert fam["ccka_cost_dollars_total"] == "counter"
    T, n = tr.shape
    ts = [T0 + 60_000 * t for t in range(T)]
    for i in (0, 7, n - 1):
        sid = 100 + i
        rep = series(s, "kube_deployment_spec_replicas", scenario=sid)
        assert [rep[x] for x in ts] == tr["replicas"][:, i].tolist()
        avail = series(s, "kube_deployment_status_replicas_available", scenario=sid)
        assert [avail[x] for x in ts] == (tr["replicas"][:, i] - tr["pending"][:, i]).tolist()
        spot = series(s, "ccka_nodes", scenario=sid, capacity_type="spot")
        od = series(s, "ccka_nodes", scenario=sid, capacity_type="on-demand")
        assert [spot[x] for x in ts] == tr["nodes_spot"][:, i].tolist()
        assert [od[x] for x in ts] == tr["nodes_od"][:, i].tolist()
        prof = series(s, "ccka_policy_profile", scenario=sid)
        assert [prof[x] for x in ts] == (tr["flags"][:, i] & 1).tolist()
        for bit, ev in ((1, "launch"), (2, "deletion"), (3, "slo_violation")):
            e = series(s, "ccka_step_event", scenario=sid, event=ev)
            assert [e[x] for x in ts] == ((tr["flags"][:, i] >> bit) & 1).tolist(), ev
        last = ts[-1]
        assert series(s, "ccka_cost_dollars_total", scenario=sid) == {last: res["cost_uphmin"][i] / 6e7}
        assert series(s, "ccka_carbon_grams_total", scenario=sid) == {last: res["gco2"][i]}
        assert series(s, "ccka_energy_kwh_total", scenario=sid) == {last: res["energy_wmin"][i] / 6e4}
        assert series(s, "ccka_slo_violation_minutes_total", scenario=sid)[last] == res["slo_minutes"][i]
        assert series(s, "ccka_launches_total", scenario=sid)[last] == res["launches"][i]
        assert series(s, "ccka_deletions_total", scenario=sid)[last] == res["deletions"][i]
        nm = series(s, "ccka_node_minutes_total", scenario=sid, capacity_type="spot")
        assert nm[last] == res["node_min_spot"][i]
        # trajectory node counts integrate to the results' node-minutes
        assert int(tr["nodes_spot"][:, i].sum()) == res["node_min_spot"][i]
        assert int(tr["nodes_od"][:, i].sum()) == res["node_min_od"][i]
        pod_h = (tr["replicas"][:, i] - tr["pending"][:, i]).astype(np.int64).sum() / 60.0
        alloc = series(s, "ccka_pod_cost_dollars_per_hour", scenario=sid)[last]
        assert alloc == pytest.approx((res["cost_uphmin"][i] / 6e7) / pod_h, rel=1e-15)
    # every scenario of the range present exactly once per step per family
    assert len(series(s, "kube_deployment_spec_replicas")) == T  # keyed by ts, union over scenarios
    n_rep = sum(1 for k in s if k[0] == "kube_deployment_spec_replicas")
    assert n_rep == T * n


def test_prometheus_subrange_and_partial_results(run):
    spec, res, tr = run
    w = spec.to_c()
    h = Host()
    sub = {"cost_uphmin": res["cost_uphmin"]}
    _, s = parse(h.export(w, sub, tr, EXPORT_PROMETHEUS, s0=5, n=3, first_id=1000))
    ids = {dict(k[1])["scenario"] for k in s}
    assert ids == {"1005", "1006", "1007"}
    names = {k[0] for k in s}
    assert "ccka_cost_dollars_total" in names and "ccka_carbon_grams_total" not in names
    assert "ccka_launches_total" not in names


def test_csv_rows(run):
    spec, res, tr = run
    h = Host()
    txt = h.export(spec.to_c(), res, tr, EXPORT_CSV, s0=2, n=4)
    lines = txt.strip().split("\n")
    assert lines[0] == "scenario,step,minute,replicas,pending,nodes_spot,nodes_od,last_type,flags"
    T = tr.shape[0]
    assert len(lines) == 1 + 4 * T
    rows = np.array([[int(x) for x in ln.split(",")] for ln in lines[1:]])
    for j, i in enumerate(range(2, 6)):
        blk = rows[j * T:(j + 1) * T]
        assert (blk[:, 0] == i).all()
        assert blk[:, 1].tolist() == list(range(T))
        assert blk[:, 2].tolist() == [(spec.start_minute + t) % 1440 for t in range(T)]
        for c, f in enumerate(("replicas", "pending", "nodes_spot", "nodes_od", "last_type", "flags")):
            assert blk[:, 3 + c].tolist() == tr[f][:, i].tolist(), f


def test_export_errors(run):
    spec, res, tr = run
    h = Host()
    w = spec.to_c()
    with pytest.raises(abi.CckaError):
        h.export(w, res, tr, 7)
    with pytest.raises(abi.CckaError):
        h.export(w, res, tr, EXPORT_CSV, s0=20, n=10)
    import ctypes as C
    need = C.c_int64(0)
    small = C.create_string_buffer(16)
    r = abi.Results()
    tp = np.ascontiguousarray(tr).ctypes.data_as(C.POINTER(abi.TrajRec))
    rc = h.L.ccka_host_export(h.h, EXPORT_CSV, C.byref(w), tp, tr.shape[1], C.byref(r), 0, 1, 0, 0,
                              small, 16, C.byref(need))
    assert rc != 0 and need.value > 16
    assert b"output buffer too small" in h.L.ccka_host_last_error(h.h)
