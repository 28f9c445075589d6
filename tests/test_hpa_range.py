"""The upstream HPA behavior range (autoscaling/v2, k8s 1.34 as .env:4 pins):
stabilizationWindowSeconds up to 3600 s, policy periodSeconds up to 1800 s,
more than two policies per direction, and the controller's sync period
(--horizontal-pod-autoscaler-sync-period, default 15 s) as `hpa_sync_s`
decisions per 60-s step (SEMANTICS 3.C). Known answers are
hand-computed from SEMANTICS; the GPU parity of the same worlds is in
tests/test_gpu_hpa_range.py."""
import ctypes as C

import numpy as np
import pytest

import pyoracle as po
from ccka import abi
from ccka.world import ScenarioSet, default_down, default_up, deployment, hpa_rules
from test_oracle_kat import tiny_world

L = po.lib()
H = abi.HPA_HIST_MAX


def behavior_n(cur, prop, mn, mx, up, down, sync=60, recs=(), valid=(), deltas=()):
    r = (C.c_int32 * H)(*([*recs] + [0] * (H - len(recs))))
    v = (C.c_uint8 * H)(*([*valid] + [0] * (H - len(valid))))
    d = (C.c_int32 * H)(*([*deltas] + [0] * (H - len(deltas))))
    return L.ccka_oracle_hpa_behavior_n(cur, prop, mn, mx, C.byref(up), C.byref(down), sync, r, v, d, H)


def test_one_hour_down_stabilisation():
    # 3600 s window at one decision per minute: entries 0..58 (ages 60..3540 s) count
    down = default_down(3600)
    recs = [5] * 58 + [30]          # the 30 is 3540 s old: inside
    assert behavior_n(10, 5, 1, 100, default_up(), down, recs=recs, valid=[1] * 59) == 10  # capped at cur
    assert behavior_n(40, 5, 1, 100, default_up(), down, recs=recs, valid=[1] * 59) == 30
    recs = [5] * 59 + [30]          # 3600 s old: not strictly newer than the window
    assert behavior_n(40, 5, 1, 100, default_up(), down, recs=recs, valid=[1] * 60) == 5


def test_four_policies_and_long_periods():
    # Max of four scale-up policies; the 1800-s Pods policy sees 29 entries of history
    pol = [(abi.HPA_PODS, 1, 60), (abi.HPA_PODS, 2, 120), (abi.HPA_PERCENT, 10, 1800), (abi.HPA_PODS, 3, 600)]
    up = hpa_rules(abi.SELECT_MAX, pol, 0)
    # no history: limits 10+1, 10+2, ceil(11.0)=11, 10+3 -> Max = 13
    assert behavior_n(10, 50, 1, 100, up, default_down()) == 13
    # +6 at 1740 s ago (entry 28) only the 1800-s policy sees: its base 4 -> ceil(4.4)=5;
    # +2 at 300 s ago (entry 4): 600-s policy base 8 -> 11; 60/120-s policies -> 11, 12
    deltas = [0] * 29
    deltas[28], deltas[4] = 6, 2
    assert behavior_n(10, 50, 1, 100, up, default_down(), deltas=deltas) == 12
    mn = hpa_rules(abi.SELECT_MIN, pol, 0)
    assert behavior_n(10, 50, 1, 100, mn, default_down(), deltas=deltas) == 10  # Min: ceil(4.4)=5 < cur -> cur
    # four scale-down policies, Max selects the biggest drop (the smallest count)
    dn = hpa_rules(abi.SELECT_MAX, [(abi.HPA_PODS, 1, 60), (abi.HPA_PERCENT, 50, 1800),
                                    (abi.HPA_PODS, 4, 300), (abi.HPA_PERCENT, 10, 60)], 0)
    assert behavior_n(20, 1, 1, 100, default_up(), dn) == 10           # 20 * 0.5
    d2 = [0] * 29
    d2[20] = -10                     # 1260 s ago: the 1800-s policy's base is 30 -> 15
    assert behavior_n(20, 1, 1, 100, default_up(), dn, deltas=d2) == 15  # min(19, 15, 16, 18)


def test_sync_period_entries():
    # at a 15-s sync a 60-s window holds the 3 newest decisions (ages 15, 30, 45 s)
    down = default_down(60)
    assert behavior_n(20, 2, 1, 100, default_up(), down, sync=15, recs=[3, 4, 9], valid=[1, 1, 1]) == 9
    assert behavior_n(20, 2, 1, 100, default_up(), down, sync=15, recs=[3, 4, 5, 9], valid=[1] * 4) == 5
    # the default up policies (15-s periods) see no history at a 15-s sync
    assert behavior_n(5, 80, 1, 100, default_up(), default_down(), sync=15, deltas=[4]) == 10


def _burst_world(sync, T=2, down=None, **kw):
    dep = deployment(abi.SCALER_HPA, replicas0=1, min_r=1, max_r=100, target=50, req_cpu=100, req_mem=64,
                     limit_cpu=0, down=down)
    return tiny_world([dep], T=T, peak_switch=0, hpa_sync_s=sync, **kw)


@pytest.mark.parametrize("sync,want", [(0, 5), (60, 5), (30, 10), (20, 20), (15, 40)])
def test_sync_substeps_compound_scale_up(sync, want):
    """t=1: the first pod is ready, 4000m of load on a 100m request at a 50 %
    target -> proposal 80. Each decision of the step may add max(+4, +100 %)
    (15-s periods: no earlier decision inside), so 1 -> 5 -> 10 -> 20 -> 40
    over the step's sub-steps; the unready pods keep the proposal at 80."""
    spec = _burst_world(sync)
    load = np.full((2, 1, 1), 4000, np.int32)
    r, tr = po.rollout(spec, ScenarioSet(1), load, traj=True)
    assert tr["replicas"][0, 0] == 1 and tr["replicas"][1, 0] == want


def test_hour_long_stabilisation_holds_replicas():
    """A 10-minute burst then idle: with a 3600-s down window the replicas hold
    for an hour after the last high recommendation, then drop."""
    spec = _burst_world(0, T=150, down=default_down(3600))
    load = np.zeros((150, 1, 1), np.int32) + 10
    load[:10] = 4000
    r, tr = po.rollout(spec, ScenarioSet(1), load, traj=True)
    reps = tr["replicas"][:, 0]
    peak = reps.max()
    assert peak > 20
    hold = reps[10:69]
    assert (hold == peak).all(), hold
    assert reps[-1] < peak


def test_pool_memory_limit():
    """NodePool spec.limits.memory bounds the pool's node memory capacity like
    limits.cpu bounds its vCPU (SEMANTICS 3.F): 0 MiB admits no node; 8 GiB
    admits only nodes that keep the pool's total within 8 GiB."""
    dep = deployment(abi.SCALER_STATIC, replicas0=30, min_r=30, max_r=30, req_cpu=200, req_mem=128,
                     cap_sel=abi.CAP_SPOT)
    spec = tiny_world([dep], T=30, peak_switch=0)
    load = np.full((30, 1, 1), 500, np.int32)
    for p in spec.pools:
        p.limit_mem_mi = 0
    r, tr = po.rollout(spec, ScenarioSet(1), load, traj=True)
    assert r["launches"][0] == 0 and tr["pending"][-1, 0] == 30
    for p in spec.pools:
        p.limit_mem_mi = 8192
    r, tr, det = po.rollout(spec, ScenarioSet(1), load, traj=True, detail=True)
    mem = (spec.catalog.mem_gib * 1024).astype(int)
    assert r["launches"][0] >= 1
    assert mem[r["last_choice"][0] & 0xFFF] <= 8192
    assert det["pool_peak_nodes"][0, 1] * mem.min() <= 8192
    assert tr["pending"][-1, 0] > 0  # 6 vCPU of pods do not fit in 8 GiB of nodes
    for p in spec.pools:
        p.limit_mem_mi = -1
    r2, tr2 = po.rollout(spec, ScenarioSet(1), load, traj=True)
    assert tr2["pending"][-1, 0] == 0


HPA_YAML = """
apiVersion: apps/v1
kind: Deployment
metadata: {name: web}
spec:
  replicas: 3
  template:
    spec:
      containers:
      - name: c
        resources:
          requests: {cpu: 250m, memory: 1Gi}
---
apiVersion: autoscaling/v2
kind: HorizontalPodAutoscaler
metadata: {name: web-hpa}
spec:
  scaleTargetRef: {apiVersion: apps/v1, kind: Deployment, name: web}
  minReplicas: 2
  maxReplicas: 60
  metrics:
  - type: Resource
    resource: {name: cpu, target: {type: Utilization, averageUtilization: 60}}
  behavior:
    scaleUp:
      stabilizationWindowSeconds: 600
      policies:
      - {type: Pods, value: 4, periodSeconds: 60}
      - {type: Percent, value: 100, periodSeconds: 300}
      - {type: Pods, value: 10, periodSeconds: 1800}
      - {type: Percent, value: 20, periodSeconds: 900}
    scaleDown:
      stabilizationWindowSeconds: 3600
      selectPolicy: Min
      policies:
      - {type: Percent, value: 10, periodSeconds: 1800}
"""


def test_host_ingests_upstream_range_and_memory_limit():
    from ccka.host import Host
    h = Host()
    h.apply(h.manifest(-1))
    h.patch("NodePool", "spot-preferred", "merge", '{"spec":{"limits":{"cpu":"64","memory":"256Gi"}}}')
    h.apply(HPA_YAML)
    w = h.build_world("small", 1440, 16)
    names = ["on-demand-slo", "spot-preferred"]
    sp = w.pools[names.index("spot-preferred")]
    assert (sp.limit_cpu_m, sp.limit_mem_mi) == (64000, 256 * 1024)
    assert w.pools[names.index("on-demand-slo")].limit_mem_mi == -1
    d = w.deploy[0]
    assert d.up.n_policies == 4 and d.up.stab_window_s == 600
    assert [(d.up.policies[i].type, d.up.policies[i].value, d.up.policies[i].period_s) for i in range(4)] == [
        (abi.HPA_PODS, 4, 60), (abi.HPA_PERCENT, 100, 300), (abi.HPA_PODS, 10, 1800), (abi.HPA_PERCENT, 20, 900)]
    assert (d.down.stab_window_s, d.down.select, d.down.n_policies) == (3600, abi.SELECT_MIN, 1)
    # five policies are beyond the model
    with pytest.raises(abi.CckaError, match="more than 4 policies"):
        h.apply(HPA_YAML.replace("      - {type: Percent, value: 20, periodSeconds: 900}",
                                 "      - {type: Percent, value: 20, periodSeconds: 900}\n"
                                 "      - {type: Pods, value: 1, periodSeconds: 60}"))
        h.build_world("small", 1440, 16)
