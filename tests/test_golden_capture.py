"""Pins the drop-in boundary to the reference's own outputs.

tests/golden/reference_capture/ holds the payloads the reference's scripts
(demo_19/10/20/21/30) handed to kubectl when run unmodified with stub
kubectl/aws (generator: tests/golden/capture_reference.sh). These tests check
that (1) our C++ generators reproduce every payload byte for byte, (2) the
YAML/JSON ingest reads them back into the engine's world exactly as the
Python world builder (and therefore the oracle and the GPU) assumes, and
(3) kubectl apply/patch emulation behaves like the scripts expect."""
import glob
import hashlib
import json
import os
import subprocess

import pytest

from ccka import abi
from ccka.host import CLI, HOST_EXPORTED, Host, lib
from ccka.world import burst_deployments, reference_pools, zone_mask

GOLD = os.path.join(os.path.dirname(__file__), "golden", "reference_capture")


def read(variant, pattern):
    files = sorted(glob.glob(os.path.join(GOLD, variant, pattern)))
    assert files, (variant, pattern)
    return [open(f).read() for f in files]


def cli(*args, **env):
    e = dict(os.environ)
    for k in ("NP_SPOT", "NP_OD", "OFFPEAK_ZONES", "PEAK_ZONES", "NAMESPACE", "COUNT", "REPLICAS"):
        e.pop(k, None)
    e.update(env)
    return subprocess.run([CLI, *args], env=e, check=True, capture_output=True, text=True).stdout


def test_fixture_integrity():
    want = {}
    for line in open(os.path.join(os.path.dirname(GOLD), "reference_capture.sha256")):
        h, f = line.split()
        want[f] = h
    for f, h in want.items():
        assert hashlib.sha256(open(os.path.join(GOLD, f), "rb").read()).hexdigest() == h, f


def test_host_library_exports():
    L = lib()
    for s in HOST_EXPORTED:
        assert hasattr(L, s), s


@pytest.mark.parametrize("variant,profile,env", [
    ("offpeak_default", "offpeak", {}),
    ("peak_default", "peak", {}),
    ("offpeak_two_zones", "offpeak", {"OFFPEAK_ZONES": "us-east-2a,us-east-2b"}),
    ("offpeak_empty_env", "offpeak", {"OFFPEAK_ZONES": ""}),
    ("peak_space_zones", "peak", {"PEAK_ZONES": "us-east-2b us-east-2c"}),
    ("offpeak_custom_np", "offpeak", {"NP_SPOT": "cheap-pool", "NP_OD": "slo-pool"}),
])
def test_requirement_and_merge_patches_byte_identical(variant, profile, env):
    spot = env.get("NP_SPOT", "spot-preferred")
    od = env.get("NP_OD", "on-demand-slo")
    for pool in (spot, od):
        got_json = cli("patch", profile, "--pool", pool, "--json", **env)
        assert got_json == read(variant, f"*_patch_nodepool_{pool}_json.json")[0]
        got_merge = cli("patch", profile, "--pool", pool, **env)
        assert got_merge == read(variant, f"*_patch_nodepool_{pool}_merge.json")[0]


def test_reset_merge_patch_byte_identical():
    for pool in ("spot-preferred", "on-demand-slo"):
        assert cli("patch", "reset", "--pool", pool) == read("reset_default", f"*_{pool}_merge.json")[0]


@pytest.mark.parametrize("variant,env,count", [
    ("burst_default", {}, 12),
    ("burst_small", {"COUNT": "3", "REPLICAS": "2", "NAMESPACE": "ns-small"}, 3),
])
def test_burst_deployments_byte_identical(variant, env, count):
    captured = read(variant, "*_apply.yaml")[1:]  # [0] is the RBAC Role/RoleBinding apply
    assert len(captured) == count
    for i in range(1, count + 1):
        assert cli("manifest", "burst", "--index", str(i), **env) == captured[i - 1], i


def test_pdb_manifest_matches_capture():
    setup = read("setup_default", "*_apply.yaml")[0]
    assert setup.endswith(cli("manifest", "pdb"))
    labels = read("setup_default", "*_label.txt")
    assert "carbon.simulated=low" in labels[0] and "carbon.simulated=medium" in labels[1]


def _payload_patch(variant, pool):
    merge = json.loads(read(variant, f"*_patch_nodepool_{pool}_merge.json")[0])
    jp = json.loads(read(variant, f"*_patch_nodepool_{pool}_json.json")[0])
    dis = merge["spec"]["disruption"]
    pol = {"WhenEmpty": abi.WHEN_EMPTY, "WhenEmptyOrUnderutilized": abi.WHEN_EMPTY_OR_UNDERUTILIZED}
    ca = int(dis["consolidateAfter"].rstrip("s")) if "consolidateAfter" in dis else -1
    reqs = {r["key"]: r["values"] for r in jp[0]["value"]}
    caps = sum({"spot": abi.CAP_SPOT, "on-demand": abi.CAP_OD}[c] for c in reqs["karpenter.sh/capacity-type"])
    return (pol[dis["consolidationPolicy"]], ca, zone_mask(reqs["topology.kubernetes.io/zone"]), caps)


def test_world_profiles_are_the_captured_patches():
    """The profile table the oracle and the GPU run with (ccka/world.py) is what
    the reference's captured payloads say."""
    pools = reference_pools()
    names = ["on-demand-slo", "spot-preferred"]  # Karpenter order: equal weight, name asc
    for q, name in enumerate(names):
        for prof, variant in ((abi.PROFILE_OFFPEAK, "offpeak_default"), (abi.PROFILE_PEAK, "peak_default")):
            p = pools[q].profile[prof]
            assert (p.policy, p.consolidate_after_s, p.zone_mask, p.cap_mask) == _payload_patch(variant, name)
        reset = json.loads(read("reset_default", f"*_{name}_merge.json")[0])["spec"]["disruption"]
        r = pools[q].profile[abi.PROFILE_RESET]
        assert (r.policy, r.consolidate_after_s) == (abi.WHEN_EMPTY, int(reset["consolidateAfter"].rstrip("s")))


def test_ingest_captured_manifests_into_world():
    """YAML ingest of the captured demo_30 Deployments + demo_10 PDB gives the
    deployments the replay config (ccka.configs.config1_world) uses."""
    h = Host()
    h.apply(h.manifest(-1))  # base NodePools
    for y in read("burst_default", "*_apply.yaml")[1:]:
        h.apply(y)
    h.apply(read("setup_default", "*_apply.yaml")[0])  # SA, Role, RoleBinding, PDB
    w = h.build_world("tiny", 1440, 16)
    want = burst_deployments(12, 5)
    assert w.n_deploy == 12 and w.pdb_min_available_pct == 50 and w.n_pools == 2
    for d in range(12):
        a, b = w.deploy[d], want[d]
        for f in ("scaler", "replicas0", "req_cpu_m", "req_mem_mi", "limit_cpu_m", "cap_sel", "pdb_member"):
            assert getattr(a, f) == getattr(b, f), (d, f)
    ref = reference_pools()
    for q in range(2):
        for prof in range(3):
            a, b = w.pools[q].profile[prof], ref[q].profile[prof]
            assert (a.policy, a.consolidate_after_s, a.zone_mask, a.cap_mask) == \
                   (b.policy, b.consolidate_after_s, b.zone_mask, b.cap_mask), (q, prof)


def test_kubectl_patch_emulation_and_fallback():
    """apply_and_verify (demo_20_offpeak_configure.sh:84-127): the primary path
    /spec/template/spec/requirements works on a v1 NodePool; on a pool without
    /spec/template/spec the JSON Patch fails like kubectl and the fallback
    path is used."""
    h = Host()
    h.apply(h.manifest(-1))
    h.patch("NodePool", "spot-preferred", "json", h.policy_patch(abi.PROFILE_OFFPEAK, "spot-preferred", True))
    h.patch("NodePool", "spot-preferred", "merge", h.policy_patch(abi.PROFILE_OFFPEAK, "spot-preferred", False))
    got = json.loads(h.get_json("NodePool", "spot-preferred"))
    reqs = {r["key"]: r["values"] for r in got["spec"]["template"]["spec"]["requirements"]}
    assert reqs["topology.kubernetes.io/zone"] == ["us-east-2a"]
    assert got["spec"]["disruption"]["consolidationPolicy"] == "WhenEmptyOrUnderutilized"
    assert got["spec"]["disruption"]["consolidateAfter"] == "0s"  # merge keeps the old value
    h.apply("apiVersion: karpenter.sh/v1beta1\nkind: NodePool\nmetadata:\n  name: legacy\nspec:\n  template: {}\n")
    with pytest.raises(abi.CckaError, match="missing"):
        h.patch("NodePool", "legacy", "json", h.policy_patch(abi.PROFILE_OFFPEAK, "legacy", True))
    h.patch("NodePool", "legacy", "json", h.policy_patch(abi.PROFILE_PEAK, "legacy", True, fallback=True))
    got = json.loads(h.get_json("NodePool", "legacy"))
    assert got["spec"]["template"]["requirements"][1]["values"] == ["on-demand"]
    with pytest.raises(abi.CckaError, match="NotFound"):
        h.patch("NodePool", "nope", "merge", "{}")


def test_yaml_subset_parser_shapes():
    h = Host()
    h.apply("""
# comment
apiVersion: autoscaling/v2
kind: HorizontalPodAutoscaler
metadata: {name: web-hpa, namespace: "ns"}
spec:
  scaleTargetRef: {apiVersion: apps/v1, kind: Deployment, name: web}
  minReplicas: 2
  maxReplicas: 40
  metrics:
  - type: Resource
    resource:
      name: cpu
      target:
        type: Utilization
        averageUtilization: 65
  behavior:
    scaleDown:
      stabilizationWindowSeconds: 120
      selectPolicy: Min
      policies:
        - {type: Pods, value: 2, periodSeconds: 60}
        - type: Percent
          value: 50
          periodSeconds: 60
---
apiVersion: apps/v1
kind: Deployment
metadata:
  name: web
spec:
  replicas: 3
  template:
    metadata:
      labels: {app: web}
    spec:
      nodeSelector:
        karpenter.sh/capacity-type: spot
      containers:
      - name: c
        resources:
          requests: {cpu: "0.25", memory: 1Gi}
          limits:
            cpu: 1
""")
    h.apply(h.manifest(-1))
    w = h.build_world("small", 60, 8)
    d = w.deploy[0]
    assert (d.scaler, d.min_replicas, d.max_replicas, d.target_util_pct) == (abi.SCALER_HPA, 2, 40, 65)
    assert (d.req_cpu_m, d.req_mem_mi, d.limit_cpu_m, d.cap_sel) == (250, 1024, 1000, abi.CAP_SPOT)
    assert d.down.select == abi.SELECT_MIN and d.down.stab_window_s == 120 and d.down.n_policies == 2
    assert (d.down.policies[0].type, d.down.policies[0].value, d.down.policies[1].type) == \
           (abi.HPA_PODS, 2, abi.HPA_PERCENT)
    assert d.up.n_policies == 2 and d.up.stab_window_s == 0  # autoscaling/v2 defaults


def test_keda_scaledobject_ingest():
    h = Host()
    h.apply(h.manifest(-1))
    h.apply("""apiVersion: apps/v1
kind: Deployment
metadata: {name: worker}
spec:
  replicas: 0
  template:
    spec:
      containers:
      - name: w
        resources: {requests: {cpu: 100m, memory: 64Mi}}
---
apiVersion: keda.sh/v1alpha1
kind: ScaledObject
metadata: {name: worker-so}
spec:
  scaleTargetRef: {name: worker}
  minReplicaCount: 0
  maxReplicaCount: 30
  cooldownPeriod: 120
  triggers:
  - type: aws-sqs-queue
    metadata:
      queueLength: "50"
      activationQueueLength: "5"
""")
    w = h.build_world("tiny", 60, 8)
    d = w.deploy[0]
    assert (d.scaler, d.keda_min, d.keda_max, d.keda_cooldown_s) == (abi.SCALER_KEDA, 0, 30, 120)
    assert (d.keda_threshold, d.keda_activation, d.cap_sel) == (50, 5, 3)


def test_keda_multi_trigger_ingest():
    """triggers[1..] of a ScaledObject become KEDA_TRIGGER entries right after
    their deployment; the deployments after it shift by the trigger count."""
    h = Host()
    h.apply(h.manifest(-1))
    h.apply("""apiVersion: apps/v1
kind: Deployment
metadata: {name: worker}
spec:
  replicas: 0
  template:
    spec:
      nodeSelector: {karpenter.sh/capacity-type: spot}
      containers:
      - name: w
        resources: {requests: {cpu: 100m, memory: 64Mi}}
---
apiVersion: apps/v1
kind: Deployment
metadata: {name: web}
spec:
  replicas: 2
  template:
    spec:
      containers:
      - name: w
        resources: {requests: {cpu: 200m, memory: 128Mi}}
---
apiVersion: keda.sh/v1alpha1
kind: ScaledObject
metadata: {name: worker-so}
spec:
  scaleTargetRef: {name: worker}
  triggers:
  - type: aws-sqs-queue
    metadata: {queueLength: "50", activationQueueLength: "5"}
  - type: prometheus
    metadata: {threshold: "200", activationThreshold: "20"}
  - type: cpu
    metadata: {value: "60"}
""")
    w = h.build_world("tiny", 60, 8)
    assert w.n_deploy == 4
    d0, t1, t2, d3 = (w.deploy[i] for i in range(4))
    assert d0.scaler == abi.SCALER_KEDA and (d0.keda_threshold, d0.keda_activation) == (50, 5)
    assert t1.scaler == abi.SCALER_KEDA_TRIGGER and (t1.keda_threshold, t1.keda_activation) == (200, 20)
    assert t2.scaler == abi.SCALER_KEDA_TRIGGER and (t2.keda_threshold, t2.keda_activation) == (60, 0)
    assert (t1.replicas0, t1.pdb_member, t1.cap_sel) == (0, 0, abi.CAP_SPOT)
    assert d3.scaler == abi.SCALER_STATIC and d3.replicas0 == 2
