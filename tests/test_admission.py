"""Kyverno guard policies as the admission pre-filter:
04_kyverno.sh:24-42 require-requests-limits and :44-72
critical-no-spot-without-pdb, enforce mode, Kyverno auto-gen for pod
controllers. The reference never runs them (README.md:42), so the expected
outcomes are derived from the policy text: parity unpinned beyond that."""
import pytest

from ccka import abi
from ccka.host import ADMIT_ALL, ADMIT_CRITICAL_NO_SPOT, ADMIT_REQUIRE_REQUESTS_LIMITS, Host


def dep(name, labels="", tolerations="", resources=None, ns="nov-22", kind="Deployment"):
    res = resources if resources is not None else (
        "        resources:\n          requests: {cpu: 200m, memory: 128Mi}\n"
        "          limits: {cpu: 500m, memory: 256Mi}\n")
    pod = (f"    metadata:\n      labels:\n        app: {name}\n{labels}"
           f"    spec:\n{tolerations}      containers:\n      - name: web\n        image: x\n{res}")
    return (f"apiVersion: apps/v1\nkind: {kind}\nmetadata:\n  name: {name}\n  namespace: {ns}\n"
            f"spec:\n  replicas: 2\n  template:\n{pod}")


SPOT_TOL = ("      tolerations:\n      - key: karpenter.sh/capacity-type\n        operator: Equal\n"
            "        value: spot\n        effect: NoSchedule\n")
CRIT = "        critical: \"true\"\n"


def test_reference_burst_manifests_are_admitted():
    h = Host()
    docs = [h.manifest(-1), h.manifest(0)] + [h.manifest(i) for i in range(1, 13)]
    for d in docs:
        assert h.admission_review(d) == []
    h.set_admission(ADMIT_ALL)
    for d in docs:
        h.apply(d)
    w = h.build_world("tiny", 60, 8)
    assert w.n_deploy == 12


def test_require_requests_limits():
    h = Host()
    no_lim = dep("a", resources="        resources:\n          requests: {cpu: 200m, memory: 128Mi}\n")
    v = h.admission_review(no_lim)
    assert len(v) == 1 and v[0]["policy"] == "require-requests-limits"
    assert v[0]["rule"] == "autogen-containers-require-limits"
    assert v[0]["path"] == "/spec/template/spec/containers/0/resources/limits/cpu/"
    assert v[0]["message"] == "All containers must have cpu/memory requests & limits"
    assert h.admission_review(dep("b", resources="")) != []
    empty_mem = dep("c", resources="        resources:\n          requests: {cpu: 200m, memory: \"\"}\n"
                                   "          limits: {cpu: 1, memory: 1Gi}\n")
    assert h.admission_review(empty_mem)[0]["path"].endswith("/requests/memory/")
    assert h.admission_review(dep("d")) == []
    # policy bit off: no check
    assert h.admission_review(no_lim, ADMIT_CRITICAL_NO_SPOT) == []


def test_critical_no_spot():
    h = Host()
    bad = dep("a", labels=CRIT, tolerations=SPOT_TOL)
    v = h.admission_review(bad)
    assert [x["policy"] for x in v] == ["critical-no-spot-without-pdb"]
    assert v[0]["rule"] == "autogen-deny-spot-for-critical"
    assert v[0]["message"] == "Critical pods must avoid Spot capacity."
    assert h.admission_review(dep("b", tolerations=SPOT_TOL)) == []          # not critical
    assert h.admission_review(dep("c", labels=CRIT)) == []                   # no spot toleration
    assert h.admission_review(dep("d", labels=CRIT, tolerations=SPOT_TOL, ns="kube-system")) == []
    od_tol = SPOT_TOL.replace("value: spot", "value: on-demand")
    assert h.admission_review(dep("e", labels=CRIT, tolerations=od_tol)) == []
    assert h.admission_review(bad, ADMIT_REQUIRE_REQUESTS_LIMITS) == []
    # both policies at once
    both = dep("f", labels=CRIT, tolerations=SPOT_TOL, resources="")
    assert {x["policy"] for x in h.admission_review(both)} == {"require-requests-limits",
                                                                "critical-no-spot-without-pdb"}


def test_pod_and_cronjob_kinds():
    h = Host()
    pod = ("apiVersion: v1\nkind: Pod\nmetadata:\n  name: p\n  labels: {critical: \"true\"}\nspec:\n"
           "  tolerations: [{key: karpenter.sh/capacity-type, operator: Equal, value: spot}]\n"
           "  containers:\n  - name: c\n    image: x\n")
    v = h.admission_review(pod)
    assert {x["rule"] for x in v} == {"containers-require-limits", "deny-spot-for-critical"}
    assert v[0]["path"].startswith("/spec/containers/0/")
    cj = ("apiVersion: batch/v1\nkind: CronJob\nmetadata: {name: cj}\nspec:\n  jobTemplate:\n    spec:\n"
          "      template:\n        spec:\n          containers:\n          - name: c\n            image: x\n")
    v = h.admission_review(cj)
    assert v[0]["rule"] == "autogen-cronjob-containers-require-limits"
    assert v[0]["path"] == "/spec/jobTemplate/spec/template/spec/containers/0/resources/requests/cpu/"
    # objects without a pod template are never matched
    assert h.admission_review(h.manifest(0)) == [] and h.admission_review(h.manifest(-1)) == []


def test_enforced_apply_filters_placement():
    """A denied Deployment is not stored (kubectl applies each document on its
    own): the world has one deployment fewer and apply reports the denial."""
    h = Host()
    h.set_admission(ADMIT_ALL)
    h.apply(h.manifest(-1))
    ok = dep("good")
    bad = dep("bad", labels=CRIT, tolerations=SPOT_TOL)
    with pytest.raises(abi.CckaError) as e:
        h.apply(ok + "---\n" + bad)
    msg = str(e.value)
    assert "validate.kyverno.svc-fail" in msg and "Deployment/nov-22/bad" in msg
    assert "critical-no-spot-without-pdb" in msg
    assert '"name":"good"' in h.get_json("Deployment", "good").replace(" ", "")
    with pytest.raises(abi.CckaError):
        h.get_json("Deployment", "bad")
    assert h.build_world("tiny", 60, 8).n_deploy == 1
    # admission off: the same document is stored
    h.set_admission(0)
    h.apply(bad)
    assert h.build_world("tiny", 60, 8).n_deploy == 2
    with pytest.raises(abi.CckaError):
        h.set_admission(8)
