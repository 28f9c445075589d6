// admission.cpp — the two Kyverno ClusterPolicies of 04_kyverno.sh:24-75.
#include "admission.h"

namespace ccka::host {

namespace {

// Kyverno auto-gen: where the pod spec / labels live for each controller kind
// (rule names gain the "autogen-" / "autogen-cronjob-" prefix)
struct PodView {
  const Value* spec = nullptr;    // PodSpec
  const Value* labels = nullptr;  // pod labels
  std::string prefix;             // JSON-pointer prefix of the PodSpec
  std::string rule_prefix;
};

bool pod_view(const Value& obj, PodView* pv) {
  const std::string kind = obj.get("kind") ? obj.get("kind")->as_string() : "";
  if (kind == "Pod") {
    pv->spec = obj.get("spec");
    pv->labels = obj.at({"metadata", "labels"});
    pv->prefix = "/spec";
    return true;
  }
  if (kind == "Deployment" || kind == "ReplicaSet" || kind == "StatefulSet" || kind == "DaemonSet" ||
      kind == "Job") {
    pv->spec = obj.at({"spec", "template", "spec"});
    pv->labels = obj.at({"spec", "template", "metadata", "labels"});
    pv->prefix = "/spec/template/spec";
    pv->rule_prefix = "autogen-";
    return true;
  }
  if (kind == "CronJob") {
    pv->spec = obj.at({"spec", "jobTemplate", "spec", "template", "spec"});
    pv->labels = obj.at({"spec", "jobTemplate", "spec", "template", "metadata", "labels"});
    pv->prefix = "/spec/jobTemplate/spec/template/spec";
    pv->rule_prefix = "autogen-cronjob-";
    return true;
  }
  return false;
}

// Kyverno pattern "?*": the field is present and its value has >= 1 character
bool nonempty(const Value* v) { return v && v->is_scalar() && !v->text.empty(); }

}  // namespace

std::vector<Violation> admission_review(const Value& obj, uint32_t policies) {
  std::vector<Violation> out;
  PodView pv;
  if (!policies || !pod_view(obj, &pv)) return out;
  const Value* spec = pv.spec;

  // require-requests-limits / containers-require-limits (04_kyverno.sh:24-42):
  // every container carries requests.{cpu,memory} and limits.{cpu,memory}
  if (policies & kAdmitRequireRequestsLimits) {
    const Value* cs = spec ? spec->get("containers") : nullptr;
    bool ok = cs && cs->is_seq() && !cs->seq.empty();
    std::string path = pv.prefix + "/containers/";
    for (size_t i = 0; ok && i < cs->seq.size(); ++i) {
      const Value& c = cs->seq[i];
      const std::string base = pv.prefix + "/containers/" + std::to_string(i) + "/resources/";
      for (const char* sec : {"requests", "limits"}) {
        const Value* r = c.at({"resources", sec});
        for (const char* res : {"cpu", "memory"}) {
          if (ok && !nonempty(r ? r->get(res) : nullptr)) {
            ok = false;
            path = base + sec + "/" + res + "/";
          }
        }
      }
    }
    if (!ok)
      out.push_back({"require-requests-limits", pv.rule_prefix + "containers-require-limits",
                     "All containers must have cpu/memory requests & limits", path});
  }

  // critical-no-spot-without-pdb / deny-spot-for-critical (04_kyverno.sh:44-72):
  // pods labelled critical=true, outside karpenter/kyverno/kube-system, may not
  // tolerate karpenter.sh/capacity-type=spot
  if (policies & kAdmitCriticalNoSpot) {
    const Value* crit = pv.labels ? pv.labels->get("critical") : nullptr;
    const Value* nsv = obj.at({"metadata", "namespace"});
    const std::string ns = nsv ? nsv->as_string() : "default";
    const bool excluded = ns == "karpenter" || ns == "kyverno" || ns == "kube-system";
    if (crit && crit->as_string() == "true" && !excluded) {
      int64_t n = 0;
      const Value* tol = spec ? spec->get("tolerations") : nullptr;
      if (tol && tol->is_seq())
        for (const Value& t : tol->seq) {
          const Value* k = t.get("key");
          const Value* v = t.get("value");
          if (k && v && k->as_string() == "karpenter.sh/capacity-type" && v->as_string() == "spot") ++n;
        }
      if (n > 0)
        out.push_back({"critical-no-spot-without-pdb", pv.rule_prefix + "deny-spot-for-critical",
                       "Critical pods must avoid Spot capacity.", pv.prefix + "/tolerations/"});
    }
  }
  return out;
}

std::string denial_message(const Value& obj, const std::vector<Violation>& v) {
  const Value* k = obj.get("kind");
  const Value* n = obj.at({"metadata", "name"});
  const Value* ns = obj.at({"metadata", "namespace"});
  std::string s = "admission webhook \"validate.kyverno.svc-fail\" denied the request: resource " +
                  (k ? k->as_string() : std::string("?")) + "/" + (ns ? ns->as_string() : std::string("default")) +
                  "/" + (n ? n->as_string() : std::string("?")) + " was blocked due to the following policies";
  for (const Violation& x : v)
    s += "; " + x.policy + ": " + x.rule + ": 'validation error: " + x.message + " rule " + x.rule +
         " failed at path " + x.path + "'";
  return s;
}

}  // namespace ccka::host
