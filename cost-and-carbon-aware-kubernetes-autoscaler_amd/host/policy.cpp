// policy.cpp — see policy.h. Output bytes are pinned against the payloads the
// reference scripts emit (tests/test_golden_capture.py).
#include "policy.h"

#include <cstdlib>
#include <sstream>

namespace ccka::host {

static std::string env_or(const char* name, const std::string& dflt) {
  const char* v = std::getenv(name);
  return (v && *v) ? std::string(v) : dflt;  // ${VAR:-default}: empty -> default
}

PolicyEnv PolicyEnv::from_environment() {
  PolicyEnv e;
  e.np_spot = env_or("NP_SPOT", e.np_spot);
  e.np_od = env_or("NP_OD", e.np_od);
  e.offpeak_zones = env_or("OFFPEAK_ZONES", e.offpeak_zones);
  e.peak_zones = env_or("PEAK_ZONES", e.peak_zones);
  e.ns = env_or("NAMESPACE", e.ns);
  e.count = std::atoi(env_or("COUNT", std::to_string(e.count)).c_str());
  e.replicas = std::atoi(env_or("REPLICAS", std::to_string(e.replicas)).c_str());
  return e;
}

std::vector<std::string> zones_from_env(const std::string& value) {
  std::string s = value;
  for (auto& c : s)
    if (c == ',') c = ' ';  // ${OFFPEAK_ZONES//,/ }
  std::vector<std::string> out;
  std::istringstream is(s);
  std::string z;
  while (is >> z) out.push_back(z);
  return out;
}

std::string json_array(const std::vector<std::string>& items) {
  std::string o = "[";
  bool first = true;
  for (auto& it : items) {
    if (it.empty()) continue;
    if (!first) o += ',';
    o += '"' + it + '"';
    first = false;
  }
  return o + "]";
}

std::string requirements_patch(Profile p, const PolicyEnv& env, const std::string& pool,
                               bool fallback_path) {
  const std::string& zones = p == Profile::Peak ? env.peak_zones : env.offpeak_zones;
  const char* op = p == Profile::Peak ? "add" : "replace";
  const std::string prefix = fallback_path ? "/spec/template" : "/spec/template/spec";
  std::string o = std::string("[{\"op\":\"") + op + "\",\"path\":\"" + prefix + "/requirements\",\"value\":[";
  o += "{\"key\":\"topology.kubernetes.io/zone\",\"operator\":\"In\",\"values\":" + json_array(zones_from_env(zones)) + "}";
  o += ',';
  if (pool == env.np_spot)
    o += "{\"key\":\"karpenter.sh/capacity-type\",\"operator\":\"In\",\"values\":[\"spot\",\"on-demand\"]}";
  else
    o += "{\"key\":\"karpenter.sh/capacity-type\",\"operator\":\"In\",\"values\":[\"on-demand\"]}";
  o += "]}]\n";
  return o;
}

std::string disruption_merge_patch(Profile p, const PolicyEnv& env, const std::string& pool) {
  switch (p) {
    case Profile::Reset:  // demo_19 hard-codes the pool names and this exact text
      return "{\n      \"spec\": {\n        \"disruption\": {\n          \"consolidationPolicy\": \"WhenEmpty\",\n"
             "          \"consolidateAfter\": \"30s\"\n        }\n      }\n    }";
    case Profile::OffPeak:
      if (pool == env.np_spot)
        return "{\"spec\":{\"disruption\":{\"consolidationPolicy\":\"WhenEmptyOrUnderutilized\"}}}";
      return "{\"spec\":{\"disruption\":{\"consolidationPolicy\":\"WhenEmpty\",\"consolidateAfter\":\"60s\"}}}";
    case Profile::Peak:
      return "{\"spec\":{\"disruption\":{\"consolidationPolicy\":\"WhenEmpty\",\"consolidateAfter\":\"120s\"}}}";
  }
  return "";
}

std::string burst_deployment_yaml(const PolicyEnv& env, int i) {
  const bool odd = i % 2 == 1;
  const std::string cap = odd ? "spot" : "on-demand";
  const std::string tol = odd ? "      tolerations: []\n"
                              : "      tolerations:\n        - key: \"critical\"\n          operator: \"Equal\"\n"
                                "          value: \"true\"\n          effect: \"NoSchedule\"\n";
  const std::string name = "burst-web-" + std::to_string(i);
  const std::string idx = std::to_string(i);
  std::string y;
  y += "apiVersion: apps/v1\nkind: Deployment\nmetadata:\n  name: " + name + "\n  namespace: " + env.ns + "\n";
  y += "  labels:\n    app: burst-web\n    group: scale-burst\n    idx: \"" + idx + "\"\n    capacity: \"" + cap + "\"\n";
  y += "spec:\n  replicas: " + std::to_string(env.replicas) + "\n  selector:\n    matchLabels:\n";
  y += "      app: burst-web\n      group: scale-burst\n      idx: \"" + idx + "\"\n";
  y += "  template:\n    metadata:\n      labels:\n        app: burst-web\n        group: scale-burst\n";
  y += "        idx: \"" + idx + "\"\n        capacity: \"" + cap + "\"\n";
  y += "    spec:\n      nodeSelector:\n        karpenter.sh/capacity-type: \"" + cap + "\"\n";
  y += tol;
  y += "      securityContext:\n        seccompProfile:\n          type: RuntimeDefault\n";
  y += "      containers:\n      - name: web\n        image: ghcr.io/nginxinc/nginx-unprivileged:stable-alpine\n";
  y += "        imagePullPolicy: IfNotPresent\n        ports:\n          - containerPort: 8080\n";
  y += "        readinessProbe:\n          httpGet:\n            path: /\n            port: 8080\n";
  y += "          initialDelaySeconds: 2\n          periodSeconds: 5\n";
  y += "        livenessProbe:\n          httpGet:\n            path: /\n            port: 8080\n";
  y += "          initialDelaySeconds: 10\n          periodSeconds: 10\n";
  y += "        securityContext:\n          runAsNonRoot: true\n          allowPrivilegeEscalation: false\n";
  y += "          capabilities:\n            drop:\n              - \"ALL\"\n";
  y += "        resources:\n          requests:\n            cpu: \"200m\"\n            memory: \"128Mi\"\n";
  y += "          limits:\n            cpu: \"500m\"\n            memory: \"256Mi\"\n";
  return y;
}

std::string pdb_yaml(const PolicyEnv& env) {
  return "# PDB to keep 50% of burst pods available during consolidations/rotations\n"
         "apiVersion: policy/v1\nkind: PodDisruptionBudget\nmetadata:\n  name: burst-pdb\n  namespace: " +
         env.ns + "\nspec:\n  minAvailable: \"50%\"\n  selector:\n    matchLabels:\n      group: scale-burst\n";
}

}  // namespace ccka::host
