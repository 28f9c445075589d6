// admission.h — Kyverno guard policies as a placement pre-filter
// (SURVEY.md §8(f)-4).
//
// The reference installs two enforce-mode ClusterPolicies (04_kyverno.sh:24-75)
// and then disables the stage (README.md:42). They are evaluated here the way
// Kyverno's admission webhook would, with its default auto-gen rules for pod
// controllers: a Pod, or the pod template of a Deployment / ReplicaSet /
// StatefulSet / DaemonSet / Job (spec.template) or CronJob
// (spec.jobTemplate.spec.template), is checked at apply time. A denied object
// is not stored, so it never reaches the world the engine rolls out.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "value.h"

namespace ccka::host {

// policy bits (CCKA_ADMIT_* in ccka_host.h)
constexpr uint32_t kAdmitRequireRequestsLimits = 1u;  // 04_kyverno.sh:24-42
constexpr uint32_t kAdmitCriticalNoSpot = 2u;         // 04_kyverno.sh:44-72

struct Violation {
  std::string policy, rule, message, path;
};

// All violations of `obj` under the enabled policies (empty: admitted).
std::vector<Violation> admission_review(const Value& obj, uint32_t policies);

// kubectl-style denial text for one object
std::string denial_message(const Value& obj, const std::vector<Violation>& v);

}  // namespace ccka::host
