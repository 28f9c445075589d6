// policy.h — the reference's policy/demand scripts as library functions.
//
// Each function reproduces, byte for byte, the payload the corresponding
// reference script hands to kubectl (pinned by tests/golden/reference_capture):
//   zones_from_env / json_array   demo_20_offpeak_configure.sh:9-54 (demo_21 :9-46)
//   requirements_patch            write_req_patch, demo_20_offpeak_configure.sh:64-81
//                                 (op replace) and demo_21_peak_configure.sh:60-77 (op add)
//   disruption_merge_patch        demo_20 :59-60, demo_21 :56-57, demo_19_reset_policies.sh:68-75
//   burst_deployment_yaml         demo_30_burst_configure.sh:57-141
//   pdb_yaml                      demo_10_setup_configure.sh:47-56
#pragma once

#include <string>
#include <vector>

namespace ccka::host {

enum class Profile { Reset = 0, OffPeak = 1, Peak = 2 };

struct PolicyEnv {
  std::string np_spot = "spot-preferred";  // NP_SPOT, demo_00_env.sh:18
  std::string np_od = "on-demand-slo";     // NP_OD, demo_00_env.sh:19
  std::string offpeak_zones = "us-east-2a";  // OFFPEAK_ZONES, demo_00_env.sh:22
  std::string peak_zones = "us-east-2c";     // PEAK_ZONES, demo_00_env.sh:23
  std::string ns = "nov-22";               // NAMESPACE, demo_00_env.sh:9
  int count = 12;                          // COUNT, demo_30_burst_configure.sh:7
  int replicas = 5;                        // REPLICAS, demo_30_burst_configure.sh:8
  // read the same environment variables with the scripts' ${VAR:-default} rules
  static PolicyEnv from_environment();
};

// "a,b" or "a b" -> {"a","b"}; bash word splitting (IFS whitespace)
std::vector<std::string> zones_from_env(const std::string& value);
std::string json_array(const std::vector<std::string>& items);
// JSON Patch file content (with the trailing newline printf writes)
std::string requirements_patch(Profile p, const PolicyEnv& env, const std::string& pool,
                               bool fallback_path = false);
// merge patch text exactly as passed to `kubectl patch --type=merge -p`
std::string disruption_merge_patch(Profile p, const PolicyEnv& env, const std::string& pool);
std::string burst_deployment_yaml(const PolicyEnv& env, int index);
std::string pdb_yaml(const PolicyEnv& env);

}  // namespace ccka::host
