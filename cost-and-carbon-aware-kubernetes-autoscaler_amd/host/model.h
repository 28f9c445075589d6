// model.h — Kubernetes objects in, ccka_world out.
//
// ManifestStore emulates the two kubectl verbs the reference's decision path
// uses: `kubectl apply -f` (demo_30_burst_configure.sh:143,
// demo_10_setup_configure.sh) and `kubectl patch nodepool --type=merge|json`
// (demo_20_offpeak_configure.sh:59-60,96; demo_21_peak_configure.sh:56-57,88;
// demo_19_reset_policies.sh:68-75). build_world() turns the stored NodePools,
// Deployments, HPAs (autoscaling/v2), ScaledObjects (keda.sh/v1alpha1) and
// PodDisruptionBudgets into the engine's ccka_world.
#pragma once

#include <string>
#include <vector>

#include "../../include/ccka.h"
#include "policy.h"
#include "value.h"

namespace ccka::host {

class ManifestStore {
 public:
  // kubectl apply -f: upsert every document by (kind, metadata.name).
  // `admission` (kAdmit* bits, admission.h): documents the enabled Kyverno
  // policies deny are not stored; the others are, and then ParseError carries
  // the denials (kubectl applies each document independently)
  void apply(const std::string& yaml_text, uint32_t admission = 0);
  // kubectl patch <kind> <name> --type=merge|json; throws ParseError
  void patch(const std::string& kind, const std::string& name, const std::string& type,
             const std::string& patch_text);
  // kubectl label <kind> <name> k=v... [--overwrite] (demo_10_setup_configure.sh:61-62):
  // whitespace-separated "k=v" set, "k-" removes; an existing different value
  // without overwrite fails like kubectl; throws ParseError
  void label(const std::string& kind, const std::string& name, const std::string& labels, bool overwrite);
  const Value* get(const std::string& kind, const std::string& name) const;
  std::vector<const Value*> all(const std::string& kind) const;

 private:
  std::vector<Value> objs_;
  Value* find(const std::string& kind, const std::string& name);
};

// Catalog + tiles the world points into (owned here; ccka_world holds pointers)
struct Tables {
  std::vector<std::string> names;
  std::vector<ccka_itype> types;
  std::vector<double> ci_gpwh, ci_gpwmin;  // [R][24]
  std::vector<int32_t> price;               // [R][24][K][Z][2]
  int regions = 1, zones = 3;
  int index(const std::string& n) const;
};

// builtin catalogs (same numbers as ccka/world.py): "tiny" (12 types), "small" (16)
Tables builtin_tables(const std::string& which, double ci_g_per_kwh = 400.0, uint64_t seed = 20251205);

struct WorldMeta {
  std::vector<std::string> pool_names;    // Karpenter order
  std::vector<std::string> deploy_names;  // engine deployment index order
  // NodePool labels the reference sets for grouping in OpenCost / dashboards
  // (demo_10_setup_configure.sh:61-62), "" when absent
  std::vector<std::string> pool_carbon;    // carbon.simulated
  std::vector<std::string> pool_strategy;  // autoscale.strategy
  std::vector<std::string> deploy_capacity;  // Deployment label `capacity` (demo_30 :88)
  std::string zone_prefix = "us-east-2";     // zone bit z = zone_prefix + 'a' + z
};

// The reference's base NodePools (it never creates them, demo_00_env.sh:17):
// our synthesized pair, Karpenter v1 defaults, all zones.
std::string default_nodepools_yaml(const PolicyEnv& env);

// Build the world from the store. Profiles RESET/OFFPEAK/PEAK are the patches
// the reference scripts would send (policy.h) for the pools they name.
WorldMeta build_world(const ManifestStore& store, const PolicyEnv& env, const Tables& tables,
                      int n_steps, int max_nodes, ccka_world* out);

// zone name -> bit (us-east-2a -> 1, ...b -> 2, ...)
uint32_t zone_bit(const std::string& zone);

}  // namespace ccka::host
