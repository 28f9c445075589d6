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
